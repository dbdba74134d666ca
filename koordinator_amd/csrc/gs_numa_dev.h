// gs_numa_dev.h — NodeNUMAResource Filter + Score of one (pod, node) pair on the device (gfx950).
//
// Restates pkg/scheduler/plugins/nodenumaresource/{plugin.go Filter/filterAmplifiedCPUs, scoring.go Score,
// resource_manager.go GetTopologyHints/Allocate, topology_hint.go} and frameworkext/topologymanager/policy*.go
// over the count summaries the host keeps in HBM (gs_layout.h C_NFLAGS.. C_ZADJ0):
//  * cpuset feasibility of allocateCPUSet is a count test: with the required-policy prefilter applied every
//    available CPU lies in a full core (FullPCPUs) or on a distinct core (SpreadByPCPUs), and takeCPUs takes
//    prefixes of core-ordered lists, so the result satisfies the policy iff per-zone counts are multiples of
//    CPUsPerCore (FullPCPUs with a NUMA split) — which CPUs are picked is a host-side Reserve concern;
//  * NUMA hints are enumerated over zone-slot masks (zones sorted by node id, so slot masks order and
//    intersect exactly like node-id masks) in bitmask.IterateBitMasks order; the hint lists of the single
//    provider are merged in sorted resource-name order (cpu before memory; the reference iterates a Go map,
//    policy.go:108 — see DESIGN.md) with mergeFilteredHints' exact update rule.
#pragma once

#include "../../include/gpuscore.h"
#include "gs_layout.h"

namespace gs {

enum : int { BIND_UNSET = 0, BIND_DEFAULT = 1, BIND_FULL = 2, BIND_SPREAD = 3 };

struct NumaRow {           // per-node NodeNUMAResource state (HBM columns, or the commit's LDS copy)
  int64_t zcap_cpu[4], zcap_mem[4];
  int64_t zraw_cpu[4], zraw_mem[4];
  double amp, namp;
  uint32_t nflags, nflags2;
  int32_t alloc_cpus;
  uint32_t tfree;
  uint32_t zfree[4];
  int32_t zadj[4];
};

struct NumaOut {
  uint32_t reason;         // gs_numa_reason (0 = feasible)
  int32_t score;
  uint32_t flags;          // GS_PLACED_NUMA / GS_PLACED_CPUSET / affinity bits, for Reserve
  uint32_t zkeys;          // allocation by hint: bit z cpu, bit 4+z memory
  int64_t zcpu[4], zmem[4];
  uint32_t aff;            // the Filter-time affinity: 0x10 | zone-slot mask, 0 = none (NUMA-policy nodes)
  uint32_t pad;
};

__device__ __forceinline__ void load_numa_row(const MirrorView& m, uint32_t i, NumaRow& r) {
#pragma unroll
  for (int z = 0; z < 4; ++z) {
    r.zcap_cpu[z] = m.c64(C_ZCAP_CPU0 + z)[i];
    r.zcap_mem[z] = m.c64(C_ZCAP_MEM0 + z)[i];
    r.zraw_cpu[z] = m.c64(C_ZRAW_CPU0 + z)[i];
    r.zraw_mem[z] = m.c64(C_ZRAW_MEM0 + z)[i];
    r.zfree[z] = (uint32_t)m.c32(C_ZFREE0 + z)[i];
    r.zadj[z] = m.c32(C_ZADJ0 + z)[i];
  }
  r.amp = __longlong_as_double(m.c64(C_AMP)[i]);
  r.namp = __longlong_as_double(m.c64(C_NAMP)[i]);
  r.nflags = (uint32_t)m.c32(C_NFLAGS)[i];
  r.nflags2 = (uint32_t)m.c32(C_NFLAGS2)[i];
  r.alloc_cpus = m.c32(C_ALLOC_CPUS)[i];
  r.tfree = (uint32_t)m.c32(C_TFREE)[i];
}

// extension.Amplify (apis/extension/node_resource_amplification.go:170-175): IEEE binary64 like Go
__device__ __forceinline__ int64_t amplify_d(int64_t x, double r) {
  if (r <= 1.0) return x;
  return (int64_t)ceil(__dmul_rn((double)x, r));
}

// available-CPU counts packed by the host: raw | full-core CPUs << 9 | cores with a free CPU << 18
__device__ __forceinline__ int cnt_raw(uint32_t v) { return (int)(v & 511u); }
__device__ __forceinline__ int cnt_sel(uint32_t v, int bind, bool required) {
  if (!required) return (int)(v & 511u);
  if (bind == BIND_FULL) return (int)((v >> 9) & 511u);
  if (bind == BIND_SPREAD) return (int)((v >> 18) & 511u);
  return (int)(v & 511u);
}

// exact floor(x*100/cap), 0 <= x <= cap < 2^53 (same scheme as pct_floor in gs_kernels.hip)
__device__ __forceinline__ int32_t numa_pct(int64_t x, int64_t cap) {
  int64_t num = x * 100;
  float qf = ((float)(uint32_t)((uint64_t)num >> 32) * 4294967296.0f + (float)(uint32_t)(uint64_t)num) *
             __builtin_amdgcn_rcpf((float)(uint32_t)((uint64_t)cap >> 32) * 4294967296.0f + (float)(uint32_t)(uint64_t)cap);
  int32_t q = (int32_t)qf;
  q = q > 100 ? 100 : q;
  int64_t prod = (int64_t)q * cap;
  if (prod > num) --q;
  else if (prod + cap <= num) ++q;
  return q;
}
// leastRequestedScore / mostRequestedScore (least_allocated.go:49-58, most_allocated.go:45-55)
__device__ __forceinline__ int32_t lr_score(int64_t req, int64_t cap) {
  if (cap == 0 || req > cap) return 0;
  return numa_pct(cap - req, cap);
}
__device__ __forceinline__ int32_t mr_score(int64_t req, int64_t cap) {
  if (cap == 0) return 0;
  if (req > cap) req = cap;
  return numa_pct(req, cap);
}
// either scorer with one division site (numa_eval inlines its scorers several times)
__device__ __forceinline__ int32_t req_score(bool most, int64_t req, int64_t cap) {
  if (cap == 0 || (!most && req > cap)) return 0;
  return numa_pct(most ? (req > cap ? cap : req) : cap - req, cap);
}
__device__ __forceinline__ int32_t sdiv(int32_t a, int32_t b) {
  int32_t q = (int32_t)((float)a * __builtin_amdgcn_rcpf((float)b));
  if (q * b > a) --q;
  else if ((q + 1) * b <= a) ++q;
  return q;
}

// IterateBitMasks order over zone slots (bitmask.go:206-222) for 1..4 zones, 4 bits per position:
//   1 zone: 1 | 2 zones: 1 2 3 | 3 zones: 1 2 4 3 5 6 7 | 4 zones: 1 2 4 8 3 5 9 6 10 12 7 11 13 14 15
__constant__ uint64_t kMaskOrderPacked[4] = {0x1ull, 0x321ull, 0x7653421ull, 0xFEDB7CA69538421ull};

__device__ __forceinline__ bool narrower(uint32_t a, uint32_t b) {   // bitmask.IsNarrowerThan
  int ca = __popc(a), cb = __popc(b);
  return ca == cb ? a < b : ca < cb;
}

// One (pod, node) evaluation. do_filter: run Filter (incl. the topology manager Admit that sets the affinity);
// do_score: Score with that affinity (none when the filter is off, as in the reference without a Filter call);
// want_alloc: fill the Reserve allocation.
// `alloc[s]`/`free[s]` give NodeInfo.Allocatable / Allocatable-Requested for slots 0..2 and the scalars.
// POLICY_NODES = false compiles only the path of nodes without a NUMA topology policy (the caller routes
// policy nodes to a kernel of their own); such a call on a policy node returns with reason 0 and no score.
// known_aff >= 0: the affinity this pair's Filter produced on the same row state (NumaOut.aff; Reserve of a
// row untouched since the batch-start evaluation): hint generation and merge are skipped.
template <bool POLICY_NODES = true, class Slots>
__device__ __forceinline__ NumaOut numa_eval(const NumaRow& r, const PodVec& p, const Profile& pf, const Slots& sl,
                                             bool do_filter, bool do_score, int known_aff = -1,
                                             uint64_t* prof = nullptr) {
  // prof (diagnostics): s_memtime cycles per segment accumulated into prof[0..5]
  uint64_t t_np = prof ? __builtin_amdgcn_s_memtime() : 0;
#define NP(i)                                          \
  do {                                                 \
    if (prof) {                                        \
      const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
      prof[i] += t_ - t_np;                            \
      t_np = t_;                                       \
    }                                                  \
  } while (0)
  NumaOut o{};
  const uint32_t pn = p.numa;
  if (pn & PN_PREFAIL) { o.reason = GS_NUMA_INVALID_REQUESTED_CPUS; return o; }
  if (pn & PN_SKIP) return o;
  const uint32_t nf = r.nflags;
  const int policy = (nf >> NF_POLICY_SHIFT) & 3, nbind = (nf >> NF_BIND_SHIFT) & 3;
  const bool has_cpu = p.req_keys & 1u, has_mem = p.req_keys & 2u;
  const int64_t cpu = has_cpu ? p.req[0] : 0;
  const int64_t mem = has_mem ? p.req[1] : 0;
  // requestCPUBind (util.go:105-122)
  bool rb = pn & PN_BIND;
  if (!rb && cpu != 0 && nbind != 0) {
    if (cpu % 1000 != 0) { o.reason = GS_NUMA_INVALID_REQUESTED_CPUS; return o; }
    rb = true;
  }
  const bool topo = nf & NF_TOPO, valid = nf & NF_TOPO_VALID;
  const int64_t alloc_cpu = sl.alloc(0), req_cpu = sl.alloc(0) - sl.free(0);
  // filterAmplifiedCPUs (plugin.go:340-373)
  if (do_filter && cpu != 0) {
    if (nf & NF_AMP_INVALID) { o.reason = GS_NUMA_INVALID_AMP_RATIO; return o; }
    const double nr = r.namp;
    if (nr > 1.0) {
      int64_t pm = rb ? amplify_d(cpu, nr) : cpu;
      if (topo && !valid) { o.reason = GS_NUMA_AVAILABLE_CPUS_ERROR; return o; }
      int64_t am = (int64_t)r.alloc_cpus * 1000;
      int64_t rq = req_cpu;
      if (rq >= am && am > 0) rq = rq - am + amplify_d(am, nr);
      if (pm > alloc_cpu - rq) { o.reason = GS_NUMA_INSUFFICIENT_AMP_CPU; return o; }
    }
  }
  const int st_req = (pn >> PN_REQ_SHIFT) & 7, st_pref = (pn >> PN_PREF_SHIFT) & 7;
  const int cpc = (nf >> NF_CPC_SHIFT) & 255;
  if (rb) {
    if (!valid) { o.reason = do_filter ? GS_NUMA_INVALID_TOPOLOGY : 0; return o; }
    if (do_filter) {
      int required = st_req;
      if (nbind == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = BIND_FULL;
      else if (nbind == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = BIND_SPREAD;
      if (st_req != BIND_UNSET && st_req != required) { o.reason = GS_NUMA_BIND_POLICY_CONFLICT; return o; }
      if (required == BIND_FULL && (cpc == 0 || p.num_cpus % cpc != 0)) { o.reason = GS_NUMA_SMT_ALIGNMENT; return o; }
      if (required != BIND_UNSET && policy == GS_NUMA_POLICY_NONE) {
        if (cnt_sel(r.tfree, required, true) < p.num_cpus) { o.reason = GS_NUMA_ALLOCATE_FAILED; return o; }
      }
    }
  }
  // getCPUBindPolicy (util.go:85-103)
  int bind = st_pref;
  bool reqflag = false;
  if (st_req != BIND_UNSET) { bind = st_req; reqflag = true; }
  else if (nbind == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS) { bind = BIND_SPREAD; reqflag = true; }
  else if (nbind == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY) { bind = BIND_FULL; reqflag = true; }
  const double amp = r.amp;
  const int64_t pcpu = (rb && amp > 1.0 && cpu != 0) ? amplify_d(cpu, amp) : cpu;   // options.requests[cpu]
  if (rb) o.flags |= GS_PLACED_CPUSET;

  // scorer over (requested, allocatable) with the pod's options.requests (scoring.go:187-226)
  auto node_score = [&](int64_t rq_cpu) -> int32_t {
    int32_t ns = 0, ws = 0;
#pragma unroll
    for (int s = 0; s < 7; ++s) {
      int32_t w = pf.numa_w[s];
      if (!w) continue;
      int64_t preq = s == 0 ? pcpu : ((p.req_keys >> s & 1u) ? p.req[s] : 0);
      if (s >= 3 && preq == 0) continue;
      int64_t al = sl.alloc(s);
      if (al == 0) continue;
      int64_t rq = (s == 0 ? rq_cpu : al - sl.free(s)) + preq;
      ns += req_score(pf.numa_most, rq, al) * w;
      ws += w;
    }
    return ws ? sdiv(ns, ws) : 0;
  };

  if (policy == GS_NUMA_POLICY_NONE) {
    const bool plain = cpu == 0 || amp <= 1.0;
    if (do_score && (plain || !(topo && !valid))) {   // scoreWithAmplifiedCPUs (scoring.go:99-116)
      const int64_t am = (int64_t)r.alloc_cpus * 1000;
      o.score = node_score(plain ? req_cpu : req_cpu - am + amplify_d(am, amp));
    }
    return o;
  }

  // ---- NUMA-policy node
  NP(0);
  if (!POLICY_NODES) return o;
  const int nz = (nf >> NF_ZONES_SHIFT) & 7;
  if (do_filter && nz == 0) { o.reason = GS_NUMA_MISSING_NUMA_RESOURCES; return o; }
  const uint32_t nf2 = r.nflags2;
  int64_t av_cpu[4], av_mem[4];
  uint32_t avk = 0;   // bit z: cpu key, bit 4+z: memory key
#pragma unroll
  for (int z = 0; z < 4; ++z) {
    av_cpu[z] = av_mem[z] = 0;
    if (z >= nz) continue;
    const bool entry = nf2 >> (NF2_ENTRY_SHIFT + z) & 1u;
    const bool ccpu = nf >> (NF_ZCPU_SHIFT + z) & 1u, cmem = nf >> (NF_ZMEM_SHIFT + z) & 1u;
    const bool acpu = entry && ((nf2 >> (NF2_ACPU_SHIFT + z) & 1u) || amp > 1.0);
    const bool amem = entry && (nf2 >> (NF2_AMEM_SHIFT + z) & 1u);
    int64_t ac = entry ? r.zraw_cpu[z] + (amp > 1.0 ? (int64_t)r.zadj[z] : 0) : 0;
    int64_t am = entry ? r.zraw_mem[z] : 0;
    if (ccpu) av_cpu[z] = r.zcap_cpu[z] - ac > 0 ? r.zcap_cpu[z] - ac : 0;
    if (cmem) av_mem[z] = r.zcap_mem[z] - am > 0 ? r.zcap_mem[z] - am : 0;
    if (ccpu || acpu) avk |= 1u << z;
    if (cmem || amem) avk |= 1u << (4 + z);
  }
  const uint32_t full_mask = (1u << nz) - 1u;
  bool aff_has = false;
  uint32_t aff = 0;
  if (do_filter && known_aff >= 0) {
    aff_has = known_aff & 0x10;
    aff = (uint32_t)known_aff & 15u;
  } else if (do_filter) {
    // GetPodTopologyHints (topology_hint.go:41-67) -> GetTopologyHints (resource_manager.go:122-138)
    bool nil_hints = false;
    int64_t hv_cpu[4];
#pragma unroll
    for (int z = 0; z < 4; ++z) hv_cpu[z] = av_cpu[z];
    if (reqflag) {   // trimNUMANodeResources (resource_manager.go:140-169)
      if (topo && !valid) {
        nil_hints = true;
      } else {
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          if (z >= nz || hv_cpu[z] == 0) continue;
          int raw = cnt_raw(r.zfree[z]);
          int n = ((int64_t)raw * 1000 >= hv_cpu[z]) ? cnt_sel(r.zfree[z], bind, true) : raw;
          if ((int64_t)n * 1000 < hv_cpu[z]) hv_cpu[z] = (int64_t)n * 1000;
        }
      }
    }
    // hint lists as bitmaps over IterateBitMasks positions (bit mi = the mi-th mask of the order), hint scores
    // (<= 100) packed 7 bits per position: no dynamically indexed arrays, nothing spills to scratch
    const uint64_t order = kMaskOrderPacked[nz - 1];
    uint32_t lc = 0, lm = 0;
    uint64_t sc_lo = 0, sc_hi = 0;
    int min_c = nz, min_m = nz;
    bool tot_c_any = false, tot_m_any = false;
    // numaScorer.score(requested = total - available (non-negative), total, pod) of the hint over mask mk
    // (resource_manager.go:454-457); evaluated only for the hints the merge below can compare
    auto mask_score = [&](uint32_t mk) -> uint64_t {
      int64_t tc = 0, tm = 0, fc = 0, fm = 0;
      bool kc = false, km = false;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        if (!(mk >> z & 1u)) continue;
        if (nf >> (NF_ZCPU_SHIFT + z) & 1u) { tc += r.zcap_cpu[z]; kc = true; }
        if (nf >> (NF_ZMEM_SHIFT + z) & 1u) { tm += r.zcap_mem[z]; km = true; }
        fc += hv_cpu[z];
        fm += av_mem[z];
      }
      int32_t ns = 0, ws = 0;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        int32_t w = pf.numa_w[s];
        if (!w) continue;
        const int64_t al = s == 0 ? (kc ? tc : 0) : (km ? tm : 0);
        if (al == 0) continue;
        const int64_t used = s == 0 ? (kc ? (tc - fc > 0 ? tc - fc : 0) : 0) : (km ? (tm - fm > 0 ? tm - fm : 0) : 0);
        const int64_t rq = used + (s == 0 ? pcpu : mem);
        ns += req_score(pf.numa_hint_most, rq, al) * w;
        ws += w;
      }
      return (uint64_t)(ws ? sdiv(ns, ws) : 0);
    };
    if (!nil_hints) {
      const int nmasks = (1 << nz) - 1;
      for (int mi = 0; mi < nmasks; ++mi) {
        if (mi == nz) {
          // all single-zone masks seen (order positions 0..nz-1): if they already settle the fast merge below
          // (preferred single-zone hints in every list, a zone common to all), larger masks cannot change
          // the kinds, minima or candidates it uses, and their hints are never compared
          const int kc1 = lc ? 1 : ((has_cpu && tot_c_any) ? 2 : 0);
          const int km1 = lm ? 1 : ((has_mem && tot_m_any) ? 2 : 0);
          uint32_t bp = (1u << nz) - 1u;
          if (kc1 == 1) bp &= lc;
          if (km1 == 1) bp &= lm;
          if ((kc1 | km1) != 0 && kc1 != 2 && km1 != 2 && (kc1 != 1 || min_c == 1) && (km1 != 1 || min_m == 1) && bp)
            break;
        }
        const uint32_t mk = (uint32_t)(order >> (4 * mi)) & 15u;
        int64_t tc = 0, tm = 0, fc = 0, fm = 0;
        bool kc = false, km = false;
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          if (!(mk >> z & 1u)) continue;
          if (nf >> (NF_ZCPU_SHIFT + z) & 1u) { tc += r.zcap_cpu[z]; kc = true; }
          if (nf >> (NF_ZMEM_SHIFT + z) & 1u) { tm += r.zcap_mem[z]; km = true; }
          fc += hv_cpu[z];
          fm += av_mem[z];
        }
        const int cnt = __popc(mk);
        // generateHints: memory group first, then cpu (resource_manager.go:464-476, 499-532)
        if (has_mem) {
          if (km) tot_m_any = true;
          if (tm >= mem) {
            if (cnt < min_m) min_m = cnt;
            if (fm >= mem) lm |= 1u << mi;
          }
        }
        if (has_cpu) {
          if (kc) tot_c_any = true;
          if (tc >= pcpu) {
            if (cnt < min_c) min_c = cnt;
            if (fc >= pcpu) lc |= 1u << mi;
          }
        }
      }
    }
    NP(1);
    auto mask_at = [&](int mi) -> uint32_t { return (uint32_t)(order >> (4 * mi)) & 15u; };
    auto score_at = [&](int mi) -> int32_t {
      return (int32_t)((mi < 9 ? sc_lo >> (7 * mi) : sc_hi >> (7 * (mi - 9))) & 127u);
    };
    // filterProvidersHints (policy.go:98-126): lists in resource-name order cpu, memory.
    // kind: 0 absent, 1 hints, 2 the empty-list marker {nil, false}
    const int kc_kind = nil_hints ? 0 : (lc ? 1 : ((has_cpu && tot_c_any) ? 2 : 0));
    const int km_kind = nil_hints ? 0 : (lm ? 1 : ((has_mem && tot_m_any) ? 2 : 0));
    const bool single = policy == GS_NUMA_POLICY_SINGLE_NUMA_NODE;
    const bool no_lists = kc_kind == 0 && km_kind == 0;   // empty map: one preferred any-numa hint
    const bool use0 = no_lists || kc_kind != 0, use1 = !no_lists && km_kind != 0;
    // mergeFilteredHints (policy.go:128-186) with filterSingleNumaHints for SingleNUMANode
    bool b_has = true, b_pref = false;
    uint32_t b_mask = full_mask;
    int32_t b_score = 0;
    // Fast path (exact): when every present list has single-zone preferred hints (min size 1), a preferred
    // merged hint is only produced by equal single-bit masks, so the preferred, narrowest candidates are the
    // single zones z present in every list, visited in ascending z; mergeFilteredHints then keeps the first
    // one of maximal score. (The 1-bit masks occupy order positions 0..nz-1.)
    const uint32_t ones = (1u << nz) - 1u;
    uint32_t both = 0xFu;
    bool fast = !no_lists && (kc_kind == 1 || kc_kind == 0) && (km_kind == 1 || km_kind == 0);
    if (fast && kc_kind == 1) { fast = min_c == 1; both &= lc & ones; }
    if (fast && km_kind == 1) { fast = min_m == 1; both &= lm & ones; }
    fast = fast && both != 0;
    // Preferred-first merge (exact): the first preferred merged hint is always taken and a non-preferred one
    // never replaces a preferred best, so the permutation scan's result equals the scan over the pairs of
    // preferred entries alone whenever one of them merges to a non-empty mask (pass 0, at most 6 x 6 pairs);
    // only otherwise does the full scan run (pass 1). Both visit pairs in policy.go's order.
    uint32_t pre0 = 0, pre1 = 0;
    if (!fast && !nil_hints) {
      for (uint32_t rr = lc; rr; rr &= rr - 1) {
        const int mi = __ffs(rr) - 1;
        if (__popc(mask_at(mi)) == min_c) pre0 |= 1u << mi;
      }
      for (uint32_t rr = lm; rr; rr &= rr - 1) {
        const int mi = __ffs(rr) - 1;
        if (__popc(mask_at(mi)) == min_m) pre1 |= 1u << mi;
      }
    }
    bool b_pref_after0 = false;   // diagnostics: pass 0 settled the merge
    for (int pass = 0; pass < 2; ++pass) {
      if (pass == 1) {
        b_pref_after0 = b_pref;
        if (fast || b_pref) break;
        b_mask = full_mask;
        b_pref = false;
        b_score = 0;
      }
      // scores of the hints this pass compares (single-zone candidates, preferred entries, then the rest)
      if (!nil_hints) {
        const uint32_t need = pass == 1 ? (lc | lm) & ~(pre0 | pre1) : (fast ? both : (pre0 | pre1));
        for (uint32_t rr = need; rr; rr &= rr - 1) {
          const int mi = __ffs(rr) - 1;
          const uint64_t hs = mask_score(mask_at(mi));
          if (mi < 9) sc_lo |= hs << (7 * mi);
          else sc_hi |= hs << (7 * (mi - 9));
        }
      }
      if (fast) {
        int best_z = 0, best_s = -1;
        for (uint32_t rr = both; rr; rr &= rr - 1) {
          const int z = __ffs(rr) - 1;
          const int sz = score_at(z);
          if (sz > best_s) { best_s = sz; best_z = z; }
        }
        b_mask = 1u << best_z;
        b_pref = true;
        b_score = best_s;
        continue;
      }
      // a list as a sequence of entries: kind 1 = its set bits, kind 2 / absent = a single pseudo entry (bit 31)
      const uint32_t set0 = kc_kind == 1 ? (pass == 0 ? pre0 : lc) : 0x80000000u;
      const uint32_t set1 = km_kind == 1 ? (pass == 0 ? pre1 : lm) : 0x80000000u;
      for (uint32_t r0 = set0; r0; r0 &= r0 - 1) {
        const int i0 = __ffs(r0) - 1;
        bool h0 = false, p0 = true;
        uint32_t m0 = 0;
        int32_t s0 = 0;
        if (kc_kind == 1) { h0 = true; m0 = mask_at(i0); p0 = __popc(m0) == min_c; s0 = score_at(i0); }
        else if (kc_kind == 2) { p0 = false; }
        if (use0 && single && !(p0 && (!h0 || __popc(m0) == 1))) continue;
        for (uint32_t r1 = set1; r1; r1 &= r1 - 1) {
          const int i1 = __ffs(r1) - 1;
          bool h1 = false, p1 = true;
          uint32_t m1 = 0;
          int32_t s1 = 0;
          if (use1) {
            if (km_kind == 1) { h1 = true; m1 = mask_at(i1); p1 = __popc(m1) == min_m; s1 = score_at(i1); }
            else { p1 = false; }
            if (single && !(p1 && (!h1 || __popc(m1) == 1))) continue;
          }
          uint32_t mg = full_mask;
          bool pg = true;
          if (use0) { mg &= h0 ? m0 : full_mask; pg = pg && p0; }
          if (use1) { mg &= h1 ? m1 : full_mask; pg = pg && p1; }
          if (mg == 0) continue;
          int32_t sg = 0;
          if (use0 && h0 && m0 == mg && s0 > sg) sg = s0;
          if (use1 && h1 && m1 == mg && s1 > sg) sg = s1;
          if (pg && !b_pref) { b_mask = mg; b_pref = pg; b_score = sg; continue; }
          if (!pg && b_pref) continue;
          if (!narrower(mg, b_mask)) {
            if (__popc(mg) == __popc(b_mask) && sg > b_score) { b_mask = mg; b_pref = pg; b_score = sg; }
            continue;
          }
          b_mask = mg; b_pref = pg; b_score = sg;
        }
      }
    }
    NP(2);
    {   // diagnostics: merge path counters: [6] fast, [7] preferred pass only, [8] full pass, [9] a lane of the
        // wave (among those here with this pair's lane) ran a full pass
      const bool full = !fast && !nil_hints && !b_pref_after0;
      const bool wave_full = __ballot(full) != 0;
      if (prof) {
        prof[fast ? 6 : (full ? 8 : 7)] += 1;
        if (wave_full) prof[9] += 1;
      }
    }
    bool admit = true;
    if (single) {
      if (b_mask == full_mask) b_has = false;   // policy_single_numa_node.go:70-73
      admit = b_pref;
    } else if (policy == GS_NUMA_POLICY_RESTRICTED) {
      admit = b_pref;
    }
    if (!admit) { o.reason = GS_NUMA_AFFINITY_ERROR; return o; }
    aff_has = b_has;
    aff = b_mask;
  }
  // resourceManager.Allocate with the affinity (resource_manager.go:171-193)
  bool fail = false;
  if (aff_has) {   // allocateResourcesByHint with the pod's original requests (:195-250)
    int64_t rc = cpu, rm = mem;
    bool ic = false, im = false;
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      if (!(aff >> z & 1u)) continue;
      if (has_cpu && (avk >> z & 1u)) {
        ic = true;
        int64_t a = av_cpu[z], got = a > rc ? rc : a;
        rc -= got;
        if (got) { o.zkeys |= 1u << z; o.zcpu[z] = got; }
      }
      if (has_mem && (avk >> (4 + z) & 1u)) {
        im = true;
        int64_t a = av_mem[z], got = a > rm ? rm : a;
        rm -= got;
        if (got) { o.zkeys |= 1u << (4 + z); o.zmem[z] = got; }
      }
    }
    if ((ic && rc != 0) || (im && rm != 0)) fail = true;
  }
  NP(3);
  if (!fail && rb) {   // allocateCPUSet (resource_manager.go:273-360), counted
    if (cnt_sel(r.tfree, bind, reqflag) < p.num_cpus) fail = true;
    // satisfiedRequiredCPUBindPolicy: FullPCPUs over full cores is met iff the count is a multiple of CPUsPerCore
    if (!fail && !o.zkeys && reqflag && bind == BIND_FULL && cpc && p.num_cpus % cpc) fail = true;
    if (!fail && o.zkeys) {
      int sum = 0;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        if (!((o.zkeys >> z & 1u) || (o.zkeys >> (4 + z) & 1u))) continue;
        int avail = cnt_sel(r.zfree[z], bind, reqflag);
        int want = (int)(o.zcpu[z] / 1000);
        int n = want < avail ? want : avail;
        if (reqflag && bind == BIND_FULL && cpc && n % cpc) fail = true;
        sum += n;
      }
      if (sum != p.num_cpus) fail = true;
    }
  }
  if (fail) {
    if (do_filter) o.reason = GS_NUMA_ADMIT_ALLOCATE_FAILED;
    o.score = 0;
    return o;
  }
  if (o.zkeys) o.flags |= GS_PLACED_NUMA;
  if (aff_has) { o.flags |= aff << GS_PLACED_AFFINITY_SHIFT; o.aff = 0x10u | aff; }
  NP(4);
  if (do_score) {   // calculateAllocatableAndRequested (scoring.go:118-164)
    if (o.zkeys) {
      int64_t ac = 0, am = 0, rqc = 0, rqm = 0;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        if (!((o.zkeys >> z & 1u) || (o.zkeys >> (4 + z) & 1u))) continue;
        if (nf >> (NF_ZCPU_SHIFT + z) & 1u) ac += r.zcap_cpu[z];
        if (nf >> (NF_ZMEM_SHIFT + z) & 1u) am += r.zcap_mem[z];
        if (nf2 >> (NF2_ENTRY_SHIFT + z) & 1u) {
          rqc += r.zraw_cpu[z] + (amp > 1.0 ? (int64_t)r.zadj[z] : 0);
          rqm += r.zraw_mem[z];
        }
      }
      if (rb) rqc = amplify_d((int64_t)r.alloc_cpus * 1000, amp);
      int32_t ns = 0, ws = 0;
#pragma unroll
      for (int s = 0; s < 2; ++s) {   // zone totals carry only cpu / memory
        int32_t w = pf.numa_w[s];
        if (!w) continue;
        const int64_t al = s == 0 ? ac : am;
        if (al == 0) continue;
        const int64_t rq = (s == 0 ? rqc : rqm) + (s == 0 ? pcpu : mem);
        ns += req_score(pf.numa_most, rq, al) * w;
        ws += w;
      }
      o.score = ws ? sdiv(ns, ws) : 0;
    } else {
      o.score = node_score(rb ? amplify_d((int64_t)r.alloc_cpus * 1000, amp) : req_cpu);
    }
  }
  NP(5);
#undef NP
  return o;
}

}  // namespace gs
