// gs_numa_dev.h — NodeNUMAResource Filter + Score of one (pod, node) pair on the device (gfx950).
//
// Restates pkg/scheduler/plugins/nodenumaresource/{plugin.go Filter/filterAmplifiedCPUs, scoring.go Score,
// resource_manager.go GetTopologyHints/Allocate, topology_hint.go} and frameworkext/topologymanager/policy*.go
// over the count summaries the host keeps in HBM (gs_layout.h C_NFLAGS.. C_ZADJ0):
//  * cpuset feasibility of allocateCPUSet is a count test: with the required-policy prefilter applied every
//    available CPU lies in a full core (FullPCPUs) or on a distinct core (SpreadByPCPUs), and takeCPUs takes
//    prefixes of core-ordered lists, so the result satisfies the policy iff per-zone counts are multiples of
//    CPUsPerCore (FullPCPUs with a NUMA split) — which CPUs are picked is a Reserve concern (gs_cpuset_dev.h);
//  * NUMA hints are enumerated over zone-slot masks (zones sorted by node id, so slot masks order and
//    intersect exactly like node-id masks) in bitmask.IterateBitMasks order; the hint lists of the single
//    provider are merged in sorted resource-name order (cpu before memory; the reference iterates a Go map,
//    policy.go:108 — see DESIGN.md) with mergeFilteredHints' exact update rule.
//
// SIMT shape. A hint list is a bitmap over the 15 positions of the 4-zone IterateBitMasks order (bitmask.go
// :206-222): masks 1 2 4 8 | 3 5 9 6 10 12 | 7 11 13 14 | 15. For nz < 4 zones the order is the same sequence
// with the masks >= 2^nz left out, so one position numbering serves every zone count, positions are sorted by
// mask size, and single-zone masks sit at positions 0..3. The row-side sums a position needs (zone totals and
// free amounts of its mask) come from a "hint source": HintRegs computes them from the row's per-zone values
// (a thread owning a node row: eval kernels, Reserve); HintTable reads them from a table built once per row in
// LDS (the commit kernel re-scores one row for many pods, one pod per lane). Everything per pod is compares
// on those sums, so a lane's work does not grow with the number of masks the row has.
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
// leastRequestedScore / mostRequestedScore (least_allocated.go:49-58, most_allocated.go:45-55) with one
// division site
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

// ---- IterateBitMasks positions (4-zone order)
constexpr uint64_t kOrd4 = 0xFEDB7CA69538421ull;   // position mi -> zone-slot mask, 4 bits per position
__host__ __device__ constexpr uint32_t ord_mask(int mi) { return (uint32_t)(kOrd4 >> (4 * mi)) & 15u; }
// positions present for nz zones (masks < 2^nz): nz = 1..4
__host__ __device__ __forceinline__ uint32_t ord_valid(int nz) {
  return nz >= 4 ? 0x7FFFu : nz == 3 ? 0x4B7u : nz == 2 ? 0x13u : nz == 1 ? 0x1u : 0u;
}
// mask size of the first position of a non-empty position set (positions are sorted by mask size)
__host__ __device__ __forceinline__ int ord_size_first(uint32_t pos) {
  const int mi = __builtin_ctz(pos);
  return mi < 4 ? 1 : mi < 10 ? 2 : mi < 14 ? 3 : 4;
}
__device__ __forceinline__ bool narrower(uint32_t a, uint32_t b) {   // bitmask.IsNarrowerThan
  int ca = __popc(a), cb = __popc(b);
  return ca == cb ? a < b : ca < cb;
}

// Row-side sums of one position: zone totals of the zones listing cpu / memory, and the available (free) amounts
// of all the mask's zones (cpu after trimNUMANodeResources for the pod's bind policy, see HintVariant).
struct HintSums {
  int64_t tc, tm, fc, fm;
};
// trimNUMANodeResources (resource_manager.go:140-169) variants of the available cpu per zone: 0 untrimmed (no
// required bind policy), 1 FullPCPUs, 2 SpreadByPCPUs, 3 another required policy (raw count)
__device__ __forceinline__ int hint_variant(bool reqflag, int bind) {
  return !reqflag ? 0 : bind == BIND_FULL ? 1 : bind == BIND_SPREAD ? 2 : 3;
}

// Per-zone availability of a NUMA-policy row (numa_eval's av_cpu / av_mem / key bits): zone capacity minus the
// allocated resources of NodeAllocation (cpu amplified by the zone adjustment), floored at 0.
struct ZoneAvail {
  int64_t av_cpu[4], av_mem[4];
  uint32_t avk;   // bit z: allocatable has a cpu key in zone z, bit 4+z: memory key
};
__device__ __forceinline__ ZoneAvail zone_avail(const NumaRow& r) {
  ZoneAvail a;
  const uint32_t nf = r.nflags, nf2 = r.nflags2;
  const int nz = (nf >> NF_ZONES_SHIFT) & 7;
  const double amp = r.amp;
  a.avk = 0;
#pragma unroll
  for (int z = 0; z < 4; ++z) {
    a.av_cpu[z] = a.av_mem[z] = 0;
    if (z >= nz) continue;
    const bool entry = nf2 >> (NF2_ENTRY_SHIFT + z) & 1u;
    const bool ccpu = nf >> (NF_ZCPU_SHIFT + z) & 1u, cmem = nf >> (NF_ZMEM_SHIFT + z) & 1u;
    const bool acpu = entry && ((nf2 >> (NF2_ACPU_SHIFT + z) & 1u) || amp > 1.0);
    const bool amem = entry && (nf2 >> (NF2_AMEM_SHIFT + z) & 1u);
    const int64_t ac = entry ? r.zraw_cpu[z] + (amp > 1.0 ? (int64_t)r.zadj[z] : 0) : 0;
    const int64_t am = entry ? r.zraw_mem[z] : 0;
    if (ccpu) a.av_cpu[z] = r.zcap_cpu[z] - ac > 0 ? r.zcap_cpu[z] - ac : 0;
    if (cmem) a.av_mem[z] = r.zcap_mem[z] - am > 0 ? r.zcap_mem[z] - am : 0;
    if (ccpu || acpu) a.avk |= 1u << z;
    if (cmem || amem) a.avk |= 1u << (4 + z);
  }
  return a;
}
// available cpu of zone z in variant v (trimNUMANodeResources: min(available, usable CPUs x 1000))
__device__ __forceinline__ int64_t trimmed_cpu(int64_t av, uint32_t zfree, int v) {
  if (v == 0 || av == 0) return av;
  const int raw = cnt_raw(zfree);
  int n = raw;
  if (v != 3 && (int64_t)raw * 1000 >= av) n = v == 1 ? (int)((zfree >> 9) & 511u) : (int)((zfree >> 18) & 511u);
  return (int64_t)n * 1000 < av ? (int64_t)n * 1000 : av;
}

// Hint source over a row in registers: sums of a position's zones computed from per-zone values.
struct HintRegs {
  int64_t zc[4], zm[4], hc[4], hm[4];   // zone totals (listed zones, else 0), available cpu (variant), memory
  __device__ HintSums sum(int mi) const {
    const uint32_t mk = ord_mask(mi);
    HintSums s{0, 0, 0, 0};
#pragma unroll
    for (int z = 0; z < 4; ++z)
      if (mk >> z & 1u) { s.tc += zc[z]; s.tm += zm[z]; s.fc += hc[z]; s.fm += hm[z]; }
    return s;
  }
};
__device__ __forceinline__ HintRegs hint_regs(const NumaRow& r, const ZoneAvail& a, int v) {
  HintRegs h;
  const uint32_t nf = r.nflags;
#pragma unroll
  for (int z = 0; z < 4; ++z) {
    h.zc[z] = (nf >> (NF_ZCPU_SHIFT + z) & 1u) ? r.zcap_cpu[z] : 0;
    h.zm[z] = (nf >> (NF_ZMEM_SHIFT + z) & 1u) ? r.zcap_mem[z] : 0;
    h.hc[z] = trimmed_cpu(a.av_cpu[z], r.zfree[z], v);
    h.hm[z] = a.av_mem[z];
  }
  return h;
}

// Hint source over a table of a row's position sums (built once per row, read by every lane of a wave).
struct HintTable {
  int64_t tc[16], tm[16], fm[16];
  int64_t fc[4][16];                    // per variant
};
struct HintTableRef {
  const HintTable* t;
  int v;
  __device__ HintSums sum(int mi) const { return HintSums{t->tc[mi], t->tm[mi], t->fc[v][mi], t->fm[mi]}; }
};
// builds entry `e` (0..63) of the table: lanes 0..59 cover position e % 15 of value kind e / 15
__device__ __forceinline__ void hint_table_fill(HintTable& t, const NumaRow& r, const ZoneAvail& a, int e) {
  if (e >= 60) return;
  const int mi = e % 15, kind = e / 15;
  const uint32_t mk = ord_mask(mi), nf = r.nflags;
  int64_t tc = 0, tm = 0, fm = 0, f[4] = {0, 0, 0, 0};
#pragma unroll
  for (int z = 0; z < 4; ++z) {
    if (!(mk >> z & 1u)) continue;
    if (kind == 0) {
      tc += (nf >> (NF_ZCPU_SHIFT + z) & 1u) ? r.zcap_cpu[z] : 0;
      tm += (nf >> (NF_ZMEM_SHIFT + z) & 1u) ? r.zcap_mem[z] : 0;
      fm += a.av_mem[z];
    } else {
      // kind 1..3: variants 0 and kind (FullPCPUs / SpreadByPCPUs / raw) of the available cpu
      f[0] += a.av_cpu[z];
      f[1] += trimmed_cpu(a.av_cpu[z], r.zfree[z], kind);
    }
  }
  if (kind == 0) { t.tc[mi] = tc; t.tm[mi] = tm; t.fm[mi] = fm; }
  else {
    if (kind == 1) t.fc[0][mi] = f[0];
    t.fc[kind][mi] = f[1];
  }
}

// numaScorer.score(requested = total - available (floored at 0), total, pod) of a hint (resource_manager.go
// :454-457): zone totals carry only cpu / memory. (The sums already exclude zones that do not list a resource.)
__device__ __forceinline__ int32_t hint_score(const HintSums& s, int64_t pcpu, int64_t mem, const Profile& pf) {
  int32_t ns = 0, ws = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int32_t w = pf.numa_w[k];
    if (!w) continue;
    const int64_t al = k == 0 ? s.tc : s.tm;
    if (al == 0) continue;
    const int64_t f = k == 0 ? s.fc : s.fm;
    const int64_t used = al - f > 0 ? al - f : 0;
    ns += req_score(pf.numa_hint_most, used + (k == 0 ? pcpu : mem), al) * w;
    ws += w;
  }
  return ws ? sdiv(ns, ws) : 0;
}

// topologyManager policy Merge + admit over the provider's hint lists (policy.go:68-186, policy_*.go), given as
// position bitmaps (lc cpu, lm memory) with the positions whose total covers the request (totc, totm); score_at(mi)
// = the hint score of position mi. Returns the admit verdict; aff_has / aff = the merged affinity.
template <class ScoreAt>
__device__ __forceinline__ bool merge_hint_lists(uint32_t totc, uint32_t lc, uint32_t totm, uint32_t lm, int nz,
                                                 int policy, bool nil_hints, bool has_cpu, bool has_mem,
                                                 bool tot_c_any, bool tot_m_any, ScoreAt&& score_at, bool& aff_has,
                                                 uint32_t& aff) {
  const int min_c = totc ? ord_size_first(totc) : nz, min_m = totm ? ord_size_first(totm) : nz;
  // filterProvidersHints (policy.go:98-126): lists in resource-name order cpu, memory.
  // kind: 0 absent, 1 hints, 2 the empty-list marker {nil, false}
  const int kc = nil_hints ? 0 : (lc ? 1 : ((has_cpu && tot_c_any) ? 2 : 0));
  const int km = nil_hints ? 0 : (lm ? 1 : ((has_mem && tot_m_any) ? 2 : 0));
  const bool single = policy == GS_NUMA_POLICY_SINGLE_NUMA_NODE;
  const bool no_lists = kc == 0 && km == 0;   // empty map: one preferred any-numa hint
  const bool use0 = no_lists || kc != 0, use1 = !no_lists && km != 0;
  const uint32_t full_mask = (1u << nz) - 1u;
  bool b_pref = false;
  uint32_t b_mask = full_mask;
  int32_t b_score = 0;
  // Fast path (exact): when every present list has single-zone preferred hints (min size 1), a preferred merged
  // hint is only produced by equal single-bit masks, so the preferred, narrowest candidates are the single zones
  // present in every list (positions 0..nz-1), visited in ascending zone order; mergeFilteredHints keeps the first
  // one of maximal score.
  uint32_t both = full_mask;
  bool fast = !no_lists && kc != 2 && km != 2;
  if (fast && kc == 1) { fast = min_c == 1; both &= lc; }
  if (fast && km == 1) { fast = min_m == 1; both &= lm; }
  fast = fast && both != 0;
  if (fast) {
    int best_s = -1;
    for (uint32_t rr = both; rr; rr &= rr - 1) {
      const int z = __ffs(rr) - 1;
      const int sz = score_at(z);
      if (sz > best_s) { best_s = sz; b_mask = 1u << z; }
    }
    b_pref = true;
    b_score = best_s;
  } else {
    // Preferred-first merge (exact): the first preferred merged hint is always taken and a non-preferred one never
    // replaces a preferred best, so the permutation scan equals the scan over the pairs of preferred entries alone
    // whenever one of them merges to a non-empty mask (pass 0); only otherwise does the full scan run (pass 1,
    // where no pair is preferred). Both visit pairs in policy.go's order.
    uint32_t pre0 = 0, pre1 = 0;
    for (uint32_t rr = lc; rr; rr &= rr - 1) {
      const int mi = __ffs(rr) - 1;
      if (__popc(ord_mask(mi)) == min_c) pre0 |= 1u << mi;
    }
    for (uint32_t rr = lm; rr; rr &= rr - 1) {
      const int mi = __ffs(rr) - 1;
      if (__popc(ord_mask(mi)) == min_m) pre1 |= 1u << mi;
    }
    for (int pass = 0; pass < 2; ++pass) {
      if (pass == 1) {
        if (b_pref) break;
        b_mask = full_mask;
        b_score = 0;
      }
      // a list as a sequence of entries: kind 1 = its set bits, kind 2 / absent = a single pseudo entry (bit 31)
      const uint32_t set0 = kc == 1 ? (pass == 0 ? pre0 : lc) : 0x80000000u;
      const uint32_t set1 = km == 1 ? (pass == 0 ? pre1 : lm) : 0x80000000u;
      for (uint32_t r0 = set0; r0; r0 &= r0 - 1) {
        const int i0 = __ffs(r0) - 1;
        const bool h0 = kc == 1;
        const uint32_t m0 = h0 ? ord_mask(i0) : 0u;
        const bool p0 = h0 ? __popc(m0) == min_c : kc == 0;
        if (use0 && single && !(p0 && (!h0 || __popc(m0) == 1))) continue;
        for (uint32_t r1 = set1; r1; r1 &= r1 - 1) {
          const int i1 = __ffs(r1) - 1;
          const bool h1 = use1 && km == 1;
          const uint32_t m1 = h1 ? ord_mask(i1) : 0u;
          const bool p1 = h1 ? __popc(m1) == min_m : !use1;
          if (use1 && single && !(p1 && (!h1 || __popc(m1) == 1))) continue;
          uint32_t mg = full_mask;
          bool pg = true;
          if (use0) { mg &= h0 ? m0 : full_mask; pg = pg && p0; }
          if (use1) { mg &= h1 ? m1 : full_mask; pg = pg && p1; }
          if (mg == 0) continue;
          if (!pg && b_pref) continue;
          // candidates that cannot replace the best skip their score: a wider mask never does, nor an equally wide
          // one that is not narrower unless its score is higher (the score is only needed then)
          const bool nar = narrower(mg, b_mask);
          if (!(pg && !b_pref) && !nar && __popc(mg) != __popc(b_mask)) continue;
          int32_t sg = 0;
          if (use0 && h0 && m0 == mg) sg = score_at(i0);
          if (use1 && h1 && m1 == mg) { const int32_t s1 = score_at(i1); if (s1 > sg) sg = s1; }
          if (pg && !b_pref) { b_mask = mg; b_pref = true; b_score = sg; continue; }
          if (!nar) {
            if (sg > b_score) { b_mask = mg; b_pref = pg; b_score = sg; }
            continue;
          }
          b_mask = mg; b_pref = pg; b_score = sg;
        }
      }
    }
  }
  aff_has = true;
  aff = b_mask;
  if (single) {
    if (b_mask == full_mask) aff_has = false;   // policy_single_numa_node.go:70-73
    return b_pref;
  }
  if (policy == GS_NUMA_POLICY_RESTRICTED) return b_pref;
  return true;
}

// ---- a second hint provider: DeviceShare (deviceshare/topology_hint.go:33-214), the extension path's GPU pods
// Its hints for one node, packed: bits 0-14 the IterateBitMasks positions that hold a hint (masks over the zones of the
// node's GPUs with enough devices in total, where the GPU allocation succeeds), bits 16-18 the size minimum over the
// masks with enough devices (hints of that size are preferred), bits 20-21 the number of resource names of the
// per-instance request (each gets the same list; 0 = the provider has no hints: its preferred any-numa hint is
// neutral). No position with r > 0: every list is empty ({nil, not preferred} in filterProvidersHints).
constexpr uint32_t GH_LIST = 0x7FFFu, GH_MIN_SHIFT = 16, GH_R_SHIFT = 20;

struct HintList {        // one list of filterProvidersHints' output
  uint32_t set;          // IterateBitMasks positions of its hints, or bit 31 alone: one mask-less hint
  int8_t min;            // hint size that is preferred (position lists)
  bool pseudo_pref;      // the mask-less hint's Preferred
  bool scored;           // NodeNUMAResource's lists carry hint scores (DeviceShare's score 0)
};
constexpr int kGenMergeMax = 1 << 16;   // search steps one pass may take (the caller fails loudly beyond)

// topologyManager Merge over any provider lists (policy.go:128-186, policy_*.go), lists in filterProvidersHints
// order, exact. mergeFilteredHints visits the permutations in lexicographic order with a non-associative update
// (a preferred hint beats a non-preferred one; then a narrower mask wins, an equally wide one only with a higher
// score), so the result depends on the order — but only through few candidates:
//  * preferred-first (as merge_hint_lists): pass 0 over the preferred entries; pass 1, all entries, only when no
//    preferred permutation merges to a non-empty mask (then every candidate is non-preferred);
//  * within a pass, once a candidate of the smallest non-empty size p* appears it replaces the best (it is narrower
//    than anything wider, or the first preferred one), and wider candidates never replace it afterwards: the result is
//    the update folded over the size-p* candidates alone, in order — a narrower mask (smaller value) always replaces,
//    another only with a higher score;
//  * the depth-first walk over the lists skips a subtree whose reachable merged masks (bit sets over the 16 masks,
//    from a backward pass) hold no size-p* mask, or, below the last scored list (the scores are then fixed), none
//    that could replace the current best.
// HintList::scored lists carry score_at(position) (NodeNUMAResource's hint scores; DeviceShare's are 0).
// *over: a pass took more than kGenMergeMax steps (the result is then not used).
template <class ScoreAt>
__host__ __device__ __noinline__ bool merge_hint_lists_gen(const HintList* L, int nl, int nz, int policy, ScoreAt&& score_at,
                                                  bool& aff_has, uint32_t& aff, bool& over) {
  const bool single = policy == GS_NUMA_POLICY_SINGLE_NUMA_NODE;
  const uint32_t full_mask = (1u << nz) - 1u;
  constexpr uint32_t PSEUDO = 0x80000000u;
  auto em = [&](int e) -> uint32_t { return e == 31 ? full_mask : ord_mask(e); };
  uint32_t s0[6], s1[6];
  int nsc = 0;   // lists [0, nsc) hold every scored one
  for (int l = 0; l < nl; ++l) {
    uint32_t all, pref;
    if (L[l].set == PSEUDO) {
      all = PSEUDO;
      pref = L[l].pseudo_pref ? PSEUDO : 0u;
    } else {
      all = L[l].set;
      pref = 0;
      for (uint32_t rr = all; rr; rr &= rr - 1) {
        const int mi = __builtin_ctz(rr);
        if (__builtin_popcount(ord_mask(mi)) == L[l].min) pref |= 1u << mi;
      }
    }
    if (single) {   // policy_single_numa_node.go:48-78: preferred mask-less or preferred single-zone hints only
      all = (L[l].set == PSEUDO) ? pref : (L[l].min == 1 ? pref & 0xFu : 0u);
      pref = all;
    }
    s0[l] = pref;
    s1[l] = all;
    if (L[l].scored) nsc = l + 1;
  }
  int16_t scache[15];
  for (int i = 0; i < 15; ++i) scache[i] = -1;
  int ent[6];
  auto s_of = [&](uint32_t x) -> int32_t {   // the merged hint's score: the scored entries whose mask equals it
    int32_t sx = 0;
    for (int l = 0; l < nsc; ++l) {
      const int e = ent[l];
      if (!L[l].scored || e == 31 || ord_mask(e) != x) continue;
      if (scache[e] < 0) scache[e] = (int16_t)score_at(e);
      if (scache[e] > sx) sx = scache[e];
    }
    return sx;
  };
  bool b_pref = false;
  uint32_t b_mask = full_mask;
  over = false;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1 && b_pref) break;
#ifndef GS_MERGE_PTR_SELECT
    uint32_t S[6];   // this pass's entry sets (a copy: a pointer selecting s0 / s1 miscompiled on gfx950)
    bool empty = false;
    for (int l = 0; l < nl; ++l) {
      S[l] = pass ? s1[l] : s0[l];
      empty |= S[l] == 0;
    }
#else   // the round-4 form, only in scripts/sanitize/merge_ptr_probe.hip (the miscompile's reproducer)
    const uint32_t* S = pass ? s1 : s0;
    bool empty = false;
    for (int l = 0; l < nl; ++l) empty |= S[l] == 0;
#endif
    if (empty) continue;   // a list without entries: no permutation
    uint32_t fw = 1u << full_mask;   // merged masks reachable after each list (bit x = mask x)
    for (int l = 0; l < nl; ++l) {
      uint32_t nx = 0;
      for (uint32_t yy = fw; yy; yy &= yy - 1)
        for (uint32_t ee = S[l]; ee; ee &= ee - 1) nx |= 1u << ((uint32_t)__builtin_ctz(yy) & em(__builtin_ctz(ee)));
      fw = nx;
    }
    const uint32_t fin = fw & ~1u;
    if (!fin) continue;
    int pstar = 5;
    for (uint32_t xx = fin; xx; xx &= xx - 1) pstar = min(pstar, __builtin_popcount((uint32_t)__builtin_ctz(xx)));
    uint32_t P = 0;
    for (uint32_t xx = fin; xx; xx &= xx - 1)
      if (__builtin_popcount((uint32_t)__builtin_ctz(xx)) == pstar) P |= 1u << __builtin_ctz(xx);
    uint16_t rb[6][16];   // rb[l][y]: merged masks reachable from the partial merge y before list l
    for (int y = 0; y < 16; ++y) rb[nl][y] = (uint16_t)(1u << y);
    for (int l = nl - 1; l >= 0; --l)
      for (int y = 0; y < 16; ++y) {
        uint32_t acc = 0;
        for (uint32_t ee = S[l]; ee; ee &= ee - 1) acc |= rb[l + 1][(uint32_t)y & em(__builtin_ctz(ee))];
        rb[l][y] = (uint16_t)acc;
      }
    bool have = false;
    uint32_t b = 0;
    int32_t sb = 0;
    auto pruned = [&](int l, uint32_t y) -> bool {
      const uint32_t cand = rb[l][y] & P;
      if (!cand) return true;
      if (!have || l < nsc) return false;
      for (uint32_t xx = cand; xx; xx &= xx - 1) {
        const uint32_t x = (uint32_t)__builtin_ctz(xx);
        if (x < b || s_of(x) > sb) return false;
      }
      return true;
    };
    uint32_t rem[6], yv[6];
    int l = 0, steps = 0;
    yv[0] = full_mask;
    rem[0] = S[0];
    while (l >= 0) {
      if (rem[l] == 0) { --l; continue; }
      const int e = __builtin_ctz(rem[l]);
      rem[l] &= rem[l] - 1;
      if (++steps > kGenMergeMax) { over = true; break; }
      ent[l] = e;
      const uint32_t y = yv[l] & em(e);
      if (pruned(l + 1, y)) continue;
      if (l + 1 == nl) {   // a size-p* candidate that replaces the best (or the first one)
        const int32_t sx = s_of(y);
        if (!have || y < b || sx > sb) { have = true; b = y; sb = sx; }
        continue;
      }
      ++l;
      yv[l] = y;
      rem[l] = S[l];
    }
    if (over) break;
    if (have) {
      b_mask = b;
      if (pass == 0) b_pref = true;
    }
  }
  aff_has = true;
  aff = b_mask;
  if (single) {
    if (b_mask == full_mask) aff_has = false;
    return b_pref;
  }
  if (policy == GS_NUMA_POLICY_RESTRICTED) return b_pref;
  return true;
}

// filterProvidersHints' lists of both providers: NodeNUMAResource's (cpu, then memory: the sorted names; kinds as
// merge_hint_lists reads them) from its position bitmaps, then DeviceShare's r identical lists (gh, GH_* above).
// Returns the number of lists (<= 5).
__host__ __device__ __forceinline__ int gen_lists(uint32_t totc, uint32_t lc, uint32_t totm, uint32_t lm, uint32_t valid,
                                         bool nil_hints, bool has_cpu, bool has_mem, bool tot_c_any, bool tot_m_any,
                                         uint32_t gh, HintList* L) {
  int nl = 0;
  const int kc = nil_hints ? 0 : (lc ? 1 : ((has_cpu && tot_c_any) ? 2 : 0));
  const int km = nil_hints ? 0 : (lm ? 1 : ((has_mem && tot_m_any) ? 2 : 0));
  if (kc == 0 && km == 0) {
    L[nl++] = HintList{0x80000000u, 0, true, false};   // no hints: one preferred any-numa hint
  } else {
    if (kc == 1) L[nl++] = HintList{lc, (int8_t)ord_size_first(totc), false, true};
    if (kc == 2) L[nl++] = HintList{0x80000000u, 0, false, false};
    if (km == 1) L[nl++] = HintList{lm, (int8_t)ord_size_first(totm), false, true};
    if (km == 2) L[nl++] = HintList{0x80000000u, 0, false, false};
  }
  const int r = (int)((gh >> GH_R_SHIFT) & 3u);
  const uint32_t gl = gh & GH_LIST & valid;
  for (int k = 0; k < r; ++k)
    L[nl++] = gl ? HintList{gl, (int8_t)((gh >> GH_MIN_SHIFT) & 7u), false, false} : HintList{0x80000000u, 0, false, false};
  return nl;
}

// GetPodTopologyHints of both providers + Merge: NodeNUMAResource's lists from the row (every position summed), then
// DeviceShare's (gh). *over: see merge_hint_lists_gen.
template <class Src>
__device__ __noinline__ bool hints_merge_gprov(const Src& src, int nz, int policy, bool nil_hints, bool has_cpu,
                                               bool has_mem, int64_t pcpu, int64_t mem, bool tot_c_any, bool tot_m_any,
                                               const Profile& pf, uint32_t gh, bool& aff_has, uint32_t& aff,
                                               bool& over) {
  const uint32_t valid = ord_valid(nz);
  uint32_t totc = 0, totm = 0, lc = 0, lm = 0;
  if (!nil_hints) {
    for (int mi = 0; mi < 15; ++mi) {
      if (!(valid >> mi & 1u)) continue;
      const HintSums s = src.sum(mi);
      if (has_cpu && s.tc >= pcpu) { totc |= 1u << mi; if (s.fc >= pcpu) lc |= 1u << mi; }
      if (has_mem && s.tm >= mem) { totm |= 1u << mi; if (s.fm >= mem) lm |= 1u << mi; }
    }
  }
  HintList L[5];
  const int nl = gen_lists(totc, lc, totm, lm, valid, nil_hints, has_cpu, has_mem, tot_c_any, tot_m_any, gh, L);
  auto score_at = [&](int mi) -> int32_t { return hint_score(src.sum(mi), pcpu, mem, pf); };
  return merge_hint_lists_gen(L, nl, nz, policy, score_at, aff_has, aff, over);
}

// GetPodTopologyHints (topology_hint.go:41-67 -> resource_manager.go:418-532: generateHints for every position,
// total >= request = the size minimum, free >= request = a hint) + merge_hint_lists, one pair per lane. Hint scores
// are evaluated once each when a comparison needs them, packed 7 bits per position.
template <class Src>
__device__ __forceinline__ bool hints_merge(const Src& src, int nz, int policy, bool nil_hints, bool has_cpu,
                                            bool has_mem, int64_t pcpu, int64_t mem, bool tot_c_any, bool tot_m_any,
                                            const Profile& pf, bool& aff_has, uint32_t& aff) {
  const uint32_t valid = ord_valid(nz);
  uint32_t totc = 0, totm = 0, lc = 0, lm = 0;
  if (!nil_hints) {
    auto add = [&](int mi) {
      const HintSums s = src.sum(mi);
      if (s.tc >= pcpu) { totc |= 1u << mi; if (s.fc >= pcpu) lc |= 1u << mi; }
      if (s.tm >= mem) { totm |= 1u << mi; if (s.fm >= mem) lm |= 1u << mi; }
    };
    // The single-zone positions (0..nz-1) first: when each requested resource has a single zone with enough free
    // resources (and one zone has both), merge_hint_lists takes its exact fast path, which reads nothing of the
    // multi-zone positions (it needs min size 1 and the single zones of each list); only otherwise are the other
    // positions summed (> 99.7% of C3's policy pairs stop here).
#pragma unroll 1
    for (int mi = 0; mi < nz; ++mi) add(mi);
    if (!has_cpu) totc = lc = 0;
    if (!has_mem) totm = lm = 0;
    const uint32_t single = (1u << nz) - 1u;
    const bool fast = (has_cpu || has_mem) && (!has_cpu || lc) && (!has_mem || lm) &&
                      ((has_cpu ? lc : single) & (has_mem ? lm : single)) != 0;
    if (!fast) {
#pragma unroll 1
      for (int mi = nz; mi < 15; ++mi)
        if (valid >> mi & 1u) add(mi);
      if (!has_cpu) totc = lc = 0;
      if (!has_mem) totm = lm = 0;
    }
  }
  uint64_t sc_lo = 0, sc_hi = 0;
  uint32_t have = 0;
  auto score_at = [&](int mi) -> int32_t {
    if (!(have >> mi & 1u)) {
      const uint64_t s = (uint64_t)hint_score(src.sum(mi), pcpu, mem, pf);
      if (mi < 9) sc_lo |= s << (7 * mi);
      else sc_hi |= s << (7 * (mi - 9));
      have |= 1u << mi;
    }
    return (int32_t)((mi < 9 ? sc_lo >> (7 * mi) : sc_hi >> (7 * (mi - 9))) & 127u);
  };
  return merge_hint_lists(totc, lc, totm, lm, nz, policy, nil_hints, has_cpu, has_mem, tot_c_any, tot_m_any, score_at,
                          aff_has, aff);
}

// The same for ONE pair evaluated by all 64 lanes of a wave with wave-uniform inputs: lane mi < 15 takes position
// mi (its sums from the row's zone values, compares, hint score), the lists are ballots, and the merge reads
// scores from the lanes. No LDS traffic.
__device__ __forceinline__ bool hints_merge_wave(const HintRegs& h, int nz, int policy, bool nil_hints, bool has_cpu,
                                                 bool has_mem, int64_t pcpu, int64_t mem, bool tot_c_any,
                                                 bool tot_m_any, const Profile& pf, bool& aff_has, uint32_t& aff) {
  const int lane = (int)__lane_id();
  const bool on = !nil_hints && lane < 15 && (ord_valid(nz) >> lane & 1u);
  const HintSums s = h.sum(lane < 15 ? lane : 0);
  const bool tc = on && has_cpu && s.tc >= pcpu, tm = on && has_mem && s.tm >= mem;
  const uint32_t totc = (uint32_t)__ballot(tc), lc = (uint32_t)__ballot(tc && s.fc >= pcpu);
  const uint32_t totm = (uint32_t)__ballot(tm), lm = (uint32_t)__ballot(tm && s.fm >= mem);
  const int32_t sc = on ? hint_score(s, pcpu, mem, pf) : 0;
  auto score_at = [&](int mi) -> int32_t { return __builtin_amdgcn_readlane(sc, mi); };
  return merge_hint_lists(totc, lc, totm, lm, nz, policy, nil_hints, has_cpu, has_mem, tot_c_any, tot_m_any, score_at,
                          aff_has, aff);
}

// One (pod, node) evaluation. do_filter: run Filter (incl. the topology manager Admit that sets the affinity);
// do_score: Score with that affinity (none when the filter is off, as in the reference without a Filter call).
// `alloc[s]`/`free[s]` give NodeInfo.Allocatable / Allocatable-Requested for slots 0..2 and the scalars.
// POLICY_NODES = false compiles only the path of nodes without a NUMA topology policy (the caller routes
// policy nodes to a kernel of their own); such a call on a policy node returns with reason 0 and no score.
// known_aff >= 0: the affinity this pair's Filter produced on the same row state (NumaOut.aff; Reserve of a
// row untouched since the batch-start evaluation): hint generation and merge are skipped.
// TABLE: the row's hint sums come from `table` (the commit kernel), else they are computed from the row's zones.
// WAVE: one pair evaluated by a whole wave with wave-uniform inputs (hints_merge_wave over the row's registers).
// GPROV: the extension path's GPU pods on NUMA-policy nodes: DeviceShare's hints (gh, GH_* above) merged as the
// second provider (hints_merge_gprov); *gh_over reports a merge past its permutation bound.
template <bool POLICY_NODES = true, bool TABLE = false, bool WAVE = false, bool GPROV = false, class Slots>
__device__ __forceinline__ NumaOut numa_eval(const NumaRow& r, const PodVec& p, const Profile& pf, const Slots& sl,
                                             bool do_filter, bool do_score, int known_aff = -1,
                                             const HintTable* table = nullptr, uint32_t gh = 0,
                                             bool* gh_over = nullptr) {
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
  if (!POLICY_NODES) return o;
  const int nz = (nf >> NF_ZONES_SHIFT) & 7;
  if (do_filter && nz == 0) { o.reason = GS_NUMA_MISSING_NUMA_RESOURCES; return o; }
  const ZoneAvail za = zone_avail(r);
  bool aff_has = false;
  uint32_t aff = 0;
  if (do_filter && known_aff >= 0) {
    aff_has = known_aff & 0x10;
    aff = (uint32_t)known_aff & 15u;
  } else if (do_filter) {
    const bool nil_hints = reqflag && topo && !valid;
    const int v = hint_variant(reqflag, bind);
    const bool tca = (nf >> NF_ZCPU_SHIFT) & ((1u << nz) - 1u), tma = (nf >> NF_ZMEM_SHIFT) & ((1u << nz) - 1u);
    bool admit;
    if (GPROV) {
      bool over = false;
      admit = hints_merge_gprov(hint_regs(r, za, v), nz, policy, nil_hints, has_cpu, has_mem, pcpu, mem, tca, tma, pf,
                                gh, aff_has, aff, over);
      if (over && gh_over) *gh_over = true;
    } else if (WAVE) admit = hints_merge_wave(hint_regs(r, za, v), nz, policy, nil_hints, has_cpu, has_mem, pcpu, mem, tca, tma,
                                       pf, aff_has, aff);
    else if (TABLE) admit = hints_merge(HintTableRef{table, v}, nz, policy, nil_hints, has_cpu, has_mem, pcpu, mem, tca, tma,
                                   pf, aff_has, aff);
    else admit = hints_merge(hint_regs(r, za, v), nz, policy, nil_hints, has_cpu, has_mem, pcpu, mem, tca, tma, pf,
                             aff_has, aff);
    if (!admit) { o.reason = GS_NUMA_AFFINITY_ERROR; return o; }
  }
  // resourceManager.Allocate with the affinity (resource_manager.go:171-193)
  bool fail = false;
  if (aff_has) {   // allocateResourcesByHint with the pod's original requests (:195-250)
    int64_t rc = cpu, rm = mem;
    bool ic = false, im = false;
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      if (!(aff >> z & 1u)) continue;
      if (has_cpu && (za.avk >> z & 1u)) {
        ic = true;
        int64_t a = za.av_cpu[z], got = a > rc ? rc : a;
        rc -= got;
        if (got) { o.zkeys |= 1u << z; o.zcpu[z] = got; }
      }
      if (has_mem && (za.avk >> (4 + z) & 1u)) {
        im = true;
        int64_t a = za.av_mem[z], got = a > rm ? rm : a;
        rm -= got;
        if (got) { o.zkeys |= 1u << (4 + z); o.zmem[z] = got; }
      }
    }
    if ((ic && rc != 0) || (im && rm != 0)) fail = true;
  }
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
  if (do_score) {   // calculateAllocatableAndRequested (scoring.go:118-164)
    if (o.zkeys) {
      const uint32_t nf2 = r.nflags2;
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
  return o;
}

}  // namespace gs
