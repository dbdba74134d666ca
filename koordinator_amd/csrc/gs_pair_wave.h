// gs_pair_wave.h — one (pod, node) Filter + Score evaluated by a whole wave, lane-parallel (gfx950).
//
// The commit kernel's selector needs, after every Reserve, the new score of the winner row for the next pod: one
// pair on the critical path of the sequential scheduleOne loop. eval_pair evaluates a pair as one long scalar
// chain (a dozen exact divisions one after the other, the hint scores inside the merge, the final NUMA score
// after Allocate). Here the divisions of the whole pair run as ONE lane-parallel round, each lane holding one
// weighted mean of at most two terms:
//   lanes  0..14  hint score of IterateBitMasks position `lane` (resource_manager.go:454-457)
//   lanes 16..19  NUMA score of a single-zone allocation in zone `lane-16` (scoring.go:118-164)
//   lanes 32..38  Fit LeastAllocated term of slot `lane-32`           ([upstream] resource_allocation.go)
//   lanes 40..41  LoadAware term of cpu / memory                       (load_aware.go:378-397)
//   lanes 48..54  NUMA node-level scorer term of slot `lane-48`         (scoring.go:187-226)
// and the uniform control flow (filters, topology-manager merge, Allocate by hint, cpuset counts) picks the terms.
// Same integer semantics and results as total_score(eval_pair<false, true>(...)) over the LDS row (the commit's
// re-scoring; checked against it on the mirror rows by tests/test_gpu_probe.py and by every commit parity test).
#pragma once
#include "gs_eval_dev.h"

namespace gs {

#ifdef GS_PAIR_PROBE
// diagnostics build (gs_probe.hip): cycle stamps of the evaluation's phases into LDS gs_pw_st[]
__shared__ uint64_t gs_pw_st[8];
#define GS_PW_STAMP(i)                                                              \
  do {                                                                              \
    __builtin_amdgcn_sched_barrier(0);                                              \
    __builtin_amdgcn_s_waitcnt(0);                                                  \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                               \
    if (__lane_id() == 0) gs_pw_st[i] = t_;                                         \
    __builtin_amdgcn_sched_barrier(0);                                              \
  } while (0)
#else
#define GS_PW_STAMP(i) do {} while (0)
#endif

// exact floor(x*100/cap) when ok (0 <= x, cap > 0; the clamping of pct_floor), else 0
__device__ __forceinline__ int32_t pct_or_zero(bool ok, int64_t x, int64_t cap) {
  return ok ? pct_floor(x, cap) : 0;
}

// Filter + Score of (p, r) for the pair (row and pod wave-uniform, in LDS); every lane gets the total score
// (-1: infeasible). m: HBM columns of slots the LDS row does not carry (scalar allocatable).
//
// Written for one wave issuing alone (~4 cycles per instruction, ~50 per dependent LDS read): every LDS field is
// read once up front, the checks of the Filters and of the NUMA prelude are folded into flags instead of early
// exits, and only the rare paths (scalar resources, amplified CPUs, several-zone allocations, the full merge)
// branch.
__device__ __forceinline__ int32_t pair_score_wave(const Row& r, const PodVec& p, const Profile& pf, const MirrorView& m) {
  const int lane = (int)__lane_id();
  const uint32_t en = pf.enabled;
  GS_PW_STAMP(0);
  // ---- every field, read once
  const int64_t f0 = r.free[0], f1 = r.free[1], f2 = r.free[2], a0 = r.alloc[0];
  const int32_t fpods = r.free_pods;
  const uint32_t dfl = r.dflags;
  const int64_t q0 = p.req[0], q1 = p.req[1], q2 = p.req[2];
  const uint32_t pfl = p.flags, smask = p.scalar_mask, pn = p.numa, rkeys = p.req_keys;
  const int32_t ncpus = p.num_cpus;
  const bool numa = en & 0x30u, nfilter = en & 0x10u, nscore = en & 0x20u;
  const NumaRow& nr = r.nr;
  uint32_t nf = 0, nf2 = 0, tfree = 0;
  int32_t alloc_cpus = 0;
  double amp = 0.0, namp = 0.0;
  int64_t zcap_c[4] = {0, 0, 0, 0}, zcap_m[4] = {0, 0, 0, 0}, zraw_c[4] = {0, 0, 0, 0}, zraw_m[4] = {0, 0, 0, 0};
  uint32_t zfree[4] = {0, 0, 0, 0};
  int32_t zadj[4] = {0, 0, 0, 0};
  if (numa) {
    nf = nr.nflags; nf2 = nr.nflags2; tfree = nr.tfree; alloc_cpus = nr.alloc_cpus; amp = nr.amp; namp = nr.namp;
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      zcap_c[z] = nr.zcap_cpu[z]; zcap_m[z] = nr.zcap_mem[z]; zraw_c[z] = nr.zraw_cpu[z]; zraw_m[z] = nr.zraw_mem[z];
      zfree[z] = nr.zfree[z]; zadj[z] = nr.zadj[z];
    }
  }
  // per-lane operands of the Fit (lanes 32..38), LoadAware (40..41) and NUMA node-scorer (48..54) terms: slot k
  const int k = lane & 7;
  const int64_t lf_free = r.free[k < 7 ? k : 0], lf_nzfree = r.nzfree[k & 1], lf_alloc = r.alloc[k & 1];
  const int64_t lp_req = p.req[k < 7 ? k : 0], lp_nz = p.nz[k & 1], lp_est = p.est[k & 1];
  const int64_t l_lacap = r.la_cap[k & 1], l_lafree = (pfl & PF_PROD_SCORE) ? r.la_pfree[k & 1] : r.la_free[k & 1];

  // ---- [upstream] Fit.Filter, LoadAware.Filter
  bool fail = false;
  if (en & 0x1u) {
    fail |= fpods < 1;
    if (!(pfl & PF_ALL_ZERO)) fail |= (q0 > f0) | (q1 > f1) | (q2 > f2);
    if (smask && !(pfl & PF_ALL_ZERO))
      for (int s = 3; s < 7; ++s)
        if ((smask >> s & 1u) && p.req[s] > r.free[s]) fail = true;
  }
  if ((en & 0x4u) && !(pfl & PF_DAEMONSET)) fail |= (dfl & ((pfl & PF_PROD) ? DF_LA_FAIL_P : DF_LA_FAIL_NP)) != 0;
  GS_PW_STAMP(1);

  // ---- NodeNUMAResource prelude (numa_eval), as flags: stop = the plugin returns here (score 0), nfail = with a
  // reason while the filter is on
  bool nstop = !numa, nfail = false;
  bool policy_node = false, rb = false, reqflag = false;
  int bind = BIND_UNSET, nz = 0;
  int64_t cpu = 0, mem = 0, pcpu = 0, rq_cpu_node = 0;
  ZoneAvail za{};
  if (numa) {
    const int policy = (nf >> NF_POLICY_SHIFT) & 3, nbind = (nf >> NF_BIND_SHIFT) & 3;
    cpu = (rkeys & 1u) ? q0 : 0;
    mem = (rkeys & 2u) ? q1 : 0;
    const bool topo = nf & NF_TOPO, valid = nf & NF_TOPO_VALID;
    const int64_t req_cpu = a0 - f0;
    const bool rb0 = pn & PN_BIND;
    const bool implied = !rb0 && cpu != 0 && nbind != 0;   // requestCPUBind (util.go:105-122)
    const bool bad_cpu = implied && cpu % 1000 != 0;
    const bool stopA = (pn & (PN_PREFAIL | PN_SKIP)) || bad_cpu;
    const bool reasonA = (pn & PN_PREFAIL) || bad_cpu;
    rb = rb0 || implied;
    // filterAmplifiedCPUs (plugin.go:340-373)
    bool stopB = false;
    if (nfilter && cpu != 0) {
      if (nf & NF_AMP_INVALID) stopB = true;
      else if (namp > 1.0) {
        const int64_t pm = rb ? amplify_d(cpu, namp) : cpu;
        const int64_t am = (int64_t)alloc_cpus * 1000;
        const int64_t rq = (req_cpu >= am && am > 0) ? req_cpu - am + amplify_d(am, namp) : req_cpu;
        stopB = (topo && !valid) || pm > a0 - rq;
      }
    }
    const int st_req = (pn >> PN_REQ_SHIFT) & 7, st_pref = (pn >> PN_PREF_SHIFT) & 7;
    const int cpc = (nf >> NF_CPC_SHIFT) & 255;
    const int required = nbind == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY ? BIND_FULL
                       : nbind == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS ? BIND_SPREAD : st_req;
    const bool rbfail = nfilter && ((st_req != BIND_UNSET && st_req != required) ||
                                    (required == BIND_FULL && (cpc == 0 || ncpus % cpc != 0)) ||
                                    (required != BIND_UNSET && policy == GS_NUMA_POLICY_NONE &&
                                     cnt_sel(tfree, required, true) < ncpus));
    const bool stopC = rb && (!valid || rbfail);
    nstop = stopA || stopB || stopC;
    nfail = nfilter && (stopA ? reasonA : (stopB || stopC));
    bind = st_req != BIND_UNSET ? st_req : nbind == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS ? BIND_SPREAD
         : nbind == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY ? BIND_FULL : st_pref;
    reqflag = st_req != BIND_UNSET || nbind == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS || nbind == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY;
    const bool ampd = amp > 1.0;
    const int64_t am = (int64_t)alloc_cpus * 1000;
    int64_t amp_cpu = cpu, amp_am = am;
    if (ampd) { amp_cpu = amplify_d(cpu, amp); amp_am = amplify_d(am, amp); }
    pcpu = (rb && cpu != 0) ? amp_cpu : cpu;
    if (policy == GS_NUMA_POLICY_NONE) {
      const bool plain = cpu == 0 || !ampd;
      if (!(nscore && (plain || !(topo && !valid)))) nstop = true;   // score 0 (reason only from above)
      rq_cpu_node = plain ? req_cpu : req_cpu - am + amp_am;
    } else {
      policy_node = true;
      nz = (nf >> NF_ZONES_SHIFT) & 7;
      if (!nstop && nfilter && nz == 0) { nstop = true; nfail = true; }
      rq_cpu_node = rb ? amp_am : req_cpu;
      // zone availability (numa_eval's av_cpu / av_mem / key bits)
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        const bool in = z < nz;
        const bool entry = in && (nf2 >> (NF2_ENTRY_SHIFT + z) & 1u);
        const bool ccpu = in && (nf >> (NF_ZCPU_SHIFT + z) & 1u), cmem = in && (nf >> (NF_ZMEM_SHIFT + z) & 1u);
        const bool acpu = entry && ((nf2 >> (NF2_ACPU_SHIFT + z) & 1u) || ampd);
        const bool amem = entry && (nf2 >> (NF2_AMEM_SHIFT + z) & 1u);
        const int64_t ac = entry ? zraw_c[z] + (ampd ? (int64_t)zadj[z] : 0) : 0;
        const int64_t amz = entry ? zraw_m[z] : 0;
        za.av_cpu[z] = ccpu ? (zcap_c[z] - ac > 0 ? zcap_c[z] - ac : 0) : 0;
        za.av_mem[z] = cmem ? (zcap_m[z] - amz > 0 ? zcap_m[z] - amz : 0) : 0;
        za.avk |= ((ccpu || acpu) ? 1u << z : 0u) | ((cmem || amem) ? 1u << (4 + z) : 0u);
      }
    }
  }
  GS_PW_STAMP(2);

  // ---- the lane round: every weighted mean of the pair in one pass of exact divisions
  const bool do_la = (en & 0x8u) && !(dfl & DF_LA_ZERO);
  const bool do_fit = en & 0x2u;
  const bool lanes_numa = !nstop;
  const int v = hint_variant(reqflag, bind);
  const bool hpos = lane < 15 && lanes_numa && policy_node && (ord_valid(nz) >> (lane & 15) & 1u);
  // hint position sums (lanes 0..14): zones of the position's mask
  HintSums hs{0, 0, 0, 0};
  {
    const uint32_t mk = ord_mask(lane < 15 ? lane : 0);
#pragma unroll
    for (int z = 0; z < 4; ++z) {
      const bool b = mk >> z & 1u;
      hs.tc += (b && (nf >> (NF_ZCPU_SHIFT + z) & 1u)) ? zcap_c[z] : 0;
      hs.tm += (b && (nf >> (NF_ZMEM_SHIFT + z) & 1u)) ? zcap_m[z] : 0;
      hs.fc += b ? trimmed_cpu(za.av_cpu[z], zfree[z], v) : 0;
      hs.fm += b ? za.av_mem[z] : 0;
    }
  }
  // per-lane weighted-mean operands: term A (cpu / the slot) and term B (memory)
  const int grp = lane >> 3;   // 0,1 hints; 2 zones; 4 Fit; 5 LoadAware; 6 NUMA node scorer
  const bool most = grp < 2 ? pf.numa_hint_most : pf.numa_most;
  int64_t capA = 0, reqA = 0, capB = 0, reqB = 0, xA = 0;
  int32_t wA = 0, wB = 0;
  bool lr = false;   // least_requested form (x = free - request, x >= 0) instead of req_score
  if (grp < 2) {         // hint_score (resource_manager.go:454-457): requested = used (floored) + the pod
    if (hpos) {
      capA = hs.tc; reqA = (hs.tc - hs.fc > 0 ? hs.tc - hs.fc : 0) + pcpu; wA = pf.numa_w[0];
      capB = hs.tm; reqB = (hs.tm - hs.fm > 0 ? hs.tm - hs.fm : 0) + mem; wB = pf.numa_w[1];
    }
  } else if (grp == 2) {   // single-zone allocation score (scoring.go:118-164)
    const int z = lane & 3;
    if ((lane & 4) == 0 && lanes_numa && policy_node && z < nz) {
      const bool entry = nf2 >> (NF2_ENTRY_SHIFT + z) & 1u;
      const int64_t zc = z == 0 ? zcap_c[0] : z == 1 ? zcap_c[1] : z == 2 ? zcap_c[2] : zcap_c[3];
      const int64_t zm = z == 0 ? zcap_m[0] : z == 1 ? zcap_m[1] : z == 2 ? zcap_m[2] : zcap_m[3];
      const int64_t rc = z == 0 ? zraw_c[0] : z == 1 ? zraw_c[1] : z == 2 ? zraw_c[2] : zraw_c[3];
      const int64_t rm = z == 0 ? zraw_m[0] : z == 1 ? zraw_m[1] : z == 2 ? zraw_m[2] : zraw_m[3];
      const int32_t ad = z == 0 ? zadj[0] : z == 1 ? zadj[1] : z == 2 ? zadj[2] : zadj[3];
      capA = (nf >> (NF_ZCPU_SHIFT + z) & 1u) ? zc : 0;
      capB = (nf >> (NF_ZMEM_SHIFT + z) & 1u) ? zm : 0;
      reqA = (rb ? rq_cpu_node : (entry ? rc + (amp > 1.0 ? (int64_t)ad : 0) : 0)) + pcpu;
      reqB = (entry ? rm : 0) + mem;
      wA = pf.numa_w[0];
      wB = pf.numa_w[1];
    }
  } else if (grp == 4) {   // Fit LeastAllocated over NonZeroRequested (least_requested)
    if (do_fit && k < 7 && pf.fit_w[k]) {
      lr = true;
      if (k < 2) { capA = lf_alloc; xA = lf_nzfree - lp_nz; wA = pf.fit_w[k]; }
      else if ((pf.fit_scalar_w_mask >> k & 1u) && !(k >= 3 && lp_req == 0)) {
        capA = m.c64(C_ALLOC_CPU + k)[r.node];
        xA = lf_free - lp_req;
        wA = capA != 0 ? pf.fit_w[k] : 0;
      }
    }
  } else if (grp == 5) {   // LoadAware leastRequestedScore over EstimateNode
    if (k < 2 && do_la && pf.la_w[k]) { lr = true; capA = l_lacap; xA = l_lafree - lp_est; wA = pf.la_w[k]; }
  } else if (grp == 6) {   // NUMA node-level scorer (scoring.go:187-226)
    if (k < 7 && lanes_numa && pf.numa_w[k]) {
      const int64_t preq = k == 0 ? pcpu : ((rkeys >> k & 1u) ? lp_req : 0);
      if (!(k >= 3 && preq == 0)) {
        capA = k < 2 ? lf_alloc : m.c64(C_ALLOC_CPU + k)[r.node];
        reqA = (k == 0 ? rq_cpu_node : capA - lf_free) + preq;
        wA = capA != 0 ? pf.numa_w[k] : 0;
      }
    }
  }
  if (capA == 0) wA = 0;
  if (capB == 0) wB = 0;
  // req_score: cap == 0 || (!most && req > cap) -> 0, else pct(most ? min(req, cap) : cap - req)
  // least_requested: cap == 0 || free - p < 0 -> 0, else pct(free - p)
  const bool okA = wA != 0 && (lr ? xA >= 0 : (most || reqA <= capA));
  const bool okB = wB != 0 && (most || reqB <= capB);
  const int64_t nA = lr ? xA : (most ? (reqA > capA ? capA : reqA) : capA - reqA);
  const int64_t nB = most ? (reqB > capB ? capB : reqB) : capB - reqB;
  GS_PW_STAMP(3);
  const int32_t tA = (okA ? pct_floor(nA, capA != 0 ? capA : 1) : 0) * wA;
  const int32_t tB = (okB ? pct_floor(nB, capB != 0 ? capB : 1) : 0) * wB;
  const int32_t ws = wA + wB;
  // per-lane weighted means (hint / zone lanes); the Fit / LoadAware / node terms are summed across lanes
  const int32_t mean = (grp < 4 && ws) ? sdiv(tA + tB, ws) : 0;
  GS_PW_STAMP(4);

  // ---- NodeNUMAResource: merge, Allocate by hint, cpuset counts, the score (uniform)
  int32_t numa_score = 0;
  bool node_scorer = lanes_numa && !policy_node;
  if (lanes_numa && policy_node) {
    const bool has_cpu = rkeys & 1u, has_mem = rkeys & 2u;
    bool aff_has = false;
    uint32_t aff = 0;
    if (nfilter) {
      const int policy = (nf >> NF_POLICY_SHIFT) & 3;
      const bool nil_hints = reqflag && (nf & NF_TOPO) && !(nf & NF_TOPO_VALID);
      const bool tca = (nf >> NF_ZCPU_SHIFT) & ((1u << nz) - 1u), tma = (nf >> NF_ZMEM_SHIFT) & ((1u << nz) - 1u);
      const bool on = !nil_hints && hpos;
      const bool tc = on && has_cpu && hs.tc >= pcpu, tm = on && has_mem && hs.tm >= mem;
      const uint32_t totc = (uint32_t)__ballot(tc), lc = (uint32_t)__ballot(tc && hs.fc >= pcpu);
      const uint32_t totm = (uint32_t)__ballot(tm), lm = (uint32_t)__ballot(tm && hs.fm >= mem);
      auto score_at = [&](int mi) -> int32_t { return __builtin_amdgcn_readlane(mean, mi); };
      if (!merge_hint_lists(totc, lc, totm, lm, nz, policy, nil_hints, has_cpu, has_mem, tca, tma, score_at, aff_has, aff))
        nfail = true;   // GS_NUMA_AFFINITY_ERROR (the filter is on)
    }
    GS_PW_STAMP(5);
    // resourceManager.Allocate with the affinity (resource_manager.go:171-250): zones where an amount is taken
    uint32_t zkeys = 0;
    bool afail = false;
    int64_t zc[4] = {0, 0, 0, 0};
    if (aff_has) {
      int64_t rc = cpu, rm = mem;
      bool ic = false, im = false;
#pragma unroll
      for (int z = 0; z < 4; ++z) {
        if (!(aff >> z & 1u)) continue;
        if (has_cpu && (za.avk >> z & 1u)) {
          ic = true;
          const int64_t got = za.av_cpu[z] > rc ? rc : za.av_cpu[z];
          rc -= got;
          if (got) { zkeys |= 1u << z; zc[z] = got; }
        }
        if (has_mem && (za.avk >> (4 + z) & 1u)) {
          im = true;
          const int64_t got = za.av_mem[z] > rm ? rm : za.av_mem[z];
          rm -= got;
          if (got) zkeys |= 1u << (4 + z);
        }
      }
      afail = (ic && rc != 0) || (im && rm != 0);
    }
    if (!afail && rb) {   // allocateCPUSet, counted
      const int cpc = (nf >> NF_CPC_SHIFT) & 255;
      afail = cnt_sel(tfree, bind, reqflag) < ncpus || (!zkeys && reqflag && bind == BIND_FULL && cpc && ncpus % cpc);
      if (!afail && zkeys) {
        int sum = 0;
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          if (!((zkeys >> z & 1u) || (zkeys >> (4 + z) & 1u))) continue;
          const int avail = cnt_sel(zfree[z], bind, reqflag);
          const int want = (int)(zc[z] / 1000);
          const int n = want < avail ? want : avail;
          if (reqflag && bind == BIND_FULL && cpc && n % cpc) afail = true;
          sum += n;
        }
        if (sum != ncpus) afail = true;
      }
    }
    if (afail) {
      nfail |= nfilter;   // GS_NUMA_ADMIT_ALLOCATE_FAILED; score 0 without the filter
    } else if (nscore && zkeys) {
      const uint32_t zones = (zkeys | (zkeys >> 4)) & 15u;
      if (__popc(zones) == 1) {
        numa_score = __builtin_amdgcn_readlane(mean, 16 + __ffs(zones) - 1);
      } else {   // several zones: calculateAllocatableAndRequested over their sums (scoring.go:118-164)
        int64_t ac = 0, am2 = 0, rqc = 0, rqm = 0;
#pragma unroll
        for (int z = 0; z < 4; ++z) {
          if (!(zones >> z & 1u)) continue;
          if (nf >> (NF_ZCPU_SHIFT + z) & 1u) ac += zcap_c[z];
          if (nf >> (NF_ZMEM_SHIFT + z) & 1u) am2 += zcap_m[z];
          if (nf2 >> (NF2_ENTRY_SHIFT + z) & 1u) {
            rqc += zraw_c[z] + (amp > 1.0 ? (int64_t)zadj[z] : 0);
            rqm += zraw_m[z];
          }
        }
        if (rb) rqc = rq_cpu_node;
        int32_t ns = 0, wsum = 0;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const int32_t w = pf.numa_w[s];
          if (!w) continue;
          const int64_t al = s == 0 ? ac : am2;
          if (al == 0) continue;
          ns += req_score(pf.numa_most, (s == 0 ? rqc : rqm) + (s == 0 ? pcpu : mem), al) * w;
          wsum += w;
        }
        numa_score = wsum ? sdiv(ns, wsum) : 0;
      }
    } else if (nscore) {
      node_scorer = true;   // no zone taken: the node-level scorer
    }
  }
  GS_PW_STAMP(6);
  // ---- lane-summed means: Fit (lanes 32..38), LoadAware (40..41), node scorer (48..54)
  const int32_t fit_n = wave_sum(grp == 4 ? tA : 0), fit_w = wave_sum(grp == 4 ? wA : 0);
  const int32_t la_n = wave_sum(grp == 5 ? tA : 0);
  if (node_scorer) {
    const int32_t n_n = wave_sum(grp == 6 ? tA : 0), n_w = wave_sum(grp == 6 ? wA : 0);
    numa_score = n_w ? sdiv(n_n, n_w) : 0;
  }
  const int32_t fit = (do_fit && fit_w) ? small_div(fit_n, fit_w) : 0;
  const int32_t la = do_la ? small_div(la_n, pf.la_wsum) : 0;
  GS_PW_STAMP(7);
  if (fail || nfail) return -1;
  return fit * pf.w_fit + la * pf.w_la + (numa ? numa_score : 0) * pf.w_numa;
}

}  // namespace gs
