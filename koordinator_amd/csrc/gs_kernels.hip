// gs_kernels.hip — CDNA4 (gfx950) kernels of the batched Filter/Score engine.
//
//   node_prep_kernel   per batch, O(N): LoadAware expiry against `now` -> dynamic filter/score flags
//   eval_kernel        the hot kernel: (node tile x pod group) workgroups, fused Fit filter + LoadAware
//                      filter + Fit LeastAllocated score + LoadAware score + weighted sum -> int16 rows
//   cand_kernel        per pod: per-wave histograms -> top score levels -> order-preserving compaction of
//                      every node of those levels (node index order) -> LevelHdr + level lists
//   commit_kernel      one workgroup: the batch's pods in order — selectHost over (listed levels of every
//                      shard, minus/plus the rows earlier pods of the batch landed on, re-scored exactly),
//                      then assume/Reserve deltas; cuts the batch if a pod's levels are exhausted
//   row_stats_kernel / row_select_kernel   exact full-row path (a level too large to list)
//   scatter_rows_kernel   host -> HBM delta rows (AoS staging -> SoA columns)
//
// Integer semantics follow Go: int64 two's complement, truncating division. The float64 spots of the
// reference (LoadAware filter %, estimator scaling) are host-side per node / per pod; per-pair work here is
// int64 with an exact reciprocal-estimate-plus-correction division (quotients lie in [0,100]).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <cstdio>
#include <vector>

#include "gs_eval_dev.h"
#include "gs_pair_wave.h"

namespace gs {

// ------------------------------------------------------------------------------------------------
// node-prep: LoadAware expiry (helper.go:36-41) evaluated at `now` for every node.
// idx != nullptr: the n0..n1 entries of idx (rows a delta update just rewrote) instead of a node range
__device__ __forceinline__ uint32_t node_prep_flags(uint32_t sf, int64_t update_time, int64_t now, int32_t filter_expired,
                                                    int32_t has_exp, int64_t exp_ns) {
  bool exists = sf & SF_METRIC;
  bool expired = !exists || !(sf & SF_UPDATE_TIME) || (exp_ns > 0 && now - update_time >= exp_ns);
  bool skip_filter = !exists || (filter_expired && has_exp && expired);
  uint32_t df = 0;
  if (!skip_filter) {
    const uint32_t npd = ((sf & SF_NP_MEM) ? 1u : 0u) | ((sf & SF_NP_AGG) ? 2u : 0u);   // reason details
    if (sf & SF_FAIL_NP) df |= DF_LA_FAIL_NP | npd << DF_NP_DETAIL_SHIFT;
    if (sf & SF_PROD_THR) {
      if (sf & SF_FAIL_P) df |= DF_LA_FAIL_P | (((sf & SF_P_MEM) ? 1u : 0u) << DF_P_DETAIL_SHIFT);
    } else if (sf & SF_FAIL_NP) {
      df |= DF_LA_FAIL_P | npd << DF_P_DETAIL_SHIFT;
    }
  }
  if (!exists || (has_exp && expired)) df |= DF_LA_ZERO;
  return df;
}

__global__ void __launch_bounds__(256) node_prep_kernel(MirrorView m, uint32_t n0, uint32_t n1, int64_t now,
                                                        int32_t filter_expired, int32_t has_exp, int64_t exp_ns,
                                                        const uint32_t* __restrict__ idx) {
  uint32_t i = n0 + blockIdx.x * 256 + threadIdx.x;
  if (i >= n1) return;
  if (idx) i = idx[i];
  m.c32(C_DFLAGS)[i] = (int32_t)node_prep_flags((uint32_t)m.c32(C_SFLAGS)[i], m.c64(C_UPDATE_TIME)[i], now,
                                                filter_expired, has_exp, exp_ns);
}

// ------------------------------------------------------------------------------------------------
// The hot kernel. Workgroup = 256 consecutive nodes of the shard x PODS_PER_BLOCK pods. Each thread keeps
// its node row in registers and sweeps the group's pods (wave-uniform pod vectors: scalar loads), writing
// one int16 score per (pod, node): one coalesced 512-B row segment per pod per workgroup.
template <bool NUMA>
__global__ void __launch_bounds__(256) eval_kernel(MirrorView m, const PodVec* __restrict__ pods, int npods,
                                                   Profile pf, uint32_t n0, uint32_t n1, int16_t* __restrict__ S,
                                                   uint32_t ld, int prod_cols) {
  const uint32_t local = blockIdx.x * 256 + threadIdx.x;
  const uint32_t len = n1 - n0;
  const bool ok = local < len;
  Row row;
  load_row(m, ok ? n0 + local : n0, prod_cols, NUMA, row);
  if (!NUMA) pf.enabled &= ~0x30u;
  // nodes with a NUMA topology policy are evaluated by eval_numa_kernel (compacted, divergence-free)
  if (NUMA && ok && ((row.nr.nflags >> NF_POLICY_SHIFT) & 3u)) return;
  const int k0 = blockIdx.y * PODS_PER_BLOCK;
  const int k1 = min(npods, k0 + PODS_PER_BLOCK);
  for (int k = k0; k < k1; ++k) {
    PairOut o = eval_pair<false, false, false>(row, pods[k], pf, m);
    S[(size_t)k * ld + local] = ok ? (int16_t)total_score(o, pf) : (int16_t)-1;
  }
}

// The NUMA-topology-policy nodes of the shard (host-maintained ascending index list): hints over zone subsets,
// the topology-manager merge, Allocate by hint. A thread keeps one node row in registers and evaluates PPT
// consecutive pods of the batch: the row (gathered through the index list, ~30% of the shard's lines) is read
// once per PPT pods instead of once per pair, while a full batch still puts ~nidx*B/PPT threads in flight.
// sv.i64 != nullptr: the rows come from the batch's slab (gather_numa_kernel: entry t = node idx[t], dense columns).
template <int PPT>
__global__ void __launch_bounds__(256) eval_numa_kernel(MirrorView m, MirrorView sv, const PodVec* __restrict__ pods,
                                                        int npods, Profile pf, const uint32_t* __restrict__ idx,
                                                        uint32_t nidx, uint32_t n0, int16_t* __restrict__ S, uint32_t ld,
                                                        int prod_cols, uint8_t* __restrict__ aff) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  const int k0 = blockIdx.y * PPT;
  if (t >= nidx || k0 >= npods) return;
  const int k1 = min(npods, k0 + PPT);
  const uint32_t node = idx[t];
  Row row;
  if (sv.i64) {
    load_row(sv, t, prod_cols, true, row);
    row.node = node;   // (eval_pair reads the scalar-slot columns of the mirror by node)
  } else {
    load_row(m, node, prod_cols, true, row);
  }
  for (int k = k0; k < k1; ++k) {
    PairOut o = eval_pair<false, false, true>(row, pods[k], pf, m);
    S[(size_t)k * ld + (node - n0)] = (int16_t)total_score(o, pf);
    aff[(size_t)k * ld + (node - n0)] = (uint8_t)(o.code ? 0u : o.aff);   // read by the commit's Reserve
  }
}

// Tiled form (the default for full batches, PPT 8): a workgroup is a tile of 64 policy rows x NUMA_TWAVES * PPT pods; lane
// = row, wave w = pods [w * PPT, (w + 1) * PPT) of the workgroup's pod range. The waves of a workgroup read the same
// rows (one fetch from HBM, three cache hits), and the workgroups of one tile are numbered so they land on one XCD
// (blocks go round-robin over the 8 XCDs: id % 8 = tile % 8) and are dispatched together (ids of 8 consecutive tiles x
// every pod range form one run of ids), so each tile leaves HBM about once per pass instead of once per pod group
// (round 4: ~26 reads of the slab per pass, 140 MB for a 4.6 MB slab at C3). ntiles8: tiles rounded up to 8.
constexpr int NUMA_TWAVES = 4;
template <int PPT>
__global__ void __launch_bounds__(64 * NUMA_TWAVES) eval_numa_tile_kernel(MirrorView m, MirrorView sv,
                                                                          const PodVec* __restrict__ pods, int npods,
                                                                          Profile pf, const uint32_t* __restrict__ idx,
                                                                          uint32_t nidx, uint32_t n0, int16_t* __restrict__ S,
                                                                          uint32_t ld, int prod_cols,
                                                                          uint8_t* __restrict__ aff, uint32_t npr,
                                                                          int xcd_map) {
  const uint32_t id = blockIdx.x;
  uint32_t pr, tile;
  if (xcd_map) {
    const uint32_t grp = id / (8u * npr), rem = id % (8u * npr);
    pr = rem / 8u;
    tile = grp * 8u + rem % 8u;
  } else {
    pr = id % npr;
    tile = id / npr;
  }
  const uint32_t t = tile * 64u + (threadIdx.x & 63u);
  const int w = threadIdx.x >> 6;
  const int k0 = (int)pr * (NUMA_TWAVES * PPT) + w * PPT;
  if (t >= nidx || k0 >= npods) return;
  const int k1 = min(npods, k0 + PPT);
  const uint32_t node = idx[t];
  Row row;
  if (sv.i64) {
    load_row(sv, t, prod_cols, true, row);
    row.node = node;
  } else {
    load_row(m, node, prod_cols, true, row);
  }
  for (int k = k0; k < k1; ++k) {
    PairOut o = eval_pair<false, false, true>(row, pods[k], pf, m);
    S[(size_t)k * ld + (node - n0)] = (int16_t)total_score(o, pf);
    aff[(size_t)k * ld + (node - n0)] = (uint8_t)(o.code ? 0u : o.aff);
  }
}

// The NUMA-policy rows of the batch's eval pass gathered into a dense slab (same column numbering, entry t = node
// idx[t]): eval_numa_kernel then reads each row once per pod group from whole cache lines instead of the ~30% of every
// line the ascending index list uses in the mirror (the gather reads the sparse lines once per batch).
__constant__ int kSlabCol64[] = {C_FREE_CPU,  C_FREE_MEM,  C_FREE_EPH,  C_ALLOC_CPU, C_ALLOC_MEM, C_NZFREE_CPU,
                                 C_NZFREE_MEM, C_LA_CAP_CPU, C_LA_CAP_MEM, C_LA_FREE_CPU, C_LA_FREE_MEM,
                                 C_LA_PFREE_CPU, C_LA_PFREE_MEM, C_ZCAP_CPU0, C_ZCAP_CPU0 + 1, C_ZCAP_CPU0 + 2,
                                 C_ZCAP_CPU0 + 3, C_ZCAP_MEM0, C_ZCAP_MEM0 + 1, C_ZCAP_MEM0 + 2, C_ZCAP_MEM0 + 3,
                                 C_ZRAW_CPU0, C_ZRAW_CPU0 + 1, C_ZRAW_CPU0 + 2, C_ZRAW_CPU0 + 3, C_ZRAW_MEM0,
                                 C_ZRAW_MEM0 + 1, C_ZRAW_MEM0 + 2, C_ZRAW_MEM0 + 3, C_AMP, C_NAMP};
__constant__ int kSlabCol32[] = {C_FREE_PODS, C_DFLAGS, C_ZFREE0, C_ZFREE0 + 1, C_ZFREE0 + 2, C_ZFREE0 + 3, C_ZADJ0,
                                 C_ZADJ0 + 1, C_ZADJ0 + 2, C_ZADJ0 + 3, C_NFLAGS, C_NFLAGS2, C_ALLOC_CPUS, C_TFREE};
constexpr int SLAB64 = 31, SLAB32 = 14;
__global__ void __launch_bounds__(256) gather_numa_kernel(MirrorView m, MirrorView sv, const uint32_t* __restrict__ idx,
                                                          uint32_t nidx) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= nidx) return;
  const uint32_t node = idx[t];
  const int c = blockIdx.y;
  if (c < SLAB64) sv.c64(kSlabCol64[c])[t] = m.c64(kSlabCol64[c])[node];
  else sv.c32(kSlabCol32[c - SLAB64])[t] = m.c32(kSlabCol32[c - SLAB64])[node];
}

// Patch of a batch's score rows evaluated concurrently with the previous batch's commit (which writes the rows
// its pods landed on back to HBM at its end): the previous batch's winner rows of this shard are evaluated again,
// on their committed state, for every pod of this batch (same pair evaluation as eval_kernel / eval_numa_kernel).
// Block k: the row pod k of the previous batch landed on.
__global__ void __launch_bounds__(128) patch_kernel(MirrorView m, const PodVec* __restrict__ pods, int npods, Profile pf,
                                                     uint32_t n0, uint32_t n1, int16_t* __restrict__ S, uint32_t ld,
                                                     int prod_cols, uint8_t* __restrict__ aff,
                                                     const PlacementDev* __restrict__ prev_out,
                                                     const int32_t* __restrict__ prev_committed) {
  const int k = blockIdx.x;
  if (k >= prev_committed[0]) return;   // pods the previous batch placed (a voided pass: -1)
  const int32_t node = prev_out[k].node;
  if (node < 0 || (uint32_t)node < n0 || (uint32_t)node >= n1) return;
  const bool numa = (pf.enabled & 0x30u) != 0;
  // the row once per block (scalar slots included), and for a NUMA-policy row its hint table (the sums of every
  // zone subset, built by 60 lanes), which every pod of the batch then reads instead of recomputing the hints
  __shared__ Row s_row;
  __shared__ HintTable s_tab;
  if (threadIdx.x == 0) {
    load_row(m, (uint32_t)node, prod_cols, numa, s_row);
    for (int sl = 3; sl < 7; ++sl) s_row.free[sl] = m.c64(C_FREE_CPU + sl)[node];
  }
  __syncthreads();
  const bool policy = numa && ((s_row.nr.nflags >> NF_POLICY_SHIFT) & 3u);
  if (policy && threadIdx.x < 64) hint_table_fill(s_tab, s_row.nr, zone_avail(s_row.nr), (int)threadIdx.x);
  __syncthreads();
  const Row r = s_row;
  for (int q = threadIdx.x; q < npods; q += 128) {
    const PairOut o = eval_pair<false, true, true, true>(r, pods[q], pf, m, &s_tab);
    S[(size_t)q * ld + ((uint32_t)node - n0)] = (int16_t)total_score(o, pf);
    if (policy) aff[(size_t)q * ld + ((uint32_t)node - n0)] = (uint8_t)(o.code ? 0u : o.aff);
  }
}

// The same patch with one wave per (row, pod) pair, lane-parallel (pair_score_wave): the kernel's time is the
// slowest pair's, and a pair evaluated by one lane runs the rare long paths (the full topology-manager merge) as one
// scalar chain, while a wave spreads them over its lanes. Block = one landed row x PW_PODS pods. The Filter-time
// affinity of a patched NUMA-policy row is left to the Reserve (AFF_RECOMPUTE: numa_eval recomputes it there).
constexpr int PW_PODS = 16;
__global__ void __launch_bounds__(64 * PW_PODS) patch_wave_kernel(MirrorView m, const PodVec* __restrict__ pods,
                                                                  int npods, Profile pf, uint32_t n0, uint32_t n1,
                                                                  int16_t* __restrict__ S, uint32_t ld, int prod_cols,
                                                                  uint8_t* __restrict__ aff,
                                                                  const PlacementDev* __restrict__ prev_out,
                                                                  const int32_t* __restrict__ prev_committed) {
  const int k = blockIdx.x;
  if (k >= prev_committed[0]) return;   // pods the previous batch placed (a voided pass: -1)
  const int32_t node = prev_out[k].node;
  if (node < 0 || (uint32_t)node < n0 || (uint32_t)node >= n1) return;
  const bool numa = (pf.enabled & 0x30u) != 0;
  __shared__ Row s_row;
  __shared__ PodVec s_pod[PW_PODS];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = blockIdx.y * PW_PODS + w;
  if (threadIdx.x == 0) {
    load_row(m, (uint32_t)node, prod_cols, numa, s_row);
    for (int sl = 3; sl < 7; ++sl) s_row.free[sl] = m.c64(C_FREE_CPU + sl)[node];
  }
  if (q < npods && lane < (int)(sizeof(PodVec) / 8))
    reinterpret_cast<uint64_t*>(&s_pod[w])[lane] = reinterpret_cast<const uint64_t*>(&pods[q])[lane];
  __syncthreads();
  if (q >= npods) return;
  const int32_t sc = pair_score_wave(s_row, s_pod[w], pf, m);
  if (lane == 0) {
    S[(size_t)q * ld + ((uint32_t)node - n0)] = (int16_t)sc;
    if (numa && ((s_row.nr.nflags >> NF_POLICY_SHIFT) & 3u)) aff[(size_t)q * ld + ((uint32_t)node - n0)] = AFF_RECOMPUTE;
  }
}

// Diagnostic variant (gs_evaluate): every plugin's verdict and score for every pair.
__global__ void __launch_bounds__(256) eval_full_kernel(MirrorView m, const PodVec* __restrict__ pods, int npods,
                                                        Profile pf, uint32_t N, int16_t* scores, uint16_t* codes,
                                                        int16_t* plugin, int prod_cols) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  Row r;
  load_row(m, i, prod_cols, (pf.enabled & 0x30u) != 0, r);
  for (int k = 0; k < npods; ++k) {
    PairOut o = eval_pair<true, false>(r, pods[k], pf, m);
    size_t off = (size_t)k * N + i;
    if (scores) scores[off] = (int16_t)total_score(o, pf);
    if (codes) codes[off] = (uint16_t)o.code;
    if (plugin) {
      plugin[off * 3 + 0] = (int16_t)o.fit;
      plugin[off * 3 + 1] = (int16_t)o.la;
      plugin[off * 3 + 2] = (int16_t)o.numa;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Candidate levels: one workgroup (W waves) per pod row of the shard; wave w owns a contiguous W-th of the
// row so that per-wave histograms give every wave its output offset within each level. W = 16 for profiles
// with small score ranges (more bandwidth per row when batches are short), else 4.
template <int W>
__global__ void __launch_bounds__(64 * W) cand_kernel(int16_t* __restrict__ S, uint32_t ld, uint32_t len,
                                                      uint32_t n0, int max_score, int lcap, uint32_t* __restrict__ lists,
                                                      LevelHdr* __restrict__ hdrs, LevelExt* __restrict__ ext,
                                                      uint64_t* stamps, CandPatch cp) {
  constexpr int CAND_THREADS = 64 * W;
  // diagnostics (stamps != nullptr): wave 0's cycles per phase, summed over the pods
  uint64_t ct_last = stamps ? __builtin_amdgcn_s_memtime() : 0;
  auto CT = [&](int i) {
    if (!stamps) return;
    const uint64_t t_ = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&stamps[i]), (unsigned long long)(t_ - ct_last));
    ct_last = t_;
  };
  extern __shared__ __align__(16) uint32_t smem[];
  const int nbins = max_score + 1;
  uint32_t* whist = smem;                                        // [W][nbins]
  uint32_t* comb = smem + W * nbins;                             // [nbins]
  int8_t* slot_of = reinterpret_cast<int8_t*>(comb + nbins);     // [nbins]
  __shared__ uint32_t segsum[CAND_THREADS];
  __shared__ uint32_t s_total;
  __shared__ int32_t s_nlev, s_next, s_score[LEVALL], s_count[LEVALL];
  __shared__ uint32_t s_woff[W][LEVALL];
  constexpr int STEPCAP = 128;                 // 512-entry steps per wave with a recorded maximum
  __shared__ int16_t s_stepmax[W][STEPCAP];    // highest score of each of the wave's steps (pass 2 skips the rest)
  const int k = blockIdx.x;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  if (cp.on) {
    // the patch of this pod's score row (patch_kernel's work, one pair per thread): the rows the previous batch landed
    // on, on their committed state; the histogram below then reads them (this block's row only: no other block
    // writes it)
    const bool numa = (cp.pf.enabled & 0x30u) != 0;
    const int np = cp.prev_committed[0];   // -1: a voided pass
    for (int j = t; j < np; j += CAND_THREADS) {
      const int32_t node = cp.prev_out[j].node;
      if (node < 0 || (uint32_t)node < cp.n0 || (uint32_t)node >= cp.n1) continue;
      Row r;
      load_row(cp.m, (uint32_t)node, cp.prod_cols, numa, r);
      const PairOut o = eval_pair<false, false, true>(r, cp.pods[k], cp.pf, cp.m);
      const size_t at = (size_t)k * ld + ((uint32_t)node - cp.n0);
      S[at] = (int16_t)total_score(o, cp.pf);
      if (numa && ((r.nr.nflags >> NF_POLICY_SHIFT) & 3u)) cp.aff[at] = (uint8_t)(o.code ? 0u : o.aff);
    }
    __threadfence_block();
    __syncthreads();
  }
  const int16_t* row = S + (size_t)k * ld;
  for (int b = t; b < W * nbins; b += CAND_THREADS) whist[b] = 0;
  if (t == 0) s_total = 0;
  __syncthreads();
  // 16-B loads: 8 scores per lane, 512 per wave step. Rows are padded with -1 up to ld (a multiple of
  // 1024), so the row is read as lenv = round_up(len, 512) entries.
  const uint32_t lenv = (len + 511) & ~511u;
  const uint32_t seg = (lenv / 512 + W - 1) / W * 512;
  const uint32_t wb = min(lenv, wave * seg), we = min(lenv, wb + seg);
  const int4* row4 = reinterpret_cast<const int4*>(row);
  // pass 1: per-wave histograms of feasible scores; 4 loads in flight per lane, the next group's loads issued
  // before this group's atomics (the pass is load-latency bound: one workgroup streams a whole row)
  auto load4 = [&](uint32_t i, int4 (&q)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = i + u * 512 < we ? row4[(i + u * 512) / 8] : make_int4(-1, -1, -1, -1);
  };
  int4 qn[4];
  load4(wb + lane * 8, qn);
  for (uint32_t i = wb + lane * 8; i < we; i += 4 * 512) {
    int4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = qn[u];
    if (i + 4 * 512 < we) load4(i + 4 * 512, qn);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int16_t* e = reinterpret_cast<const int16_t*>(&q[u]);
      int mx = -1;
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        if (e[x] >= 0) atomicAdd(&whist[wave * nbins + e[x]], 1u);
        mx = max(mx, (int)e[x]);
      }
      mx = wave_max(mx);
      const uint32_t st = (i - lane * 8 + u * 512 - wb) / 512;
      if (lane == 0 && st < (uint32_t)STEPCAP) s_stepmax[wave][st] = (int16_t)mx;
    }
  }
  __syncthreads();
  CT(0);
  const int per = (nbins + CAND_THREADS - 1) / CAND_THREADS;
  {
    uint32_t s = 0;
    for (int b = t * per; b < min(nbins, (t + 1) * per); ++b) {
      uint32_t h = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) h += whist[w * nbins + b];
      comb[b] = h;
      if (cp.hist) cp.hist[(size_t)k * nbins + b] = h;
      slot_of[b] = -1;
      s += h;
    }
    segsum[t] = s;
    if (s) atomicAdd(&s_total, s);
  }
  __syncthreads();
  CT(1);
  if (wave == 0) {
    // levels from the top until the pod's position in the batch is covered: pod k can find at most k of
    // the listed nodes dirtied by earlier pods, so k+1 listed nodes always leave a clean one. Wave 0 walks the
    // bins 64 at a time from the top (lane l: bin hi - l); a level stops the list when the levels before it are
    // LEVALL, or it would pass lcap (LCAP; XCAP when the lists are all-gathered), or the nodes before it cover the
    // target.
    const uint32_t target = (uint32_t)k + 1 + (uint32_t)cp.extra;
    const uint64_t lt = (1ull << lane) - 1ull;
    int nlev = 0, next = -1;
    uint32_t cum = 0;
    for (int hi = nbins - 1; hi >= 0; hi -= 64) {
      const int b = hi - lane;
      const uint32_t c = b >= 0 ? comb[b] : 0u;
      const bool nz = c != 0;
      const uint64_t nzm = __ballot(nz);
      if (!nzm) continue;
      const uint32_t cb = cum + (uint32_t)(wave_incl_scan((int)c) - (int)c);
      const int nb = nlev + __popcll(nzm & lt);
      const bool stop = nz && (nb == LEVALL || cb + c > (uint32_t)lcap || cb >= target);
      const uint64_t sm = __ballot(stop);
      const int ls = sm ? __builtin_ctzll(sm) : 64;
      if (nz && lane < ls) {
        s_score[nb] = b;
        s_count[nb] = (int32_t)c;
        slot_of[b] = (int8_t)nb;
      }
      if (sm) {
        next = __builtin_amdgcn_readlane(b, ls);
        nlev += __popcll(nzm & ((1ull << ls) - 1ull));
        break;
      }
      nlev += __popcll(nzm);
      cum += (uint32_t)wave_sum((int)c);
    }
    for (int j = nlev + lane; j < LEVALL; j += 64) { s_score[j] = -1; s_count[j] = 0; }
    if (lane == 0) {
      s_nlev = nlev;
      s_next = next;
    }
  }
  __syncthreads();
  CT(2);
  const int nlev = s_nlev;
  for (int e = t; e < W * LEVALL; e += CAND_THREADS) {
    const int w = e / LEVALL, j = e % LEVALL;
    uint32_t off = 0;
    if (j < nlev) {
      for (int jj = 0; jj < j; ++jj) off += s_count[jj];
      for (int ww = 0; ww < w; ++ww) off += whist[ww * nbins + s_score[j]];
    }
    s_woff[w][j] = off;
  }
  __syncthreads();
  CT(3);
  // pass 2: order-preserving compaction of the listed levels (node order = (lane, element) order), level by level
  // over the levels present in each 512-node step
  uint32_t* out = lists + (size_t)k * lcap;
  if (nlev > 0) {
    uint32_t run_l = lane < LEVALL ? s_woff[wave][lane] : 0;   // level `lane`'s next output position (this wave)
    // steps whose highest score is below the lowest listed level hold no listed node: not read again
    const int thr = s_score[nlev - 1];
    auto next_step = [&](uint32_t b) {
      for (; b < we; b += 512) {
        const uint32_t st = (b - wb) / 512;
        if (st >= (uint32_t)STEPCAP || s_stepmax[wave][st] >= thr) break;
      }
      return b;
    };
    // the next 3 steps' loads are in flight while a step is scanned
    constexpr int PD = 4;
    uint32_t bq[PD];
    int4 vq[PD];
    uint32_t nb = next_step(wb);
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      bq[u] = nb;
      vq[u] = nb < we ? row4[(nb + lane * 8) / 8] : make_int4(-1, -1, -1, -1);
      nb = nb < we ? next_step(nb + 512) : we;
    }
    while (bq[0] < we) {
      const uint32_t base = bq[0];
      const int4 q = vq[0];
#pragma unroll
      for (int u = 0; u + 1 < PD; ++u) { bq[u] = bq[u + 1]; vq[u] = vq[u + 1]; }
      bq[PD - 1] = nb;
      vq[PD - 1] = nb < we ? row4[(nb + lane * 8) / 8] : make_int4(-1, -1, -1, -1);
      nb = nb < we ? next_step(nb + 512) : we;
      const int16_t* e = reinterpret_cast<const int16_t*>(&q);
      int slot[8];
      uint32_t present = 0;
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        slot[x] = e[x] >= thr ? slot_of[e[x]] : -1;   // every non-empty bin >= thr is a listed level
        if (slot[x] >= 0) present |= 1u << slot[x];
      }
      // levels present anywhere in the step (OR over the wave)
      uint32_t pw = (uint32_t)wave_or((int)present);
      for (; pw; pw &= pw - 1) {
        const int j = __ffs(pw) - 1;
        int c = 0;
#pragma unroll
        for (int x = 0; x < 8; ++x) c += slot[x] == j;
        const int incl = wave_incl_scan(c);
        int pos = __builtin_amdgcn_readlane((int)run_l, j) + incl - c;
#pragma unroll
        for (int x = 0; x < 8; ++x)
          if (slot[x] == j) out[pos++] = n0 + base + lane * 8 + x;
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        if (lane == j) run_l += tot;
      }
    }
  }
  CT(4);
  if (t == 0) {
    LevelHdr h;
    h.nlev = nlev < MAXLEV ? nlev : MAXLEV;
    h.feasible = (int32_t)s_total;
    h.next = nlev > MAXLEV ? s_score[MAXLEV] : s_next;
    int32_t tot = 0;
    for (int j = 0; j < MAXLEV; ++j) { h.score[j] = s_score[j]; h.count[j] = s_count[j]; tot += s_count[j]; }
    h.total = tot;
    hdrs[k] = h;
    LevelExt x;
    x.nlev = nlev;
    x.next = s_next;
    for (int j = 0; j < LEVX; ++j) { x.score[j] = s_score[MAXLEV + j]; x.count[j] = s_count[MAXLEV + j]; }
    ext[k] = x;
  }
}

// ------------------------------------------------------------------------------------------------
// Candidate levels of a short batch (a few pods over a long row, the plain runs between C5's extension pods):
// cand_kernel streams each row from one CU (33 us at 100k nodes, LDS-atomic bound). Here every row is cut into G
// slices spread over the chip: cs_hist_kernel histograms each (slice, pod), cs_pick_kernel (one block per pod) sums
// them, picks the levels as cand_kernel's wave 0 does and gives every slice its output position within each level,
// and cs_list_kernel compacts each slice in node order. The lists, headers and extensions equal cand_kernel's (the
// plain case: no patch, no stale-level margin).
__global__ void __launch_bounds__(256) cs_hist_kernel(const int16_t* __restrict__ S, uint32_t ld, uint32_t lenv,
                                                      int nbins, uint32_t slice, int G, uint32_t* __restrict__ ghist) {
  extern __shared__ __align__(16) uint32_t hist[];
  const int g = blockIdx.x, k = blockIdx.y, t = threadIdx.x;
  for (int b = t; b < nbins; b += 256) hist[b] = 0;
  __syncthreads();
  const uint32_t b0 = (uint32_t)g * slice, b1 = min(lenv, b0 + slice);
  const int4* row4 = reinterpret_cast<const int4*>(S + (size_t)k * ld);
  for (uint32_t i = b0 + t * 8; i < b1; i += 2 * 2048) {
    const int4 q0 = row4[i / 8];
    const int4 q1 = i + 2048 < b1 ? row4[(i + 2048) / 8] : make_int4(-1, -1, -1, -1);
    const int16_t* e0 = reinterpret_cast<const int16_t*>(&q0);
    const int16_t* e1 = reinterpret_cast<const int16_t*>(&q1);
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      if (e0[x] >= 0) atomicAdd(&hist[e0[x]], 1u);
      if (e1[x] >= 0) atomicAdd(&hist[e1[x]], 1u);
    }
  }
  __syncthreads();
  uint32_t* out = ghist + ((size_t)k * G + g) * nbins;
  for (int b = t; b < nbins; b += 256) out[b] = hist[b];
}

__global__ void __launch_bounds__(256) cs_pick_kernel(const uint32_t* __restrict__ ghist, int nbins, int G, int lcap,
                                                      uint32_t* __restrict__ offs, LevelHdr* __restrict__ hdrs,
                                                      LevelExt* __restrict__ ext) {
  extern __shared__ __align__(16) uint32_t comb[];   // [nbins]
  __shared__ uint32_t s_total;
  __shared__ int32_t s_nlev, s_next, s_score[LEVALL], s_count[LEVALL];
  __shared__ uint32_t s_v[CS_GMAX][LEVALL];
  const int k = blockIdx.x, t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const uint32_t* h = ghist + (size_t)k * G * nbins;
  for (int b = t; b < nbins; b += 256) comb[b] = 0;
  if (t == 0) s_total = 0;
  __syncthreads();
  // the slice histograms are contiguous: entry e is bin e % nbins of slice e / nbins
  const int tot = G * nbins;
  for (int e0 = t; e0 < tot; e0 += 4 * 256) {
    uint32_t v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = e0 + u * 256 < tot ? h[e0 + u * 256] : 0u;
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (v[u]) atomicAdd(&comb[(e0 + u * 256) % nbins], v[u]);
  }
  __syncthreads();
  {
    uint32_t s = 0;
    for (int b = t; b < nbins; b += 256) s += comb[b];
    s = (uint32_t)wave_sum((int)s);
    if (lane == 0 && s) atomicAdd(&s_total, s);
  }
  if (wave == 0) {   // cand_kernel's level pick (target k + 1)
    const uint32_t target = (uint32_t)k + 1;
    const uint64_t lt = (1ull << lane) - 1ull;
    int nlev = 0, next = -1;
    uint32_t cum = 0;
    for (int hi = nbins - 1; hi >= 0; hi -= 64) {
      const int b = hi - lane;
      const uint32_t c = b >= 0 ? comb[b] : 0u;
      const bool nz = c != 0;
      const uint64_t nzm = __ballot(nz);
      if (!nzm) continue;
      const uint32_t cb = cum + (uint32_t)(wave_incl_scan((int)c) - (int)c);
      const int nb = nlev + __popcll(nzm & lt);
      const bool stop = nz && (nb == LEVALL || cb + c > (uint32_t)lcap || cb >= target);
      const uint64_t sm = __ballot(stop);
      const int ls = sm ? __builtin_ctzll(sm) : 64;
      if (nz && lane < ls) {
        s_score[nb] = b;
        s_count[nb] = (int32_t)c;
      }
      if (sm) {
        next = __builtin_amdgcn_readlane(b, ls);
        nlev += __popcll(nzm & ((1ull << ls) - 1ull));
        break;
      }
      nlev += __popcll(nzm);
      cum += (uint32_t)wave_sum((int)c);
    }
    for (int j = nlev + lane; j < LEVALL; j += 64) { s_score[j] = -1; s_count[j] = 0; }
    if (lane == 0) {
      s_nlev = nlev;
      s_next = next;
    }
  }
  __syncthreads();
  const int nlev = s_nlev;
  // each slice's node count at each listed level, then per level the running start over the slices
  for (int e = t; e < G * LEVALL; e += 256) {
    const int g = e / LEVALL, j = e % LEVALL;
    s_v[g][j] = j < nlev ? h[(size_t)g * nbins + s_score[j]] : 0u;
  }
  __syncthreads();
  if (t < LEVALL) {
    uint32_t base = 0;
    for (int jj = 0; jj < t && jj < nlev; ++jj) base += (uint32_t)s_count[jj];
    uint32_t* o = offs + (size_t)k * G * LEVALL;
    for (int g = 0; g < G; ++g) {
      o[g * LEVALL + t] = base;
      base += s_v[g][t];
    }
  }
  if (t == 0) {
    LevelHdr hd;
    hd.nlev = nlev < MAXLEV ? nlev : MAXLEV;
    hd.feasible = (int32_t)s_total;
    hd.next = nlev > MAXLEV ? s_score[MAXLEV] : s_next;
    int32_t sum = 0;
    for (int j = 0; j < MAXLEV; ++j) { hd.score[j] = s_score[j]; hd.count[j] = s_count[j]; sum += s_count[j]; }
    hd.total = sum;
    hdrs[k] = hd;
    LevelExt x;
    x.nlev = nlev;
    x.next = s_next;
    for (int j = 0; j < LEVX; ++j) { x.score[j] = s_score[MAXLEV + j]; x.count[j] = s_count[MAXLEV + j]; }
    ext[k] = x;
  }
}

__global__ void __launch_bounds__(64) cs_list_kernel(const int16_t* __restrict__ S, uint32_t ld, uint32_t lenv,
                                                     uint32_t n0, int nbins, uint32_t slice, int G, int lcap,
                                                     const uint32_t* __restrict__ offs,
                                                     const LevelHdr* __restrict__ hdrs,
                                                     const LevelExt* __restrict__ ext, uint32_t* __restrict__ lists) {
  extern __shared__ __align__(16) int8_t slot_of[];   // [nbins]: bin -> listed level, -1 none
  const int g = blockIdx.x, k = blockIdx.y, lane = threadIdx.x;
  const int nlev = ext[k].nlev;
  if (nlev <= 0) return;
  for (int b = lane; b < nbins; b += 64) slot_of[b] = -1;
  __syncthreads();
  int sc = -1;
  if (lane < nlev) sc = lane < MAXLEV ? hdrs[k].score[lane] : ext[k].score[lane - MAXLEV];
  if (lane < nlev) slot_of[sc] = (int8_t)lane;
  const int thr = __shfl(sc, nlev - 1);
  __syncthreads();
  uint32_t run_l = lane < LEVALL ? offs[((size_t)k * G + g) * LEVALL + lane] : 0u;
  uint32_t* out = lists + (size_t)k * lcap;
  const uint32_t b0 = (uint32_t)g * slice, b1 = min(lenv, b0 + slice);
  const int4* row4 = reinterpret_cast<const int4*>(S + (size_t)k * ld);
  for (uint32_t gb = b0; gb < b1; gb += 4 * 512) {
    int4 qs[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      qs[u] = gb + u * 512 < b1 ? row4[(gb + u * 512 + lane * 8) / 8] : make_int4(-1, -1, -1, -1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t base = gb + u * 512;
      const int16_t* e = reinterpret_cast<const int16_t*>(&qs[u]);
      int slot[8];
      uint32_t present = 0;
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        slot[x] = e[x] >= thr ? slot_of[e[x]] : -1;   // every non-empty bin >= thr is a listed level
        if (slot[x] >= 0) present |= 1u << slot[x];
      }
      uint32_t pw = (uint32_t)wave_or((int)present);
      for (; pw; pw &= pw - 1) {
        const int j = __ffs(pw) - 1;
        int c = 0;
#pragma unroll
        for (int x = 0; x < 8; ++x) c += slot[x] == j;
        const int incl = wave_incl_scan(c);
        int pos = __builtin_amdgcn_readlane((int)run_l, j) + incl - c;
#pragma unroll
        for (int x = 0; x < 8; ++x)
          if (slot[x] == j) out[pos++] = n0 + base + lane * 8 + x;
        const int tot = __builtin_amdgcn_readlane(incl, 63);
        if (lane == j) run_l += tot;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Stale levels fixed up once the previous batch has committed:cand_kernel ran beside that batch's commit on rows whose
// landed nodes ("prev rows") still held their pre-commit scores, listing cp.extra nodes beyond pod k's k+1 and writing
// its histogram. Block k (pod k): re-evaluate the prev rows on their committed state (S, aff patched), move them in the
// histogram, and re-pick the levels from the top down. A score above the stale `next` is fully known: every non-prev
// node there is in the stale lists (levels are whole), every prev node is here; so the new levels stop at the first
// bin at or below the stale `next`, which is then the new `next` (exact: from the updated histogram). Each new level's
// nodes: its stale segment minus the prev rows, merged (node order) with the prev rows whose new score it is.
constexpr int FIX_THREADS = 256;
__device__ __forceinline__ int lower_bound_u32(const uint32_t* a, int n, uint32_t x) {
  int lo = 0;
  while (n > 0) {
    const int h = n >> 1;
    if (a[lo + h] < x) { lo += h + 1; n -= h + 1; } else { n = h; }
  }
  return lo;
}
__global__ void __launch_bounds__(FIX_THREADS) fix_levels_kernel(int16_t* __restrict__ S, uint32_t ld, int max_score,
                                                                 int lcap, uint32_t* __restrict__ lists,
                                                                 LevelHdr* __restrict__ hdrs, LevelExt* __restrict__ ext,
                                                                 CandPatch cp, uint64_t* stamps) {
  // diagnostics (stamps != nullptr): thread 0's cycles per phase, summed over the pods (entries 5..7 of the cand stamps)
  uint64_t ct_last = stamps ? __builtin_amdgcn_s_memtime() : 0;
  auto CT = [&](int i) {
    if (!stamps) return;
    const uint64_t t_ = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&stamps[i]), (unsigned long long)(t_ - ct_last));
    ct_last = t_;
  };
  extern __shared__ __align__(16) uint32_t smem[];
  const int nbins = max_score + 1;
  uint32_t* hist = smem;                 // [nbins] the row's histogram, prev rows moved
  uint32_t* olist = smem + nbins;        // [lcap] the stale listed nodes
  __shared__ uint32_t p_raw[MAX_BATCH], p_node[MAX_BATCH];   // prev rows (raw order; distinct, ascending)
  __shared__ int32_t p_old[MAX_BATCH], p_new[MAX_BATCH];
  __shared__ unsigned long long m_old[LEVALL][2], m_new[LEVALL][2];
  __shared__ int32_t n_ol[LEVALL];
  __shared__ int32_t o_score[LEVALL], o_count[LEVALL], o_off[LEVALL];
  __shared__ int32_t n_score[LEVALL], n_count[LEVALL], n_off[LEVALL];
  __shared__ int32_t s_onlev, s_onext, s_ofeas, s_np, s_fd, s_nlev, s_next, s_top;
  __shared__ int32_t r_old[MAX_BATCH], r_new[MAX_BATCH], p_sidx[MAX_BATCH];   // per raw entry; raw index by rank
  __shared__ int32_t s_wd[2];
  int8_t* lev_of = reinterpret_cast<int8_t*>(olist + lcap);   // [nbins] bin -> new level (-1: not listed)
  const int k = blockIdx.x, t = threadIdx.x, lane = t & 63;
  // the landed node of entry t (cp.extra = the previous batch's size bounds its placements) loads beside the count
  const int32_t node_t = t < cp.extra ? cp.prev_out[t].node : -1;
  const int npr = min(cp.prev_committed[0], MAX_BATCH);   // -1: a voided pass (its lists are never used)
  if (npr <= 0) return;
  __shared__ unsigned int s_ev_max[2];   // diagnostics: the block's slowest lane (row loads, row loads + evaluation)
  if (stamps && t < 2) s_ev_max[t] = 0;
  if (stamps) __syncthreads();
  // phase 1 (no barrier): the evaluation of the landed rows is the long chain (row loads ~15k cycles, then one pair
  // evaluation, ~26k for the slowest lane of a wave whose rows differ), so waves 0-1 do only that: thread j < npr
  // evaluates landed entry j (duplicates too: a node several pods landed on gives the same result each time; its stale
  // score is read here, before any entry's write below). Beside it wave 3 reads the stale levels and stages the stale
  // lists in LDS, and wave 2 the histogram (their HBM round trips overlap the evaluation).
  static_assert(FIX_THREADS == 256 && MAX_BATCH <= 128, "fix_levels_kernel: waves 0-1 evaluate, 2-3 load");
  if (t >= FIX_THREADS - 64) {   // the stale levels: one lane per level (independent loads), offsets by a wave scan
    const LevelHdr& h = hdrs[k];
    const LevelExt& x = ext[k];
    const int onl = x.nlev;
    const int j = lane;
    int sc = -1, cnt = 0;
    if (j < LEVALL) {
      sc = j < MAXLEV ? h.score[j] : x.score[j - MAXLEV];
      cnt = j < onl ? (j < MAXLEV ? h.count[j] : x.count[j - MAXLEV]) : 0;
    }
    const int incl = wave_incl_scan(cnt);
    if (j < LEVALL) {
      o_score[j] = sc;
      o_count[j] = cnt;
      o_off[j] = incl - cnt;
    }
    if (lane == 0) {
      s_onlev = onl;
      s_onext = x.next;
      s_ofeas = h.feasible;
      s_fd = 0;
      s_top = onl > 0 ? h.score[0] : x.next;   // the highest non-empty bin before the landed rows move
    }
    // the stale lists into LDS (8 loads in flight per lane)
    const int otot = onl > 0 ? __shfl(incl, onl - 1) : 0;
    const uint32_t* src = lists + (size_t)k * lcap;
    for (int e0 = 0; e0 < otot; e0 += 8 * 64) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 64 + lane;
        v[u] = e < otot ? src[e] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int e = e0 + u * 64 + lane;
        if (e < otot) olist[e] = v[u];
      }
    }
  } else if (t >= FIX_THREADS - 128) {
    for (int b = lane; b < nbins; b += 64) hist[b] = cp.hist[(size_t)k * nbins + b];
  }
  const bool numa = (cp.pf.enabled & 0x30u) != 0;
  size_t at = 0;
  int so = -1, sn = -1, aff_v = -1;
  bool valid = false;
  if (t < npr) {
    const int32_t node = node_t;
    valid = node >= 0 && (uint32_t)node >= cp.n0 && (uint32_t)node < cp.n1;
    p_raw[t] = valid ? (uint32_t)node : 0xffffffffu;
    if (valid) {
      const uint64_t e0 = stamps ? __builtin_amdgcn_s_memtime() : 0;
      if (stamps && t == 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(&stamps[10]), (unsigned long long)(e0 - ct_last));
      at = (size_t)k * ld + ((uint32_t)node - cp.n0);
      so = S[at];
      Row r;
      load_row(cp.m, (uint32_t)node, cp.prod_cols, numa, r);
      if (stamps) {
        __builtin_amdgcn_s_waitcnt(0);
        atomicMax(&s_ev_max[0], (unsigned int)(__builtin_amdgcn_s_memtime() - e0));
      }
      const PairOut o = eval_pair<false, false, true>(r, cp.pods[k], cp.pf, cp.m);
      sn = total_score(o, cp.pf);
      if (numa && ((r.nr.nflags >> NF_POLICY_SHIFT) & 3u)) aff_v = o.code ? 0 : (int)o.aff;
      if (stamps) atomicMax(&s_ev_max[1], (unsigned int)(__builtin_amdgcn_s_memtime() - e0));
    }
    r_old[t] = so;
    r_new[t] = sn;
  }
  __syncthreads();
  if (stamps && t == 0) {
    atomicAdd(reinterpret_cast<unsigned long long*>(&stamps[8]), (unsigned long long)s_ev_max[0]);
    atomicAdd(reinterpret_cast<unsigned long long*>(&stamps[9]), (unsigned long long)s_ev_max[1]);
    atomicAdd(reinterpret_cast<unsigned long long*>(&stamps[11]),
              (unsigned long long)(__builtin_amdgcn_s_memtime() - ct_last));   // kernel start -> every lane evaluated
  }
  // phase 2: landed entries ranked by (node, index). The patched scores go out at the end of the kernel: vmcnt counts
  // stores too, and the compiler's vmcnt(0) before the ranking made the stores' round trip part of the chain
  if (t < 128) {   // waves 0-1: the 128 keys in two registers per lane, compared through readlane (no LDS per key)
    const uint32_t x = t < npr ? p_raw[t] : 0u;
    const uint32_t k0 = lane < npr ? p_raw[lane] : 0u, k1 = 64 + lane < npr ? p_raw[64 + lane] : 0u;
    int rank = 0;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      const uint32_t y0 = __builtin_amdgcn_readlane(k0, i), y1 = __builtin_amdgcn_readlane(k1, i);
      rank += (i < npr && (y0 < x || (y0 == x && i < t))) ? 1 : 0;
      rank += (64 + i < npr && (y1 < x || (y1 == x && 64 + i < t))) ? 1 : 0;
    }
    if (t < npr) p_sidx[rank] = t;
  }
  __syncthreads();
  // the first entry of each node, in node order: the distinct landed rows, moved in the histogram
  bool keep = false;
  int idx = 0, wpre = 0;
  uint32_t xs = 0;
  if (t < 2 * 64) {
    if (t < npr) {
      idx = p_sidx[t];
      xs = p_raw[idx];
      keep = xs != 0xffffffffu && (t == 0 || p_raw[p_sidx[t - 1]] != xs);
    }
    const uint64_t m = __ballot(keep);
    wpre = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wd[t >> 6] = __popcll(m);
  }
  __syncthreads();
  if (keep) {
    const int pos = (t >= 64 ? s_wd[0] : 0) + wpre;
    const int o_ = r_old[idx], n_ = r_new[idx];
    p_node[pos] = xs;
    p_old[pos] = o_;
    p_new[pos] = n_;
    if (o_ >= 0) atomicSub(&hist[o_], 1u);
    if (n_ >= 0) atomicAdd(&hist[n_], 1u);
    const int fd = (n_ >= 0 ? 1 : 0) - (o_ >= 0 ? 1 : 0);
    if (fd) atomicAdd(&s_fd, fd);
    atomicMax(&s_top, n_);
  }
  if (t == 0) s_np = s_wd[0] + s_wd[1];
  __syncthreads();
  CT(5);
  const int np = s_np;
  if (t < 64) {
    // levels from the top (cand_kernel's rule for pod k: k+1 nodes, LEVALL levels, lcap nodes), known bins only
    const uint32_t target = (uint32_t)k + 1;
    const int onext = s_onext;
    const uint64_t lt = (1ull << lane) - 1ull;
    int nlev = 0, next = -1;
    uint32_t cum = 0;
    for (int hi = min(s_top, nbins - 1); hi >= 0; hi -= 64) {
      const int b = hi - lane;
      const uint32_t c = b >= 0 ? hist[b] : 0u;
      const bool nz = c != 0;
      const uint64_t nzm = __ballot(nz);
      if (!nzm) continue;
      const uint32_t cb = cum + (uint32_t)(wave_incl_scan((int)c) - (int)c);
      const int nb = nlev + __popcll(nzm & lt);
      const bool stop = nz && (nb == LEVALL || cb + c > (uint32_t)lcap || cb >= target || b <= onext);
      const uint64_t sm = __ballot(stop);
      const int ls = sm ? __builtin_ctzll(sm) : 64;
      if (nz && lane < ls) {
        n_score[nb] = b;
        n_count[nb] = (int32_t)c;
      }
      if (sm) {
        next = __builtin_amdgcn_readlane(b, ls);
        nlev += __popcll(nzm & ((1ull << ls) - 1ull));
        break;
      }
      nlev += __popcll(nzm);
      cum += (uint32_t)wave_sum((int)c);
    }
    for (int j = nlev + lane; j < LEVALL; j += 64) { n_score[j] = -1; n_count[j] = 0; }
    WAVE_FENCE();
    const int cnt = lane < LEVALL ? n_count[lane] : 0;
    if (lane < LEVALL) n_off[lane] = wave_incl_scan(cnt) - cnt;
    if (lane == 0) {
      s_nlev = nlev;
      s_next = next;
    }
  }
  __syncthreads();
  CT(6);
  const int nlev = s_nlev;
  // per new level j: the prev rows (bit i = p_node[i], node order) whose stale / new score is its score, and the stale
  // level of the same score (-1: none); a bin -> new level map
  for (int b = t; b < nbins; b += FIX_THREADS) lev_of[b] = -1;
  if (t < LEVALL * 2) { m_old[t >> 1][t & 1] = 0; m_new[t >> 1][t & 1] = 0; }
  __syncthreads();
  if (t < nlev) {
    lev_of[n_score[t]] = (int8_t)t;
    int o = -1;
    for (int i = 0; i < s_onlev; ++i) o = o_score[i] == n_score[t] ? i : o;
    n_ol[t] = o;
  }
  __syncthreads();
  if (t < np) {
    const int jo = p_old[t] >= 0 ? lev_of[p_old[t]] : -1, jn = p_new[t] >= 0 ? lev_of[p_new[t]] : -1;
    if (jo >= 0) atomicOr(&m_old[jo][t >> 6], 1ull << (t & 63));
    if (jn >= 0) atomicOr(&m_new[jn][t >> 6], 1ull << (t & 63));
  }
  __syncthreads();
  auto below = [](const unsigned long long (&m)[2], int pos) {   // bits < pos
    const int lo = min(pos, 64), hi = max(pos - 64, 0);
    return __popcll(lo >= 64 ? m[0] : (m[0] & ((1ull << lo) - 1ull))) +
           __popcll(hi >= 64 ? m[1] : (m[1] & ((1ull << hi) - 1ull)));
  };
  uint32_t* out = lists + (size_t)k * lcap;
  const int onlev = s_onlev;
  const int otot = onlev > 0 ? o_off[onlev - 1] + o_count[onlev - 1] : 0;
  // stale entries of a still-listed level, not prev rows: after the kept entries and the new prev rows of a smaller
  // node at their level
  for (int e = t; e < otot; e += FIX_THREADS) {
    int oj = 0;   // the stale level holding entry e: last o_off <= e
    for (int step = 16; step; step >>= 1)
      if (oj + step < onlev && o_off[oj + step] <= e) oj += step;
    const int j = lev_of[o_score[oj]];
    if (j < 0) continue;
    const uint32_t x = olist[e];
    const int pos = lower_bound_u32(p_node, np, x);
    if (pos < np && p_node[pos] == x) continue;
    out[n_off[j] + (e - o_off[oj]) - below(m_old[j], pos) + below(m_new[j], pos)] = x;
  }
  // prev rows at a listed level: after the new prev rows and the kept stale entries of a smaller node
  if (t < np) {
    const int sn = p_new[t];
    const int j = sn >= 0 ? lev_of[sn] : -1;
    if (j >= 0) {
      const int oj = n_ol[j];
      const int before = oj >= 0 ? lower_bound_u32(olist + o_off[oj], o_count[oj], p_node[t]) - below(m_old[j], t) : 0;
      out[n_off[j] + below(m_new[j], t) + before] = p_node[t];
    }
  }
  CT(7);
  if (t == 0) {
    LevelHdr h;
    h.nlev = nlev < MAXLEV ? nlev : MAXLEV;
    h.feasible = s_ofeas + s_fd;
    h.next = nlev > MAXLEV ? n_score[MAXLEV] : s_next;
    int32_t tot = 0;
    for (int j = 0; j < MAXLEV; ++j) { h.score[j] = n_score[j]; h.count[j] = n_count[j]; tot += n_count[j]; }
    h.total = tot;
    hdrs[k] = h;
    LevelExt x;
    x.nlev = nlev;
    x.next = s_next;
    for (int j = 0; j < LEVX; ++j) { x.score[j] = n_score[MAXLEV + j]; x.count[j] = n_count[MAXLEV + j]; }
    ext[k] = x;
  }
  if (valid) {   // the patched scores and Filter-time affinities of the landed rows
    S[at] = (int16_t)sn;
    if (aff_v >= 0) cp.aff[at] = (uint8_t)aff_v;
  }
}

// ------------------------------------------------------------------------------------------------
// Several shards: the all-gathered candidate levels of every shard merged into ONE block of the single-rank layout, so
// that the speculative commit runs over one list per pod as on one shard. Kept: the distinct scores above every shard's
// `next` (each such level is complete on every shard), in descending order, while they fit LEVALL levels and LCAP
// nodes; a level's nodes in shard order, i.e. node order (shards are contiguous ranges, each shard's level segment is
// ascending). The merged `next` is the highest score not kept (every shard's `next`, or the first dropped level).
// Block k = pod k; thread e = (shard e / LEVALL, level e % LEVALL).
// Several ranks, score-row exchange: rank r evaluated its shard [r*per, min(N, (r+1)*per)) into the block layout of
// launch_unpack_scores (gs_kernels.h); here the R all-gathered blocks become the batch's full-width score rows and
// Filter-time affinities, so every rank continues with the one-shard pipeline over the whole cluster. Grid: (pld/256,
// npods, R). Block (0, 0, 0) checks the blocks' exchange tags as merge_levels_kernel does.
__global__ void __launch_bounds__(256) unpack_scores_kernel(const uint8_t* __restrict__ xin, size_t xblock, int R,
                                                            int npods, uint32_t per, uint32_t pld, uint32_t N,
                                                            int16_t* __restrict__ S, uint8_t* __restrict__ aff,
                                                            uint32_t ld, int32_t* __restrict__ xerr) {
  const int r = blockIdx.z, k = blockIdx.y;
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (r == 0 && k == 0 && blockIdx.x == 0 && threadIdx.x == 0) {
    const XTag* t0 = reinterpret_cast<const XTag*>(xin + xblock - sizeof(XTag));
    int bad = 0;
    for (int q = 0; q < R && !bad; ++q) {
      const XTag* tq = reinterpret_cast<const XTag*>(xin + (size_t)q * xblock + xblock - sizeof(XTag));
      if (tq->magic != XTAG_MAGIC || tq->site != t0->site || tq->seq != t0->seq || tq->batch != t0->batch ||
          tq->rank != q || tq->bytes != (uint32_t)xblock)
        bad = 1 + q;
    }
    xerr[0] = bad;
    if (bad && !xerr[1]) {
      xerr[1] = 1;
      uint32_t* dst = reinterpret_cast<uint32_t*>(xerr + XERR_TAGS);
      for (int q = 0; q < R; ++q) {
        const uint32_t* tq = reinterpret_cast<const uint32_t*>(xin + (size_t)q * xblock + xblock - sizeof(XTag));
        for (int w = 0; w < (int)(sizeof(XTag) / 4); ++w) dst[q * (sizeof(XTag) / 4) + w] = tq[w];
      }
    }
  }
  const uint32_t node = (uint32_t)r * per + i;
  if (i >= per || node >= N) return;
  const uint8_t* blk = xin + (size_t)r * xblock;
  S[(size_t)k * ld + node] = reinterpret_cast<const int16_t*>(blk)[(size_t)k * pld + i];
  aff[(size_t)k * ld + node] = blk[(size_t)npods * pld * 2 + (size_t)k * pld + i];
}

hipError_t launch_unpack_scores(const uint8_t* xin, size_t xblock, int nranks, int npods, uint32_t per, uint32_t pld,
                                uint32_t N, int16_t* S, uint8_t* aff, uint32_t ld, int32_t* xerr, hipStream_t st) {
  if (npods <= 0 || nranks <= 0) return hipSuccess;
  hipLaunchKernelGGL(unpack_scores_kernel, dim3((per + 255) / 256, npods, nranks), dim3(256), 0, st, xin, xblock,
                     nranks, npods, per, pld, N, S, aff, ld, xerr);
  return hipGetLastError();
}

__global__ void __launch_bounds__(256) merge_levels_kernel(const uint8_t* __restrict__ xin, size_t xblock, int R,
                                                           int bmax, int lstride, uint8_t* __restrict__ xout,
                                                           int32_t* __restrict__ xerr) {
  constexpr int NEMAX = MAX_RANKS * LEVALL;
  static_assert(NEMAX <= 256, "one thread per shard level");
  __shared__ int32_t e_score[NEMAX], e_count[NEMAX], e_rep[NEMAX];
  __shared__ int32_t s_next[MAX_RANKS], s_feas[MAX_RANKS];
  __shared__ int32_t m_score[LEVALL], m_count[LEVALL];
  __shared__ int32_t s_nlev, s_drop;
  const int k = blockIdx.x, t = threadIdx.x, NE = R * LEVALL;
  if (k == 0 && t == 0) {   // the blocks' exchange tags: every rank sent the same exchange of the sequence
    const XTag* t0 = reinterpret_cast<const XTag*>(xin + xblock - sizeof(XTag));
    int bad = 0;
    for (int r = 0; r < R && !bad; ++r) {
      const XTag* tr = reinterpret_cast<const XTag*>(xin + (size_t)r * xblock + xblock - sizeof(XTag));
      if (tr->magic != XTAG_MAGIC || tr->site != t0->site || tr->seq != t0->seq || tr->batch != t0->batch ||
          tr->rank != r || tr->bytes != (uint32_t)xblock)
        bad = 1 + r;
    }
    xerr[0] = bad;
    // the first mismatch's tags, kept for the host's report (the blocks themselves are overwritten by the next
    // exchange, which a stream-ordered transport has enqueued before the host reads this batch's verdict)
    if (bad && !xerr[1]) {
      xerr[1] = 1;
      uint32_t* dst = reinterpret_cast<uint32_t*>(xerr + XERR_TAGS);
      for (int r = 0; r < R; ++r) {
        const uint32_t* tr = reinterpret_cast<const uint32_t*>(xin + (size_t)r * xblock + xblock - sizeof(XTag));
        for (int w = 0; w < (int)(sizeof(XTag) / 4); ++w) dst[r * (sizeof(XTag) / 4) + w] = tr[w];
      }
    }
  }
  // rank blocks: lists at lstride entries per pod; the merged block has the single-rank layout (LCAP per pod)
  const size_t ihoff = (size_t)bmax * lstride * 4, ixoff = ihoff + (size_t)bmax * sizeof(LevelHdr);
  const size_t hoff = (size_t)bmax * LCAP * 4, xoff = hoff + (size_t)bmax * sizeof(LevelHdr);
  if (t == 0) { s_nlev = 0; s_drop = -1; }
  if (t < LEVALL) { m_score[t] = -1; m_count[t] = 0; }
  int off = 0;   // this level's offset in its shard's list
  if (t < NE) {
    const int r = t / LEVALL, j = t % LEVALL;
    const LevelHdr* h = reinterpret_cast<const LevelHdr*>(xin + r * xblock + ihoff) + k;
    const LevelExt* x = reinterpret_cast<const LevelExt*>(xin + r * xblock + ixoff) + k;
    const int nl = x->nlev;
    int s = -1, c = 0;
    if (j < nl) {
      s = j < MAXLEV ? h->score[j] : x->score[j - MAXLEV];
      c = j < MAXLEV ? h->count[j] : x->count[j - MAXLEV];
    }
    e_score[t] = s;
    e_count[t] = c;
    if (j == 0) { s_next[r] = x->next; s_feas[r] = h->feasible; }
  }
  __syncthreads();
  int mnext = -1, feas = 0;
  for (int r = 0; r < R; ++r) { mnext = max(mnext, s_next[r]); feas += s_feas[r]; }
  int s = -1;
  if (t < NE) {
    s = e_score[t];
    const int r = t / LEVALL, j = t % LEVALL;
    for (int jj = 0; jj < j; ++jj) off += e_count[r * LEVALL + jj];
    bool rep = s > mnext;   // the first shard holding score s represents its merged level
    for (int u = 0; u < t && rep; ++u) rep = e_score[u] != s;
    e_rep[t] = rep;
  }
  __syncthreads();
  int pos = -1;
  if (t < NE && s > mnext) {

    int rank = 0, cum = 0, before = 0, tot = 0;
    for (int u = 0; u < NE; ++u) {
      const int su = e_score[u];
      if (su > s) { cum += e_count[u]; rank += e_rep[u]; }
      else if (su == s) { tot += e_count[u]; if (u < t) before += e_count[u]; }
    }
    if (rank < LEVALL && cum + tot <= LCAP) {
      pos = cum + before;
      if (e_rep[t]) { m_score[rank] = s; m_count[rank] = tot; atomicAdd(&s_nlev, 1); }
    } else if (e_rep[t]) {
      atomicMax(&s_drop, s);
    }
  }
  __syncthreads();
  // the kept levels' nodes: entry by entry, every thread copying
  uint32_t* out = reinterpret_cast<uint32_t*>(xout) + (size_t)k * LCAP;
  __shared__ int32_t s_pos[NEMAX], s_off[NEMAX];
  if (t < NE) { s_pos[t] = pos; s_off[t] = off; }
  __syncthreads();
  for (int u = 0; u < NE; ++u) {
    const int pu = s_pos[u];
    if (pu < 0) continue;
    const uint32_t* in = reinterpret_cast<const uint32_t*>(xin + (u / LEVALL) * xblock) + (size_t)k * lstride + s_off[u];
    const int cu = e_count[u];
    for (int x = t; x < cu; x += 256) out[pu + x] = in[x];
  }
  if (t == 0) {
    const int nlev = s_nlev, next = max(mnext, s_drop);
    LevelHdr h;
    h.nlev = nlev < MAXLEV ? nlev : MAXLEV;
    h.feasible = feas;
    h.next = nlev > MAXLEV ? m_score[MAXLEV] : next;
    int32_t tot = 0;
    for (int j = 0; j < MAXLEV; ++j) { h.score[j] = m_score[j]; h.count[j] = m_count[j]; tot += m_count[j]; }
    h.total = tot;
    reinterpret_cast<LevelHdr*>(xout + hoff)[k] = h;
    LevelExt x;
    x.nlev = nlev;
    x.next = next;
    for (int j = 0; j < LEVX; ++j) { x.score[j] = m_score[MAXLEV + j]; x.count[j] = m_count[MAXLEV + j]; }
    reinterpret_cast<LevelExt*>(xout + xoff)[k] = x;
  }
}

hipError_t launch_merge_levels(const uint8_t* xin, size_t xblock, int nranks, int npods, int bmax, int lstride,
                               uint8_t* xout, int32_t* xerr, hipStream_t st) {
  if (npods <= 0) return hipSuccess;
  if (nranks < 2 || nranks > MAX_RANKS || lstride > LCAP || nranks * lstride > LCAP) return hipErrorInvalidValue;
  if (xblock < sizeof(XTag) || xblock % 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(merge_levels_kernel, dim3(npods), dim3(256), 0, st, xin, xblock, nranks, bmax, lstride, xout,
                     xerr);
  return hipGetLastError();
}

__global__ void write_tag_kernel(uint8_t* __restrict__ dst, XTag t) {
  if (threadIdx.x == 0) *reinterpret_cast<XTag*>(dst) = t;
}

hipError_t launch_write_tag(uint8_t* dst, const XTag& t, hipStream_t st) {
  if (reinterpret_cast<uintptr_t>(dst) % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(write_tag_kernel, dim3(1), dim3(64), 0, st, dst, t);
  return hipGetLastError();
}

int64_t host_tiebreak_position(uint64_t seed, uint64_t seq, int64_t T) { return tiebreak_position(seed, seq, T); }

// selectHost tie-break lookup of the speculative commit (tiebreak_records + the lane-parallel count in
// gs_commit_spec.hip tb_pos) against tiebreak_position, on the host: random (seed, seq) and T at, around and
// between the records, the records' limit and beyond it. Returns the number of mismatches.
extern "C" int gsx_tiebreak_selftest(uint64_t seed, int iters, char* msg, size_t len) {
  uint64_t st = seed * 0x9E3779B97F4A7C15ull + 1;
  auto rnd = [&]() { st += 0x9E3779B97F4A7C15ull; return mix64(st); };
  int bad = 0;
  if (msg && len) msg[0] = 0;
  for (int it = 0; it < iters; ++it) {
    const uint64_t sd = rnd(), sq = rnd();
    int32_t r[TB_N];
    tiebreak_records(sd, sq, r);
    const int32_t lim = r[TB_N - 1];
    std::vector<int64_t> Ts = {1, 2, 3, (int64_t)(rnd() % 1000) + 1, (int64_t)(rnd() % 200000) + 1,
                               (int64_t)(rnd() % (1ull << 31)) + 1, (int64_t)lim, (int64_t)lim + 1};
    for (int k = 0; k < TB_N - 1 && r[k] != INT32_MAX; ++k)
      for (int64_t d = -1; d <= 1; ++d) Ts.push_back((int64_t)r[k] + d);
    for (int64_t T : Ts) {
      if (T < 1) continue;
      int64_t got;
      if (T > (int64_t)lim) {
        got = tiebreak_position(sd, sq, T);   // the kernel's fallback
      } else {
        int cnt = 0;
        for (int k = 0; k < TB_N - 1; ++k) cnt += (r[k] != INT32_MAX && (int64_t)r[k] <= T) ? 1 : 0;
        got = cnt ? (int64_t)r[cnt - 1] : 1;
      }
      const int64_t want = tiebreak_position(sd, sq, T);
      if (got != want) {
        if (!bad && msg && len)
          snprintf(msg, len, "seed %llu seq %llu T %lld: lookup %lld, walk %lld", (unsigned long long)sd,
                   (unsigned long long)sq, (long long)T, (long long)got, (long long)want);
        ++bad;
      }
    }
  }
  return bad;
}

// ST: diagnostic build with s_memtime phase stamps (accumulated per phase, written to a.stamps)
template <bool ST>
__global__ void __launch_bounds__(COMMIT_THREADS) commit_kernel(CommitArgs a) {
  uint64_t st_acc[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_stage = 0;                      // header staging cycles (inside p0)   // numa_eval segments of thread 128's policy-row rescoring (ST)
  uint64_t st_last = ST ? __builtin_amdgcn_s_memtime() : 0;
#define STAMP(i)                                    \
  do {                                              \
    if (ST) {                                       \
      uint64_t t_ = __builtin_amdgcn_s_memtime();   \
      st_acc[i] += t_ - st_last;                    \
      st_last = t_;                                 \
    }                                               \
  } while (0)
  extern __shared__ __align__(16) unsigned char cm[];
  const int B = a.npods;
  const int R = a.nranks;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint64_t lt_mask = (1ull << lane) - 1ull;
  // pod vectors at a 136-B stride: the re-scoring threads read different pods, and a 128-B stride would put
  // every lane of a wave on the same two LDS banks
  auto pods = [&](int i) -> PodVec& { return *reinterpret_cast<PodVec*>(cm + (size_t)i * POD_STRIDE); };
  Row* drows = reinterpret_cast<Row*>(cm + (size_t)B * POD_STRIDE);          // B dirty slots
  int16_t* dsc = reinterpret_cast<int16_t*>(drows + B);                      // [pod][slot] current score
  int16_t* dso = dsc + B * B;                                                // [pod][slot] batch-start score
  // offsets from the LDS base, not integer-cast pointers: the address space stays visible to the compiler (an
  // integer round trip turns every access into a flat load that waits on outstanding global loads)
  const size_t hoff = ((size_t)B * POD_STRIDE + (size_t)B * sizeof(Row) + (size_t)B * B * 4 + 15) & ~(size_t)15;
  int32_t* hkey = reinterpret_cast<int32_t*>(cm + hoff);                     // HASH
  int32_t* hval = hkey + HASH;                                               // HASH
  CpuStateDev* cst = reinterpret_cast<CpuStateDev*>(hval + HASH);            // B dirty slots: CPU state

  __shared__ int32_t sh_score[MAX_RANKS * MAXLEV], sh_count[MAX_RANKS * MAXLEV], sh_dec[MAX_RANKS * MAXLEV];
  __shared__ uint32_t dnew[MAX_BATCH], tmp[MAX_BATCH];
  __shared__ uint32_t win[WIN];
  __shared__ int32_t pre_old[WIN + 1];
  __shared__ Row orow;                                  // batch-start copy of a freshly dirtied row
  __shared__ int s_action, s_slot, s_fresh, s_M, s_F;  // wave-0 decision for pod k (0 commit, 1 skip, 2 cut,
                                                       // 3 resolve from the full row)
  // a pod resolved from its whole score row (host slow path for pod 0, or in-kernel on one shard): its selectHost
  __shared__ int s_fk, s_fnode, s_fscore, s_ffeas, s_Md, s_Fd, s_ndc;
  __shared__ int64_t s_fties;
  __shared__ int s_red[2 * COMMIT_WAVES];
  __shared__ uint32_t s_winner;
  __shared__ int64_t s_T;
  __shared__ int s_cut;                                // the pod just committed needs host-side Reserve
  __shared__ int s_aff;                                // known affinity of pod k on its winner row (-1: recompute)
  __shared__ uint64_t s_cpuset[4];                     // CPUs of a device-side cpuset Reserve
  __shared__ HintTable s_ht, s_ht2;                    // NUMA hint sums of the winner row (new / batch-start state)
  const bool numa_on = (a.pf.enabled & 0x30u) != 0;
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();   // the kernel's duration -> committed[4] (100 MHz ticks)
  // speculative pass queued behind another batch: only if that one committed every pod with nothing left for
  // the host (committed[1] == 1); otherwise a no-op (committed = -1) the host discards
  if (a.prev && a.prev[1] != 1) {
    if (tid == 0) { a.committed[0] = -1; a.committed[1] = 0; a.committed[3] = 0; a.committed[4] = 0; }
    return;
  }

  __shared__ uint32_t s_start;                         // nextStartNodeIndex (node sampling)
  __shared__ int32_t s_wred[3][COMMIT_WAVES];                     // window selection: block scans / reductions
  __shared__ int32_t s_wend, s_wproc, s_ndirty;       // s_ndirty: dirty slots (wave 0's nd, published)
  if (tid == 0) {
    s_ndirty = 0;
    s_start = a.window_k ? (a.prev ? (uint32_t)a.prev[2] : a.start) : 0u;
    s_fk = a.forced_node >= 0 ? 0 : -1;
    s_fnode = a.forced_node;
    s_fscore = a.forced_score;
    s_ffeas = a.forced_feasible;
    s_fties = a.forced_ties;
  }
  // fresh-row fetch map of this wave-0 lane (loop invariant): kind 0 none, 1 i64 column, 2 i32 column, 3 the
  // Filter-time affinity byte, 4 the node index; destination region 0 orow, 1 the slot's CPU state, 2 s_aff
  int f_kind = 0, f_region = 0, f_off = 0, f_size = 8;
  const void* f_src = nullptr;
  if (lane < ROW_I64) { f_kind = 1; f_src = a.m.c64(kRowCol[lane]); f_off = lane * 8; }
  else if (lane == ROW_I64) { f_kind = 2; f_src = a.m.c32(C_FREE_PODS); f_off = offsetof(Row, free_pods); f_size = 4; }
  else if (lane == ROW_I64 + 1) { f_kind = 2; f_src = a.m.c32(C_DFLAGS); f_off = offsetof(Row, dflags); f_size = 4; }
  else if (lane == ROW_I64 + 2) { f_kind = 4; f_off = offsetof(Row, node); }
  else if (numa_on) {
    // CpuStateDev's 11 words (C_CPU_UN0 .. C_CPU_XC1), meta, topo; lanes 32..61 the NUMA row
    if (lane >= 20 && lane < 31) { f_kind = 1; f_src = a.m.c64(C_CPU_UN0 + (lane - 20)); f_region = 1; f_off = (lane - 20) * 8; }
    else if (lane == 31) { f_kind = 2; f_src = a.m.c32(C_CPU_META); f_region = 1; f_off = offsetof(CpuStateDev, meta); f_size = 4; }
    else if (lane == 62) { f_kind = 2; f_src = a.m.c32(C_TOPO_DEV); f_region = 1; f_off = offsetof(CpuStateDev, topo); f_size = 4; }
    else if (lane == 63) { f_kind = 3; f_src = a.aff; f_region = 2; f_size = 4; }
    else if (lane >= 32 && lane < 32 + NUMA_I64) {
      f_kind = 1; f_src = a.m.c64(C_ZCAP_CPU0 + (lane - 32)); f_off = offsetof(Row, nr) + (lane - 32) * 8;
    } else if (lane >= 50 && lane < 50 + NUMA_I32) {
      f_kind = 2; f_src = a.m.c32(C_NFLAGS + (lane - 50)); f_off = offsetof(Row, nr.nflags) + (lane - 50) * 4; f_size = 4;
    }
  }
  for (int i = tid; i < B; i += COMMIT_THREADS) pods(i) = a.pods[i];
  for (int i = tid; i < HASH; i += COMMIT_THREADS) { hkey[i] = -1; hval[i] = -1; }
  const MirrorView& m = a.m;
  const int nhl = R * MAXLEV;                    // header lanes: lane = r*MAXLEV + j
  // LevelHdrs and seq of HCH pods at a time are staged in LDS (one HBM round trip per chunk)
  constexpr int HCH = 16;
  __shared__ int32_t hs_score[HCH][MAX_RANKS * MAXLEV], hs_count[HCH][MAX_RANKS * MAXLEV];
  __shared__ int32_t hs_nlev[HCH][MAX_RANKS], hs_feas[HCH][MAX_RANKS], hs_next[HCH][MAX_RANKS];
  __shared__ uint64_t hs_seq[HCH];
  int nd = 0;
  int committed = B;
  bool host_cut = false;   // the batch ended at a pod whose cpuset Reserve the host performs
  __syncthreads();

  // wave 0: the winner's slot in the dirty set (its batch-start row, CPU state and Filter-time affinity fetched
  // from HBM when fresh: one load per lane, all issued before a single wait), and the decision for pod k
  auto fetch_winner = [&](int k, uint32_t winner, int M, int F, int64_t T) {
    int slot = hash_find(hkey, hval, winner);
    const bool fresh = slot < 0;
    if (fresh) {
      slot = nd;
      if (lane == 0) {
        uint32_t h = (winner * 2654435761u) & (HASH - 1);
        while (hkey[h] >= 0) h = (h + 1) & (HASH - 1);
        hkey[h] = (int32_t)winner;
        hval[h] = slot;
      }
      ++nd;
      if (lane == 0) s_ndirty = nd;
      // one load per lane, all issued before a single wait (the per-lane source/destination map is built once)
      int64_t v = 0;
      if (f_kind == 1) v = reinterpret_cast<const int64_t*>(f_src)[winner];
      else if (f_kind == 2) v = reinterpret_cast<const int32_t*>(f_src)[winner];
      else if (f_kind == 3) {   // the batch-start Filter's affinity for this pair (own shard, NUMA-policy nodes)
        const bool own = f_src && winner >= a.own0 && winner < a.own1;
        const uint8_t b8 = own ? reinterpret_cast<const uint8_t*>(f_src)[(size_t)k * a.ld + (winner - a.own0)]
                               : AFF_RECOMPUTE;
        v = b8 == AFF_RECOMPUTE ? (int64_t)-1 : (int64_t)b8;   // (a patched row's: recomputed)
      } else if (f_kind == 4) v = (int64_t)winner;   // Row.node, Row.pad = 0
      if (f_kind) {
        unsigned char* dst = f_region == 0 ? reinterpret_cast<unsigned char*>(&orow)
                           : f_region == 1 ? reinterpret_cast<unsigned char*>(&cst[slot])
                                           : reinterpret_cast<unsigned char*>(&s_aff);
        if (f_size == 8) *reinterpret_cast<int64_t*>(dst + f_off) = v;
        else *reinterpret_cast<int32_t*>(dst + f_off) = (int32_t)v;
      }
    }
    if (lane == 0) {
      s_action = 0; s_slot = slot; s_fresh = fresh; s_winner = winner; s_M = M; s_F = F; s_T = T;
      if (!fresh || !numa_on) s_aff = -1;   // a dirty row changed since the batch-start Filter
    }
  };
  // Node sampling ([upstream] findNodesThatPassFilters, parallelism-1 order): positions i = 0.. from s_start in
  // rotation order; a node's verdict for pod k is its batch-start score S[k][n] unless an earlier pod of the batch
  // landed on it (its current score dsc). The window is the first K = window_k feasible positions; the (K+1)-th
  // feasible position ends the search uncounted (processedNodes = its position, else N). selectHost: max and
  // ties over the window, the jp-th tie in window order. All threads; 8 consecutive positions per thread.
  auto block_scan = [&](int v, int slot, int* total) -> int {   // exclusive prefix over tid order
    int incl = v;
    for (int off = 1; off < 64; off <<= 1) {
      const int u = __shfl_up(incl, off);
      if (lane >= off) incl += u;
    }
    if (lane == 63) s_wred[slot][wave] = incl;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < COMMIT_WAVES; ++w) { const int x = s_wred[slot][w]; if (w < wave) base += x; tot += x; }
    __syncthreads();
    *total = tot;
    return base + incl - v;
  };
  auto window_select = [&](int k) {
    // 16 positions per thread (4096 per pass): the first pass's verdicts stay in registers and the tie location
    // reuses them when the window ends inside it (a window of K feasible nodes usually does)
    constexpr int WCH = 16;
    const uint32_t N = a.nnodes, K = a.window_k, st0 = s_start;
    const int16_t* row = a.S + (size_t)k * a.ld;
    auto node_at = [&](uint32_t i) -> uint32_t {
      const uint32_t n = st0 + i;
      return n >= N ? n - N : n;
    };
    auto load_pass = [&](uint32_t base, int* v) {   // all S loads issued before the dirty-row probes
#pragma unroll
      for (int j = 0; j < WCH; ++j) {
        const uint32_t i = base + (uint32_t)tid * WCH + j;
        v[j] = i < N ? (int)row[node_at(i) - a.own0] : -1;
      }
      if (s_ndirty > 0) {
#pragma unroll
        for (int j = 0; j < WCH; ++j) {
          const uint32_t i = base + (uint32_t)tid * WCH + j;
          if (i >= N) continue;
          const int sl = hash_find(hkey, hval, node_at(i));
          if (sl >= 0) v[j] = (int)dsc[k * B + sl];
        }
      }
    };
    if (tid == 0) { s_wend = (int)N - 1; s_wproc = (int)N; }
    int found = 0, lmax = -1, lcnt = 0, v[WCH];
    uint32_t passes = 0;
    for (uint32_t base = 0; base < N; base += COMMIT_THREADS * WCH) {
      load_pass(base, v);
      ++passes;
      int c = 0;
#pragma unroll
      for (int j = 0; j < WCH; ++j) c += v[j] >= 0 ? 1 : 0;
      int total = 0;
      int idx = found + block_scan(c, 0, &total);   // window index of this thread's first feasible position
#pragma unroll
      for (int j = 0; j < WCH; ++j) {
        if (v[j] < 0) continue;
        const uint32_t i = base + (uint32_t)tid * WCH + j;
        if ((uint32_t)idx < K) {
          if (v[j] > lmax) { lmax = v[j]; lcnt = 1; }
          else if (v[j] == lmax) ++lcnt;
          if ((uint32_t)idx == K - 1) s_wend = (int)i;
        } else if ((uint32_t)idx == K) {
          s_wproc = (int)i;
        }
        ++idx;
      }
      found += total;
      if ((uint32_t)found > K) break;   // block-uniform
    }
    // M, T over the window
    const int wm = wave_max(lmax);
    if (lane == 0) s_wred[1][wave] = wm;
    __syncthreads();
    int M = s_wred[1][0];
    for (int w = 1; w < COMMIT_WAVES; ++w) M = max(M, s_wred[1][w]);
    const int tl = wave_sum(lmax == M ? lcnt : 0);
    if (lane == 0) s_wred[2][wave] = tl;
    __syncthreads();
    int64_t T = 0;
    for (int w = 0; w < COMMIT_WAVES; ++w) T += s_wred[2][w];
    const int F = (int)min((uint32_t)found, K);
    const uint32_t wend = (uint32_t)s_wend, proc = (uint32_t)s_wproc;
    if (M < 0) {   // FitError: nothing assumed; every node was processed
      if (tid == 0) {
        a.out[k] = PlacementDev{-1, (uint32_t)F, 0, 0, 0, 0, 0, {0, 0, 0, 0}, {0, 0, 0, 0}};
        s_action = 1;
        s_start = (st0 + proc) % N;
      }
      __syncthreads();
      return;
    }
    // the jp-th tie at M in window order (registers hold the single pass when the window ended inside it)
    const int64_t jp = tiebreak_position(a.seed, a.seq[k], T);
    int64_t before = 0;
    if (tid == 0) s_fnode = -1;
    for (uint32_t base = 0; base <= wend; base += COMMIT_THREADS * WCH) {
      if (passes > 1) load_pass(base, v);
      int c = 0;
#pragma unroll
      for (int j = 0; j < WCH; ++j) {
        const uint32_t i = base + (uint32_t)tid * WCH + j;
        c += (i <= wend && v[j] == M) ? 1 : 0;
      }
      int total = 0;
      const int64_t ex = before + block_scan(c, 0, &total);
      if (c > 0 && jp > ex && jp <= ex + c) {
        int64_t need = jp - ex;
#pragma unroll
        for (int j = 0; j < WCH; ++j) {
          const uint32_t i = base + (uint32_t)tid * WCH + j;
          if (i <= wend && v[j] == M && --need == 0) s_fnode = (int)node_at(i);
        }
      }
      before += total;
      if (before >= jp) break;   // block-uniform
    }
    __syncthreads();
    if (tid == 0) {
      s_action = s_fnode >= 0 ? 0 : 2;   // 2: unreachable (the tie exists), the host fails loudly
      s_winner = (uint32_t)s_fnode;
      s_M = M; s_F = F; s_T = T;
      s_start = (st0 + proc) % N;
    }
    __syncthreads();
  };
  for (int k = 0; k < B; ++k) {
   const uint64_t t_stage0 = ST ? __builtin_amdgcn_s_memtime() : 0;
   if (k % HCH == 0 && !a.window_k) {
     for (int e = tid; e < HCH * nhl; e += COMMIT_THREADS) {
       int kk = e / nhl, l = e % nhl;
       if (k + kk < B) {
         const LevelHdr* h = hdr_ptr(a, l / MAXLEV, k + kk);
         hs_score[kk][l] = h->score[l % MAXLEV];
         hs_count[kk][l] = h->count[l % MAXLEV];
       }
     }
     for (int e = tid; e < HCH * R; e += COMMIT_THREADS) {
       int kk = e / R, r = e % R;
       if (k + kk < B) {
         const LevelHdr* h = hdr_ptr(a, r, k + kk);
         hs_nlev[kk][r] = h->nlev;
         hs_feas[kk][r] = h->feasible;
         hs_next[kk][r] = h->next;
       }
     }
     for (int e = tid; e < HCH; e += COMMIT_THREADS)
       if (k + e < B) hs_seq[e] = a.seq[k + e];
     __syncthreads();
   }
   if (ST) st_stage += __builtin_amdgcn_s_memtime() - t_stage0;   // header staging share of p0
   for (;;) {   // one pass; a second, forced one after an in-kernel full-row resolution
   if (a.window_k) {   // node sampling: findNodesThatPassFilters over the rotation window, then selectHost
     window_select(k);
     if (wave == 0 && s_action == 0) fetch_winner(k, s_winner, s_M, s_F, s_T);
     __syncthreads();
     break;
   }
   if (wave == 0) do {   // ===================== wave 0: selectHost for pod k =====================
    const int kc = k % HCH;
    const int r_l = lane / MAXLEV, j_l = lane % MAXLEV;
    int hs = lane < nhl ? hs_score[kc][lane] : -1, hc = lane < nhl ? hs_count[kc][lane] : 0;
    const int feas_l = lane < R ? hs_feas[kc][lane] : 0, next_l = lane < R ? hs_next[kc][lane] : -1;
    const uint64_t seqk = hs_seq[kc];
    const bool lvl = lane < nhl && j_l < hs_nlev[kc][r_l < MAX_RANKS ? r_l : 0];
    if (!lvl) { hs = -1; hc = 0; }
    if (lane < nhl) { sh_score[lane] = hs; sh_count[lane] = hc; sh_dec[lane] = 0; }
    WAVE_FENCE();
    STAMP(0);
    const bool forced = k == s_fk;
    // ---- dirty rows: batch-start / current scores of pod k, listed-level decrements
    int Md = -1, Fd = 0;
    for (int s = lane; s < nd; s += 64) {
      int sc = dsc[k * B + s], so = dso[k * B + s];
      Md = max(Md, sc);
      Fd += (sc >= 0 ? 1 : 0) - (so >= 0 ? 1 : 0);
      if (so >= 0) {
        int base = (int)(drows[s].node / a.shard_size) * MAXLEV;
        for (int j = 0; j < MAXLEV; ++j)
          if (sh_score[base + j] == so) { atomicAdd(&sh_dec[base + j], 1); break; }
      }
    }
    Md = wave_max(Md);
    Fd = wave_sum(Fd);
    WAVE_FENCE();
    STAMP(1);
    const int clean = lvl ? hc - sh_dec[lane] : 0;
    int M = max(wave_max(clean > 0 ? hs : -1), Md);
    int F = Fd + wave_sum(lane < R ? feas_l : 0);
    if (forced) {
      M = s_fscore;
      F = s_ffeas;
    } else if (__ballot(lane < R && M <= next_l)) {
      // a shard may hold unlisted nodes at M: one shard resolves pod k from its whole row right here; with
      // several shards the batch is cut and the host resolves it (row_stats / row_select / exchange)
      if (lane == 0) {
        s_action = (R == 1 && a.S) ? 3 : 2;
        s_Md = Md;
        s_Fd = Fd;
        s_ndc = nd;   // the dirty-slot count lives in wave 0's registers only
      }
      break;
    }
    if (M < 0) {       // FitError: no feasible node anywhere, nothing assumed
      if (lane == 0) {
        a.out[k] = PlacementDev{-1, (uint32_t)F, 0, 0, 0, 0, 0, {0, 0, 0, 0}, {0, 0, 0, 0}};
        s_action = 1;
      }
      break;
    }
    uint32_t winner = 0xffffffffu;
    int64_t T = 0;
    STAMP(2);
    if (forced) {
      if (s_fnode < 0) { if (lane == 0) s_action = 2; break; }   // unreachable for a valid max: cut, host re-run
      winner = (uint32_t)s_fnode;
      T = s_fties;
    } else {
      // ---- tie set at M: clean listed nodes + dirty rows now at M ("dnew") - dirty rows listed at M ("old")
      const int cm_lane = (lvl && hs == M) ? clean : 0;
      int ndn = 0;
      for (int s0 = 0; s0 < nd; s0 += 64) {
        int s = s0 + lane;
        bool isn = s < nd && dsc[k * B + s] == M;
        uint64_t bn = __ballot(isn);
        if (isn) dnew[ndn + __popcll(bn & lt_mask)] = drows[s].node;
        ndn += __popcll(bn);
      }
      WAVE_FENCE();
      T = (int64_t)wave_sum(cm_lane) + ndn;
      int64_t jp = tiebreak_position(a.seed, seqk, T);
      if (ndn > 1) wave_rank_sort(dnew, ndn, tmp, lane);
      STAMP(3);
      // per shard: clean ties + dirty ties (lane r < R), owning shard r* by prefix
      int here = 0;
      {
        int c = 0;
        for (int j = 0; j < MAXLEV; ++j) c += __shfl(cm_lane, (lane < R ? lane : 0) * MAXLEV + j);
        if (lane < R) {
          uint32_t sb = (uint32_t)lane * a.shard_size, se = sb + a.shard_size;
          int dn = 0;
          for (int u = 0; u < ndn; ++u) dn += dnew[u] >= sb && dnew[u] < se;
          here = c + dn;
        }
      }
      int incl = here;
      for (int off = 1; off < 64; off <<= 1) {
        int v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
      }
      uint64_t hit = __ballot(lane < R && incl >= jp);
      const int rstar = hit ? (__ffsll((long long)hit) - 1) : (R - 1);
      jp -= __shfl(incl - here, rstar);
      // level-M segment of r*'s list
      int off = 0, len = 0;
      for (int j = 0; j < MAXLEV; ++j) {
        int sc = sh_score[rstar * MAXLEV + j];
        if (sc < 0) break;
        if (sc == M) { len = sh_count[rstar * MAXLEV + j]; break; }
        off += sh_count[rstar * MAXLEV + j];
      }
      const uint32_t sb = (uint32_t)rstar * a.shard_size, se = sb + a.shard_size;
      int nn_lo = 0;
      while (nn_lo < ndn && dnew[nn_lo] < sb) ++nn_lo;
      int nn_hi = nn_lo;
      while (nn_hi < ndn && dnew[nn_hi] < se) ++nn_hi;
      // dirty rows of r* listed at M (batch-start score M)
      int ndo_r = 0;
      for (int s = lane; s < nd; s += 64) {
        uint32_t node = drows[s].node;
        ndo_r += (dso[k * B + s] == M && node >= sb && node < se) ? 1 : 0;
      }
      ndo_r = wave_sum(ndo_r);
      const int lo = (int)max<int64_t>(0, jp - 2 - (nn_hi - nn_lo));
      const int hi = (int)min<int64_t>(len - 1, jp - 1 + ndo_r);
      const int W = hi - lo + 1;
      // ---- the jp-th node of (listed level-M nodes of r* - old) U dnew, node order, over window L[lo..hi]
      const uint32_t* L = list_ptr(a, rstar, k) + off;
      uint32_t cand = 0xffffffffu;
      if (len > 0) {
        for (int i = lane; i < W; i += 64) win[i] = L[lo + i];
        WAVE_FENCE();
        STAMP(4);
        // old rows before the window, then a running count over the window (membership via the hash)
        int base_old = 0;
        for (int s = lane; s < nd; s += 64) {
          uint32_t node = drows[s].node;
          base_old += (dso[k * B + s] == M && node >= sb && node < win[0]) ? 1 : 0;
        }
        base_old = wave_sum(base_old);
        int running = base_old;
        for (int i0 = 0; i0 < W; i0 += 64) {
          int i = i0 + lane;
          uint32_t x = i < W ? win[i] : 0xffffffffu;
          bool isold = false;
          if (i < W) {
            int sl = hash_find(hkey, hval, x);
            isold = sl >= 0 && dso[k * B + sl] == M;
          }
          uint64_t bo = __ballot(isold);
          int older = running + __popcll(bo & lt_mask);
          if (i < W) {
            pre_old[i] = older;
            int newer = 0;
            for (int u = nn_lo; u < nn_hi; ++u) newer += dnew[u] < x;
            if (!isold && (int64_t)(lo + i - older + newer + 1) == jp) cand = x;
          }
          running += __popcll(bo);
        }
        if (lane == 0) pre_old[W] = running;
        WAVE_FENCE();
      }
      for (int u0 = nn_lo + lane; u0 < nn_hi; u0 += 64) {
        uint32_t n = dnew[u0];
        int64_t ltn = -1;   // #listed level-M nodes < n, when it can decide position jp
        int older = 0;
        if (len == 0) {
          ltn = 0;
        } else {
          int p = 0, q = W;      // lower_bound(win, n)
          while (p < q) { int mid = (p + q) >> 1; if (win[mid] < n) p = mid + 1; else q = mid; }
          if (p == 0) ltn = (lo == 0) ? 0 : -1;
          else if (p == W) ltn = (hi == len - 1) ? len : -1;
          else ltn = lo + p;
          older = pre_old[p];
        }
        if (ltn >= 0 && ltn - older + (u0 - nn_lo) + 1 == jp) cand = n;
      }
      uint64_t got = __ballot(cand != 0xffffffffu);
      if (!got) { if (lane == 0) s_action = 2; break; }   // unreachable for a valid max: cut, exact re-run
      winner = __shfl(cand, __ffsll((long long)got) - 1);
    }
    STAMP(5);
    fetch_winner(k, winner, M, F, T);
    STAMP(6);
   } while (0);
    __syncthreads();
    if (s_action != 3) break;
    // ---- exact full-row resolution of pod k on the single shard: batch-start scores S[k][*] for clean nodes,
    // current scores for dirty rows; max, ties and feasible count, then the j*-th tie in node order
    {
      const int16_t* row = a.S + (size_t)k * a.ld;
      const uint32_t len = a.own1 - a.own0, chunk = (len + COMMIT_THREADS - 1) / COMMIT_THREADS;
      const uint32_t i0 = min(len, (uint32_t)tid * chunk), i1 = min(len, i0 + chunk);
      int lmax = -1, lfeas = 0;
      for (uint32_t i = i0; i < i1; ++i) {
        const int x = row[i];
        lfeas += x >= 0 ? 1 : 0;
        if (x > lmax && hash_find(hkey, hval, a.own0 + i) < 0) lmax = x;
      }
      lmax = wave_max(lmax);
      lfeas = wave_sum(lfeas);
      if (lane == 0) { s_red[wave] = lmax; s_red[COMMIT_WAVES + wave] = lfeas; }
      __syncthreads();
      int M = s_Md, F = s_Fd;
      for (int w = 0; w < COMMIT_WAVES; ++w) { M = max(M, s_red[w]); F += s_red[COMMIT_WAVES + w]; }
      __syncthreads();
      int cnt = 0;
      if (M >= 0) {
        for (uint32_t i = i0; i < i1; ++i)
          if (row[i] == M && hash_find(hkey, hval, a.own0 + i) < 0) ++cnt;
        for (int s = 0; s < s_ndc; ++s) {
          const uint32_t n = drows[s].node;
          if (n >= a.own0 + i0 && n < a.own0 + i1 && dsc[k * B + s] == M) ++cnt;
        }
      }
      int incl = cnt;
      for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
      }
      if (lane == 63) s_red[wave] = incl;
      __syncthreads();
      int base = 0;
      for (int w = 0; w < wave; ++w) base += s_red[w];
      int64_t T = 0;
      for (int w = 0; w < COMMIT_WAVES; ++w) T += s_red[w];
      const int64_t jp = T > 0 ? tiebreak_position(a.seed, hs_seq[k % HCH], T) : 0;
      const int64_t excl = base + incl - cnt;
      if (tid == 0) s_fnode = -1;
      __syncthreads();
      if (T > 0 && jp > excl && jp <= excl + cnt) {   // this thread's chunk holds the jp-th tie
        int64_t need = jp - excl;
        for (uint32_t i = i0; i < i1; ++i) {
          const int sl = hash_find(hkey, hval, a.own0 + i);
          const bool tie = sl >= 0 ? dsc[k * B + sl] == M : row[i] == M;
          if (tie && --need == 0) { s_fnode = (int)(a.own0 + i); break; }
        }
      }
      if (tid == 0) { s_fk = k; s_fscore = M; s_fties = T; s_ffeas = F; }
      __syncthreads();
    }
   }
    // ===================== all waves: assume + Reserve, re-score later pods =====================
    const int action = s_action;
    if (action == 2) { committed = k; break; }
    if (action == 1) continue;
    const int slot = s_slot;
    const bool fresh = s_fresh;
    Row& d = drows[slot];
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    if (wv == 0 && numa_on && s_aff < 0) {   // hint table of the winner's pre-Reserve state (affinity unknown)
      const NumaRow nr = fresh ? orow.nr : d.nr;
      if ((nr.nflags >> NF_POLICY_SHIFT) & 3u) hint_table_fill(s_ht, nr, zone_avail(nr), lane);
      WAVE_FENCE();
    }
    if (tid == 0) {
      const Row dr = fresh ? orow : d;   // registers: the Reserve's pair evaluation re-reads row words
      if (fresh) d = dr;
      const PodVec& pk = pods(k);
      const bool forced = k == s_fk;
      PlacementDev pl{(int32_t)s_winner, (uint32_t)s_F, (int64_t)s_M, (uint32_t)s_T, forced ? 1u : 0u, 0, 0,
                      {0, 0, 0, 0}, {0, 0, 0, 0}};
      s_cut = 0;
      const uint32_t nf = dr.nr.nflags;
      // Reserve returns at once unless requestCPUBind (util.go:105-122) or the node has a NUMA policy
      const bool maybe_rb = (pk.numa & PN_BIND) || (((nf >> NF_BIND_SHIFT) & 3u) && (pk.req_keys & 1u) && pk.req[0]);
      if (numa_on && !(pk.numa & (PN_SKIP | PN_PREFAIL)) && (maybe_rb || ((nf >> NF_POLICY_SHIFT) & 3u))) {
        // NodeNUMAResource Reserve (plugin.go:375-422) on the pre-assume row: the Filter-time affinity and the
        // NUMA split of Allocate; a cpuset pod's CPUs are selected here (gs_cpuset_dev.h) when the node's
        // topology is in the device scope, else the batch ends with it and the host selects them
        NumaOut no = numa_eval<true, true>(dr.nr, pk, a.pf, SlotsLds{dr, m}, a.pf.enabled & 0x10u, false, s_aff, &s_ht);
        STAMP(10);
        const bool rb = no.flags & GS_PLACED_CPUSET;
        if (no.reason) pl.flags |= PL_RESERVE_FAILED;   // cannot happen for a feasible winner
        if (rb || ((nf >> NF_POLICY_SHIFT) & 3u)) {
          pl.flags |= no.flags;
          pl.zkeys = no.zkeys;
#pragma unroll
          for (int z = 0; z < 4; ++z) { pl.zcpu[z] = no.zcpu[z]; pl.zmem[z] = no.zmem[z]; }
          if (nf & NF_TOPO_VALID) {   // resourceManager.Update -> NodeAllocation.addPodAllocation
            uint32_t f2 = dr.nr.nflags2;
#pragma unroll
            for (int z = 0; z < 4; ++z) {
              const bool zc = no.zkeys >> z & 1u, zm = no.zkeys >> (4 + z) & 1u;
              if (!zc && !zm) continue;
              d.nr.zraw_cpu[z] = dr.nr.zraw_cpu[z] + no.zcpu[z];
              d.nr.zraw_mem[z] = dr.nr.zraw_mem[z] + no.zmem[z];
              f2 |= (1u << (NF2_ENTRY_SHIFT + z)) | (zc ? 1u << (NF2_ACPU_SHIFT + z) : 0u) |
                    (zm ? 1u << (NF2_AMEM_SHIFT + z) : 0u);
            }
            d.nr.nflags2 = f2;
          }
          if (rb) {
            CpuStateDev& cs = cst[slot];
            if (cpuset_on_device(cs, pk)) {   // (the topology's TopoDev is read from HBM: scalar loads)
              if (cpuset_reserve(a.topos + cs.topo, (GS_LDS CpuStateDev*)&cs, pk, nf, no.zkeys, no.zcpu[0],
                                 no.zcpu[1], no.zcpu[2], no.zcpu[3],
                                 (GS_LDS NumaRow*)&d.nr, (GS_LDS uint64_t*)s_cpuset)) {
                pl.flags |= PL_DEVICE_CPUSET;
#pragma unroll
                for (int j = 0; j < 4; ++j) pl.cpuset[j] = s_cpuset[j];
              } else {
                pl.flags |= PL_RESERVE_FAILED;
              }
              STAMP(11);
            } else {
              s_cut = 1;
            }
          }
        }
      }
      a.out[k] = pl;
      for (int s = 0; s < 7; ++s) d.free[s] = dr.free[s] - pk.req[s];
      d.nzfree[0] = dr.nzfree[0] - pk.nz[0];
      d.nzfree[1] = dr.nzfree[1] - pk.nz[1];
      d.free_pods = dr.free_pods - 1;
      d.la_free[0] = dr.la_free[0] - pk.est[0];
      d.la_free[1] = dr.la_free[1] - pk.est[1];
      if (pk.flags & PF_PROD) {
        d.la_pfree[0] = dr.la_pfree[0] - pk.est[0];
        d.la_pfree[1] = dr.la_pfree[1] - pk.est[1];
      }
    }
    // NUMA-policy winner row: wave 0 builds the hint table of its new state (one entry per lane) for the
    // re-scoring lanes; wave 1 that of a fresh row's batch-start state when its batch-start scores are evaluated
    // (a node outside this rank's shard)
    if (wv == 0 && numa_on) {
      WAVE_FENCE();
      const uint32_t nfw = d.nr.nflags;
      if ((nfw >> NF_POLICY_SHIFT) & 3u) {
        const NumaRow nr = d.nr;
        hint_table_fill(s_ht, nr, zone_avail(nr), lane);
      }
    } else if (wv == 1 && numa_on && fresh && !(orow.node >= a.own0 && orow.node < a.own1)) {
      const NumaRow nr = orow.nr;
      if ((nr.nflags >> NF_POLICY_SHIFT) & 3u) hint_table_fill(s_ht2, nr, zone_avail(nr), lane);
    }
    __syncthreads();
    if (s_cut) { committed = k + 1; host_cut = true; break; }
    if (tid == 0) STAMP(7);
    // Re-scoring, pods q = k+1 .. over the waves, RS_PODS per wave: lanes 0..RS_PODS-1 evaluate the winner row's
    // current score (one row for all lanes: the NUMA hint sums come from the table); lanes 32.. of a fresh row fetch
    // its batch-start score from the score rows S when the node is in this rank's shard, else evaluate it.
    {
      constexpr int RS_PODS = MAX_BATCH / COMMIT_WAVES;
      const int sub = lane & 31;
      const bool cur = lane < 32;
      const int q = sub < RS_PODS ? k + 1 + wv * RS_PODS + sub : B;
      const uint64_t t0_ = ST ? __builtin_amdgcn_s_memtime() : 0;
      const uint32_t node = d.node;
      const bool own = node >= a.own0 && node < a.own1;
      const bool load_so = !cur && fresh && own && q < B;
      int16_t so = 0;
      if (load_so) so = a.S_own[(size_t)q * a.ld + (node - a.own0)];
      const bool policy_row = numa_on && ((d.nr.nflags >> NF_POLICY_SHIFT) & 3u);   // (ST stamps)
      if (q < B && cur) {   // the row is wave-uniform (LDS at a uniform slot): its words can live in SGPRs
        const Row rr = d;
        dsc[q * B + slot] = (int16_t)row_score(rr, pods(q), a.pf, m, &s_ht);
      }
      if (fresh && !own && q < B && !cur) {   // several ranks only
        const Row rr = orow;
        dso[q * B + slot] = (int16_t)row_score(rr, pods(q), a.pf, m, &s_ht2);
      }
      if (load_so) dso[q * B + slot] = so;
      if (ST && tid == 128 && policy_row) {
        st_acc[12] += 1;
        st_acc[13] += __builtin_amdgcn_s_memtime() - t0_;
      }
    }
    __syncthreads();
    if (tid == 0) {   // rescoring time, split by the winner row's NUMA policy (p8: policy node, p9: none)
      if ((d.nr.nflags >> NF_POLICY_SHIFT) & 3u) STAMP(8);
      else STAMP(9);
    }
  }
  // write back dirty rows (slots are dense: count them from the hash)
  __shared__ int s_nd;
  if (tid == 0) {
    int n = 0;
    for (int i = 0; i < HASH; ++i) n += hkey[i] >= 0;
    s_nd = n;
  }
  __syncthreads();
  nd = s_nd;
  for (int e = tid; e < nd * ROW_I64; e += COMMIT_THREADS) {
    int s = e / ROW_I64, j = e % ROW_I64;
    if (row_word_mutable(j)) m.c64(kRowCol[j])[drows[s].node] = reinterpret_cast<const int64_t*>(&drows[s])[j];
  }
  for (int s = tid; s < nd; s += COMMIT_THREADS) m.c32(C_FREE_PODS)[drows[s].node] = drows[s].free_pods;
  // NUMA words Reserve changes: ZRAW (8 i64), NFLAGS2 .. ZADJ3 (11 i32), CPU state (11 i64 + meta)
  constexpr int NW = 8 + 11 + 11 + 1;
  static_assert(C_ZADJ0 + 3 - C_NFLAGS2 + 1 == 11, "NUMA i32 write-back columns contiguous");
  if (numa_on)
    for (int e = tid; e < nd * NW; e += COMMIT_THREADS) {
      const int sl = e / NW, j = e % NW;
      const uint32_t node = drows[sl].node;
      if (j < 8) m.c64(C_ZRAW_CPU0 + j)[node] = (&drows[sl].nr.zraw_cpu[0])[j];
      else if (j < 19) m.c32(C_NFLAGS2 + (j - 8))[node] = reinterpret_cast<const int32_t*>(&drows[sl].nr.nflags2)[j - 8];
      else if (j < 30) m.c64(C_CPU_UN0 + (j - 19))[node] = reinterpret_cast<const int64_t*>(&cst[sl])[j - 19];
      else m.c32(C_CPU_META)[node] = (int32_t)cst[sl].meta;
    }
  if (tid == 0) {
    a.committed[0] = committed;
    a.committed[1] = (committed == B && !host_cut) ? 1 : 0;
    a.committed[2] = (int32_t)s_start;
    a.committed[3] = 0;
    a.committed[4] = (int32_t)(__builtin_amdgcn_s_memrealtime() - rt0);
  }
  if (ST && tid == 0) {
    for (int i = 0; i < 12; ++i) a.stamps[i] += st_acc[i];
    a.stamps[24] += st_stage;
  }
  if (ST && tid == 128) {
    a.stamps[12] += st_acc[12];
    a.stamps[13] += st_acc[13];
  }
#undef STAMP
}

// ------------------------------------------------------------------------------------------------
// Exact full-row path: (max, ties at max, feasible) of one score row, then the node at a tie position.
__global__ void __launch_bounds__(1024) row_stats_kernel(const int16_t* __restrict__ S, uint32_t len,
                                                          RowStat* __restrict__ out) {
  __shared__ int red_m[16], red_t[16], red_f[16];
  int t = threadIdx.x;
  int mx = -1, cnt = 0, feas = 0;
  for (uint32_t i = t; i < len; i += 1024) {
    int v = S[i];
    if (v >= 0) ++feas;
    if (v > mx) { mx = v; cnt = 1; }
    else if (v == mx && v >= 0) ++cnt;
  }
  for (int off = 32; off > 0; off >>= 1) {
    int om = __shfl_xor(mx, off), oc = __shfl_xor(cnt, off), of = __shfl_xor(feas, off);
    if (om > mx) { mx = om; cnt = oc; } else if (om == mx) cnt += oc;
    feas += of;
  }
  int w = t >> 6;
  if ((t & 63) == 0) { red_m[w] = mx; red_t[w] = cnt; red_f[w] = feas; }
  __syncthreads();
  if (t == 0) {
    int M = -1, C = 0, F = 0;
    for (int i = 0; i < 16; ++i) {
      if (red_m[i] > M) { M = red_m[i]; C = red_t[i]; } else if (red_m[i] == M) C += red_t[i];
      F += red_f[i];
    }
    RowStat r;
    r.max_score = M;
    r.ties = M >= 0 ? C : 0;
    r.feasible = F;
    r.pad = 0;
    *out = r;
  }
}

__global__ void __launch_bounds__(1024) row_select_kernel(const int16_t* __restrict__ S, uint32_t len, int score,
                                                           int64_t target, uint32_t n0, int32_t* __restrict__ out) {
  __shared__ int cnts[1024];
  int t = threadIdx.x;
  uint32_t per = (len + 1023) / 1024;
  uint32_t b = t * per, e = min(len, b + per);
  int c = 0;
  for (uint32_t i = b; i < e; ++i) c += S[i] == score;
  cnts[t] = c;
  __syncthreads();
  if (t == 0) {
    int64_t acc = 0;
    for (int i = 0; i < 1024; ++i) {
      int64_t nacc = acc + cnts[i];
      if (nacc >= target) {
        uint32_t bb = i * per, ee = min(len, bb + per);
        int64_t pos = acc;
        for (uint32_t j = bb; j < ee; ++j)
          if (S[j] == score && ++pos == target) { *out = (int32_t)(n0 + j); return; }
      }
      acc = nacc;
    }
    *out = -1;
  }
}

// ------------------------------------------------------------------------------------------------
// prep: the rows' LoadAware verdicts at `now` computed from the staged words (node_prep_kernel's rule, one launch less
// on the delta path's chain)
__global__ void __launch_bounds__(256) scatter_rows_kernel(MirrorView m, const uint32_t* __restrict__ idx,
                                                           const int64_t* __restrict__ rows, uint32_t nrows, int prep,
                                                           int64_t now, int32_t filter_expired, int32_t has_exp,
                                                           int64_t exp_ns) {
  uint32_t r = blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  uint32_t i = idx[r];
  const int64_t* src = rows + (size_t)r * ROW_WORDS;
  for (int c = 0; c < NUM_I64_COLS; ++c) m.c64(c)[i] = src[c];
  for (int c = 0; c < NUM_I32_COLS; ++c) m.c32(c)[i] = (int32_t)src[NUM_I64_COLS + c];
  if (prep)
    m.c32(C_DFLAGS)[i] = (int32_t)node_prep_flags((uint32_t)src[NUM_I64_COLS + C_SFLAGS], src[C_UPDATE_TIME], now,
                                                  filter_expired, has_exp, exp_ns);
}

// ------------------------------------------------------------------------------------------------
// launchers
hipError_t launch_node_prep(const MirrorView& m, uint32_t n0, uint32_t n1, int64_t now, int32_t filter_expired,
                            int32_t has_exp, int64_t exp_ns, hipStream_t st) {
  if (n1 <= n0) return hipSuccess;
  uint32_t grid = (n1 - n0 + 255) / 256;
  hipLaunchKernelGGL(node_prep_kernel, dim3(grid), dim3(256), 0, st, m, n0, n1, now, filter_expired, has_exp, exp_ns,
                     nullptr);
  return hipGetLastError();
}

hipError_t launch_node_prep_idx(const MirrorView& m, const uint32_t* idx, uint32_t n, int64_t now, int32_t filter_expired,
                                int32_t has_exp, int64_t exp_ns, hipStream_t st) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(node_prep_kernel, dim3((n + 255) / 256), dim3(256), 0, st, m, 0u, n, now, filter_expired, has_exp,
                     exp_ns, idx);
  return hipGetLastError();
}

bool commit_cu_exclusive() {
  static const bool on = getenv("GS_COMMIT_EXCL") && atoi(getenv("GS_COMMIT_EXCL")) != 0;
  return on;
}

size_t eval_lds_bytes() { return commit_cu_exclusive() ? 256 : 0; }

hipError_t launch_eval(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t n0, uint32_t n1,
                       int16_t* S, uint32_t ld, int prod_cols, const uint32_t* numa_idx, uint32_t numa_n,
                       uint8_t* aff, hipStream_t st, hipStream_t st2, hipEvent_t fork, hipEvent_t join,
                       const MirrorView* slab) {
  uint32_t len = n1 - n0;
  uint32_t gx = (len + 255) / 256;
  uint32_t gy = (npods + PODS_PER_BLOCK - 1) / PODS_PER_BLOCK;
  if (gx == 0 || gy == 0) return hipSuccess;
  const size_t xl = eval_lds_bytes();
  if (pf.enabled & 0x30u) {
    // eval_kernel (nodes without a NUMA policy) and eval_numa_kernel write disjoint score entries: with a side
    // stream they run concurrently, eval_kernel's blocks filling the CUs eval_numa_kernel's low-occupancy waves
    // (and its tail) leave idle
    const bool side = st2 && fork && join && numa_n;
    hipError_t e;
    if (side) {
      if ((e = hipEventRecord(fork, st)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(st2, fork, 0)) != hipSuccess) return e;
    }
    // short batches: one pair per thread keeps the grid wide
    static const int ppt_env = getenv("GS_NUMA_PPT") ? atoi(getenv("GS_NUMA_PPT")) : NUMA_PPT;
    const int ppt = npods >= 32 ? ppt_env : 1;
    const dim3 g((numa_n + 255) / 256, (npods + ppt - 1) / ppt);
    // the slab pays once a row is read by several pod groups (full batches)
    MirrorView sv{nullptr, nullptr, 0};
    if (slab && slab->i64 && numa_n && npods >= 32) {
      sv = *slab;
      hipLaunchKernelGGL(gather_numa_kernel, dim3((numa_n + 255) / 256, SLAB64 + SLAB32), dim3(256), xl, st, m, sv,
                         numa_idx, numa_n);
    }
    // GS_NUMA_TILE=0 (experiments): the untiled grid
    // (GS_NUMA_TILE=2: tiled without the XCD numbering)
    static const int tile_mode = getenv("GS_NUMA_TILE") ? atoi(getenv("GS_NUMA_TILE")) : 1;
    const bool tile = tile_mode != 0;
    if (numa_n == 0) {
    } else if (tile && ppt == NUMA_PPT) {
      // pods per thread of the tiled kernel: 8 (GS_NUMA_TILE_PPT: 2, 4, 8). Tiled, 8 pods per thread: 337 us per pass
      // and 2.4 MB of reads; untiled (4): 241 us and 58.5 MB. The pass runs beside the previous batch's commit, which
      // it slows less when tiled: 182.8-183.7k vs 180.0-180.5k pods/s in three alternations
      static const int tppt = getenv("GS_NUMA_TILE_PPT") ? atoi(getenv("GS_NUMA_TILE_PPT")) : 8;
      const uint32_t ntiles8 = ((numa_n + 63) / 64 + 7) / 8 * 8;
      const uint32_t npr = (npods + NUMA_TWAVES * tppt - 1) / (NUMA_TWAVES * tppt);
      const int xm = tile_mode == 1 ? 1 : 0;
      if (tppt == 2)
        hipLaunchKernelGGL(eval_numa_tile_kernel<2>, dim3(ntiles8 * npr), dim3(64 * NUMA_TWAVES), xl, st, m, sv, pods,
                           npods, pf, numa_idx, numa_n, n0, S, ld, prod_cols, aff, npr, xm);
      else if (tppt == 8)
        hipLaunchKernelGGL(eval_numa_tile_kernel<8>, dim3(ntiles8 * npr), dim3(64 * NUMA_TWAVES), xl, st, m, sv, pods,
                           npods, pf, numa_idx, numa_n, n0, S, ld, prod_cols, aff, npr, xm);
      else
        hipLaunchKernelGGL(eval_numa_tile_kernel<NUMA_PPT>, dim3(ntiles8 * npr), dim3(64 * NUMA_TWAVES), xl, st, m, sv,
                           pods, npods, pf, numa_idx, numa_n, n0, S, ld, prod_cols, aff, npr, xm);
    } else if (ppt == 2) {
      hipLaunchKernelGGL(eval_numa_kernel<2>, g, dim3(256), xl, st, m, sv, pods, npods, pf, numa_idx, numa_n, n0, S, ld,
                         prod_cols, aff);
    } else if (ppt == 4) {
      hipLaunchKernelGGL(eval_numa_kernel<4>, g, dim3(256), xl, st, m, sv, pods, npods, pf, numa_idx, numa_n, n0, S, ld,
                         prod_cols, aff);
    } else if (ppt == 8) {
      hipLaunchKernelGGL(eval_numa_kernel<8>, g, dim3(256), xl, st, m, sv, pods, npods, pf, numa_idx, numa_n, n0, S, ld,
                         prod_cols, aff);
    } else {
      hipLaunchKernelGGL(eval_numa_kernel<1>, dim3((numa_n + 255) / 256, npods), dim3(256), xl, st, m, sv, pods, npods,
                         pf, numa_idx, numa_n, n0, S, ld, prod_cols, aff);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(eval_kernel<true>, dim3(gx, gy), dim3(256), xl, side ? st2 : st, m, pods, npods, pf, n0, n1, S,
                       ld, prod_cols);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (side) {
      if ((e = hipEventRecord(join, st2)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(st, join, 0)) != hipSuccess) return e;
    }
  } else {
    hipLaunchKernelGGL(eval_kernel<false>, dim3(gx, gy), dim3(256), xl, st, m, pods, npods, pf, n0, n1, S, ld, prod_cols);
  }
  return hipGetLastError();
}

hipError_t launch_patch(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t n0, uint32_t n1,
                        int16_t* S, uint32_t ld, int prod_cols, uint8_t* aff, const PlacementDev* prev_out,
                        const int32_t* prev_committed, int prev_npods, hipStream_t st) {
  if (prev_npods <= 0 || npods <= 0) return hipSuccess;
  // one lane per pair (default: 63 us per C3 batch); GS_PATCH_WAVE=1: one wave per pair (measured 91 us)
  static const bool wave = getenv("GS_PATCH_WAVE") && getenv("GS_PATCH_WAVE")[0] == '1';
  if (!wave)
    hipLaunchKernelGGL(patch_kernel, dim3(prev_npods), dim3(128), 0, st, m, pods, npods, pf, n0, n1, S, ld, prod_cols,
                       aff, prev_out, prev_committed);
  else
    hipLaunchKernelGGL(patch_wave_kernel, dim3(prev_npods, (npods + PW_PODS - 1) / PW_PODS), dim3(64 * PW_PODS), 0, st,
                       m, pods, npods, pf, n0, n1, S, ld, prod_cols, aff, prev_out, prev_committed);
  return hipGetLastError();
}

hipError_t launch_eval_full(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t N,
                            int16_t* scores, uint16_t* codes, int16_t* plugin, int prod_cols, hipStream_t st) {
  uint32_t grid = (N + 255) / 256;
  hipLaunchKernelGGL(eval_full_kernel, dim3(grid), dim3(256), 0, st, m, pods, npods, pf, N, scores, codes, plugin,
                     prod_cols);
  return hipGetLastError();
}

static size_t cand_smem_bytes(int max_score, int waves) {
  size_t nb = (size_t)max_score + 1;
  return nb * 4 * waves + nb * 4 + ((nb + 15) & ~(size_t)15);
}
// The 16-wave variant measured slower on MI355X (its serial level scan walks 4x more segments): kept for
// experiments, not selected.
static bool cand_wide(int max_score) {
  static const int env = getenv("GS_CAND_WIDE") ? atoi(getenv("GS_CAND_WIDE")) : 0;
  return env == 1 && cand_smem_bytes(max_score, 16) <= 48 * 1024;
}

static uint64_t* g_cand_stamps = nullptr;
void set_cand_stamps(uint64_t* p) { g_cand_stamps = p; }

hipError_t launch_fix_levels(int16_t* S, uint32_t ld, int npods, int max_score, int lcap, uint32_t* lists,
                             LevelHdr* hdrs, LevelExt* ext, const CandPatch& cp, hipStream_t st) {
  if (lcap < 1 || lcap > LCAP || !cp.hist || max_score < 0 || max_score > MAX_SCORE_LIMIT || npods > MAX_BATCH)
    return hipErrorInvalidValue;
  const size_t smem = ((size_t)max_score + 1 + (size_t)lcap) * 4 + (size_t)max_score + 1;
  hipLaunchKernelGGL(fix_levels_kernel, dim3(npods), dim3(FIX_THREADS), smem, st, S, ld, max_score, lcap, lists, hdrs, ext,
                     cp, g_cand_stamps);
  return hipGetLastError();
}


size_t cand_split_scratch_bytes() {
  return (size_t)4 * CS_MAXB * CS_GMAX * (MAX_SCORE_LIMIT + 1 + LEVALL);
}

hipError_t launch_cand(int16_t* S, uint32_t ld, uint32_t len, uint32_t n0, int npods, int max_score, int lcap,
                       uint32_t* lists, LevelHdr* hdrs, LevelExt* ext, hipStream_t st, const CandPatch* patch,
                       uint32_t* split_scratch) {
  if (lcap < 1 || lcap > LCAP) return hipErrorInvalidValue;
  CandPatch cp{};
  if (patch) cp = *patch;
  static const bool no_split = getenv("GS_CAND_SPLIT") && getenv("GS_CAND_SPLIT")[0] == '0';
  const uint32_t lenv = (len + 511) & ~511u;
  if (split_scratch && !no_split && !cp.on && !cp.hist && cp.extra == 0 && !g_cand_stamps && npods >= 1 &&
      npods <= CS_MAXB && max_score >= 0 && max_score <= MAX_SCORE_LIMIT && lenv >= 2 * 2048) {
    // slices of whole 2048-entry steps, at most CS_GMAX of them (rows are padded with -1 up to ld >= lenv)
    const uint32_t g0 = min((uint32_t)CS_GMAX, (lenv + 2047) / 2048);
    const uint32_t slice = ((lenv + g0 - 1) / g0 + 2047) & ~2047u;
    const int G = (int)((lenv + slice - 1) / slice);
    const int nbins = max_score + 1;
    uint32_t* ghist = split_scratch;
    uint32_t* offs = split_scratch + (size_t)CS_MAXB * CS_GMAX * (MAX_SCORE_LIMIT + 1);
    hipLaunchKernelGGL(cs_hist_kernel, dim3(G, npods), dim3(256), (size_t)4 * nbins, st, S, ld, lenv, nbins, slice, G,
                       ghist);
    hipLaunchKernelGGL(cs_pick_kernel, dim3(npods), dim3(256), (size_t)4 * nbins, st, ghist, nbins, G, lcap, offs, hdrs,
                       ext);
    hipLaunchKernelGGL(cs_list_kernel, dim3(G, npods), dim3(64), ((size_t)nbins + 15) & ~(size_t)15, st, S, ld, lenv,
                       n0, nbins, slice, G, lcap, offs, hdrs, ext, lists);
    return hipGetLastError();
  }
  if (cand_wide(max_score))
    hipLaunchKernelGGL(cand_kernel<16>, dim3(npods), dim3(1024), cand_smem_bytes(max_score, 16), st, S, ld, len, n0,
                       max_score, lcap, lists, hdrs, ext, g_cand_stamps, cp);
  else
    hipLaunchKernelGGL(cand_kernel<4>, dim3(npods), dim3(256), cand_smem_bytes(max_score, 4), st, S, ld, len, n0,
                       max_score, lcap, lists, hdrs, ext, g_cand_stamps, cp);
  return hipGetLastError();
}

size_t commit_smem_bytes(int B) {
  size_t b = (size_t)B * POD_STRIDE + (size_t)B * sizeof(Row) + (size_t)B * B * 2 * 2;
  b = (b + 15) & ~(size_t)15;
  b += (size_t)HASH * 8 + 16;
  b += (size_t)B * sizeof(CpuStateDev);
  return b;
}

// The speculative commit kernel runs every batch except under node sampling, whose rotation window is resolved by
// commit_kernel (one shard).
bool commit_spec_selected(uint32_t window_k) { return !window_k; }

hipError_t launch_commit(const CommitArgs& a, hipStream_t st) {
  // several shards: the speculative kernel reads the merged levels (launch_merge_levels)
  if (commit_spec_selected(a.window_k)) return launch_commit_spec(a, st);
  if (a.stamps)
    hipLaunchKernelGGL(commit_kernel<true>, dim3(1), dim3(COMMIT_THREADS), commit_smem_bytes(a.npods), st, a);
  else
    hipLaunchKernelGGL(commit_kernel<false>, dim3(1), dim3(COMMIT_THREADS), commit_smem_bytes(a.npods), st, a);
  return hipGetLastError();
}

hipError_t launch_row_stats(const int16_t* S, uint32_t len, RowStat* out, hipStream_t st) {
  hipLaunchKernelGGL(row_stats_kernel, dim3(1), dim3(1024), 0, st, S, len, out);
  return hipGetLastError();
}

hipError_t launch_row_select(const int16_t* S, uint32_t len, int score, int64_t target, uint32_t n0, int32_t* out,
                             hipStream_t st) {
  hipLaunchKernelGGL(row_select_kernel, dim3(1), dim3(1024), 0, st, S, len, score, target, n0, out);
  return hipGetLastError();
}

hipError_t launch_scatter_rows(const MirrorView& m, const uint32_t* idx, const int64_t* rows, uint32_t nrows,
                               hipStream_t st, const ScatterPrep* prep) {
  if (!nrows) return hipSuccess;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((nrows + 255) / 256), dim3(256), 0, st, m, idx, rows, nrows,
                     prep ? 1 : 0, prep ? prep->now : 0, prep ? prep->filter_expired : 0, prep ? prep->has_exp : 0,
                     prep ? prep->exp_ns : 0);
  return hipGetLastError();
}

hipError_t set_kernel_attributes() {
  hipError_t e = set_commit_spec_attributes();
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(commit_kernel<false>),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)commit_smem_bytes(MAX_BATCH));
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(commit_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)commit_smem_bytes(MAX_BATCH));
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(cand_kernel<16>), hipFuncAttributeMaxDynamicSharedMemorySize,
                          48 * 1024);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(cand_kernel<4>), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)cand_smem_bytes(MAX_SCORE_LIMIT, 4));
}

}  // namespace gs
