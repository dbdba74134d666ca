// gs_kernels.hip — CDNA4 (gfx950) kernels of the batched Filter/Score engine.
//
//   node_prep_kernel   per batch, O(N): LoadAware expiry against `now` -> dynamic filter/score flags
//   eval_kernel        the hot kernel: B pods x shard nodes, fused Fit filter + LoadAware filter +
//                      Fit LeastAllocated score + LoadAware score + weighted sum -> int16 score rows
//   cand_kernel        per pod: histogram -> threshold -> compaction -> bitonic sort -> candidate list
//   commit_kernel      one wave: sequential selectHost + assume/Reserve deltas over the batch, with
//                      exact re-scoring of the nodes earlier pods of the batch landed on
//   row_stats_kernel / row_select_kernel   exact full-row path (massive ties)
//   scatter_rows_kernel   host -> HBM delta rows (AoS staging -> SoA columns)
//
// Integer semantics follow Go: int64 two's complement, truncating division. The three float64 spots
// of the reference (LoadAware filter %, estimator scaling, amplification) are host-side per node /
// per pod (PreFilter / mirror update); the per-pair work here is pure int64 with an exact
// reciprocal-estimate-plus-correction division (quotients are in [0,100]).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_kernels.h"

namespace gs {

// ------------------------------------------------------------------------------------------------
// exact floor((x*100)/cap) for 0 <= x <= cap, cap > 0, x*100 < 2^63
__device__ __forceinline__ float u64_to_f32(uint64_t v) {
  return (float)(uint32_t)(v >> 32) * 4294967296.0f + (float)(uint32_t)v;
}

__device__ __forceinline__ int32_t pct_floor(int64_t x, int64_t cap) {
  int64_t num = x * 100;
  float qf = u64_to_f32((uint64_t)num) * __builtin_amdgcn_rcpf(u64_to_f32((uint64_t)cap));
  int32_t q = (int32_t)qf;
  q = q > 100 ? 100 : q;
  int64_t prod = (int64_t)q * cap;
  if (prod > num) --q;                  // estimate one too high
  else if (prod + cap <= num) ++q;      // estimate one too low
  return q;
}

// leastRequestedScore(requested, capacity) with requested = capacity - free + p  (load_aware.go:388-397,
// [upstream] least_allocated.go): capacity == 0 -> 0; requested > capacity -> 0.
__device__ __forceinline__ int32_t least_requested(int64_t free, int64_t p, int64_t cap) {
  if (cap == 0) return 0;
  int64_t x = free - p;
  if (x < 0) return 0;
  return pct_floor(x, cap);
}

// exact a / b for 0 <= a < 2^24, 1 <= b < 2^24 (weighted-mean divisions)
__device__ __forceinline__ int32_t small_div(int32_t a, int32_t b) {
  int32_t q = (int32_t)((float)a * __builtin_amdgcn_rcpf((float)b));
  if (q * b > a) --q;
  else if ((q + 1) * b <= a) ++q;
  return q;
}

// node row as held in registers by the filter+score kernel
struct Row {
  int64_t free[3];      // cpu, mem, eph
  int64_t alloc[2];     // cpu, mem
  int64_t nzfree[2];
  int64_t la_cap[2];
  int64_t la_free[2];
  int64_t la_pfree[2];
  int32_t free_pods;
  uint32_t dflags;
  uint32_t node;        // global index
};

__device__ __forceinline__ void load_row(const MirrorView& m, uint32_t i, bool prod_cols, Row& r) {
  r.free[0] = m.i64[C_FREE_CPU][i];
  r.free[1] = m.i64[C_FREE_MEM][i];
  r.free[2] = m.i64[C_FREE_EPH][i];
  r.alloc[0] = m.i64[C_ALLOC_CPU][i];
  r.alloc[1] = m.i64[C_ALLOC_MEM][i];
  r.nzfree[0] = m.i64[C_NZFREE_CPU][i];
  r.nzfree[1] = m.i64[C_NZFREE_MEM][i];
  r.la_cap[0] = m.i64[C_LA_CAP_CPU][i];
  r.la_cap[1] = m.i64[C_LA_CAP_MEM][i];
  r.la_free[0] = m.i64[C_LA_FREE_CPU][i];
  r.la_free[1] = m.i64[C_LA_FREE_MEM][i];
  if (prod_cols) {
    r.la_pfree[0] = m.i64[C_LA_PFREE_CPU][i];
    r.la_pfree[1] = m.i64[C_LA_PFREE_MEM][i];
  } else {
    r.la_pfree[0] = r.la_pfree[1] = 0;
  }
  r.free_pods = m.i32[C_FREE_PODS][i];
  r.dflags = (uint32_t)m.i32[C_DFLAGS][i];
  r.node = i;
}

struct PairOut {
  uint32_t code;
  int32_t fit, la;
};

// Filter (Fit + LoadAware) and Score (Fit LeastAllocated + LoadAware) of one pod on one node.
template <bool FULL>
__device__ __forceinline__ PairOut eval_pair(const Row& r, const PodVec& p, const Profile& pf, const MirrorView& m) {
  PairOut o{0u, 0, 0};
  // ---- [upstream] noderesources Fit.Filter -> fitsRequest
  if (pf.enabled & 0x1u) {
    if (r.free_pods < 1) o.code |= 0x01u;                               // len(Pods)+1 > AllowedPodNumber
    if (!(p.flags & PF_ALL_ZERO)) {
      if (p.req[0] > r.free[0]) o.code |= 0x02u;
      if (p.req[1] > r.free[1]) o.code |= 0x04u;
      if (p.req[2] > r.free[2]) o.code |= 0x08u;
      if (p.scalar_mask) {
        for (int s = 3; s < 7; ++s)
          if ((p.scalar_mask & (1u << s)) && p.req[s] > m.i64[C_FREE_EPH + s - 2][r.node]) o.code |= 0x10u;
      }
    }
  }
  // ---- LoadAware.Filter (load_aware.go:123-171), usage verdicts precomputed per node
  if ((pf.enabled & 0x4u) && !(p.flags & PF_DAEMONSET)) {
    uint32_t bit = (p.flags & PF_PROD) ? DF_LA_FAIL_P : DF_LA_FAIL_NP;
    if (r.dflags & bit) o.code |= 0x20u;
  }
  if (!FULL && o.code) return o;
  // ---- Fit.Score, LeastAllocated over NonZeroRequested ([upstream] resource_allocation.go)
  if (pf.enabled & 0x2u) {
    int32_t ns = 0, ws = 0;
    if (pf.fit_w[0] && r.alloc[0] != 0) {
      ns += least_requested(r.nzfree[0], p.nz[0], r.alloc[0]) * pf.fit_w[0];
      ws += pf.fit_w[0];
    }
    if (pf.fit_w[1] && r.alloc[1] != 0) {
      ns += least_requested(r.nzfree[1], p.nz[1], r.alloc[1]) * pf.fit_w[1];
      ws += pf.fit_w[1];
    }
    if (pf.fit_scalar_w_mask) {
      for (int s = 2; s < 7; ++s) {
        if (!(pf.fit_scalar_w_mask & (1u << s))) continue;
        int64_t preq = p.req[s];
        if (s >= 3 && preq == 0) continue;                              // un-requested scalar: bypass
        int64_t cap = m.i64[C_ALLOC_CPU + s][r.node];
        if (cap == 0) continue;
        ns += least_requested(m.i64[C_FREE_CPU + s][r.node], preq, cap) * pf.fit_w[s];
        ws += pf.fit_w[s];
      }
    }
    o.fit = ws ? small_div(ns, ws) : 0;
  }
  // ---- LoadAware.Score (load_aware.go:269-335): est + la_used vs EstimateNode
  if ((pf.enabled & 0x8u) && !(r.dflags & DF_LA_ZERO)) {
    bool prod = p.flags & PF_PROD_SCORE;
    int32_t ns = 0;
    if (pf.la_w[0]) ns += least_requested(prod ? r.la_pfree[0] : r.la_free[0], p.est[0], r.la_cap[0]) * pf.la_w[0];
    if (pf.la_w[1]) ns += least_requested(prod ? r.la_pfree[1] : r.la_free[1], p.est[1], r.la_cap[1]) * pf.la_w[1];
    o.la = small_div(ns, pf.la_wsum);
  }
  return o;
}

__device__ __forceinline__ int32_t total_score(const PairOut& o, const Profile& pf) {
  if (o.code) return -1;
  return o.fit * pf.w_fit + o.la * pf.w_la;
}

// ------------------------------------------------------------------------------------------------
// node-prep: LoadAware expiry (helper.go:36-41) evaluated at `now` for every node of the shard.
__global__ void __launch_bounds__(256) node_prep_kernel(MirrorView m, uint32_t n0, uint32_t n1, int64_t now,
                                                        int32_t filter_expired, int32_t has_exp, int64_t exp_ns) {
  uint32_t i = n0 + blockIdx.x * 256 + threadIdx.x;
  if (i >= n1) return;
  uint32_t sf = (uint32_t)m.i32[C_SFLAGS][i];
  bool exists = sf & SF_METRIC;
  bool expired = !exists || !(sf & SF_UPDATE_TIME) || (exp_ns > 0 && now - m.i64[C_UPDATE_TIME][i] >= exp_ns);
  bool skip_filter = !exists || (filter_expired && has_exp && expired);
  uint32_t df = 0;
  if (!skip_filter) {
    if (sf & SF_FAIL_NP) df |= DF_LA_FAIL_NP;
    if ((sf & SF_PROD_THR) ? (sf & SF_FAIL_P) : (sf & SF_FAIL_NP)) df |= DF_LA_FAIL_P;
  }
  if (!exists || (has_exp && expired)) df |= DF_LA_ZERO;
  m.i32[C_DFLAGS][i] = (int32_t)df;
}

// ------------------------------------------------------------------------------------------------
// The hot kernel. Block = 256 threads x NPT nodes; every thread keeps its NPT node rows in registers
// and sweeps all B pods (pod vectors are wave-uniform: scalar loads), writing one int16 score per
// (pod,node): coalesced NPT*2-byte stores per lane, one contiguous row segment per pod.
constexpr int NPT = 2;

__global__ void __launch_bounds__(256) eval_kernel(MirrorView m, const PodVec* __restrict__ pods, int npods,
                                                   Profile pf, uint32_t n0, uint32_t n1, int16_t* __restrict__ S,
                                                   uint32_t ld, int prod_cols) {
  uint32_t local = (blockIdx.x * 256 + threadIdx.x) * NPT;
  uint32_t len = n1 - n0;
  Row row[NPT];
  bool ok[NPT];
#pragma unroll
  for (int j = 0; j < NPT; ++j) {
    ok[j] = local + j < len;
    load_row(m, ok[j] ? n0 + local + j : n0, prod_cols, row[j]);
  }
  if (local >= ld) return;
  for (int k = 0; k < npods; ++k) {
    const PodVec& p = pods[k];
    int16_t out[NPT];
#pragma unroll
    for (int j = 0; j < NPT; ++j) {
      PairOut o = eval_pair<false>(row[j], p, pf, m);
      out[j] = ok[j] ? (int16_t)total_score(o, pf) : (int16_t)-1;
    }
    uint32_t packed = (uint32_t)(uint16_t)out[0] | ((uint32_t)(uint16_t)out[1] << 16);
    *reinterpret_cast<uint32_t*>(S + (size_t)k * ld + local) = packed;
  }
}

// Diagnostic variant (gs_evaluate): every plugin's verdict and score for every pair.
__global__ void __launch_bounds__(256) eval_full_kernel(MirrorView m, const PodVec* __restrict__ pods, int npods,
                                                        Profile pf, uint32_t N, int16_t* scores, uint16_t* codes,
                                                        int16_t* plugin, int prod_cols) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N) return;
  Row r;
  load_row(m, i, prod_cols, r);
  for (int k = 0; k < npods; ++k) {
    PairOut o = eval_pair<true>(r, pods[k], pf, m);
    size_t off = (size_t)k * N + i;
    if (scores) scores[off] = (int16_t)total_score(o, pf);
    if (codes) codes[off] = (uint16_t)o.code;
    if (plugin) {
      plugin[off * 2 + 0] = (int16_t)o.fit;
      plugin[off * 2 + 1] = (int16_t)o.la;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Candidate extraction: one block per pod row of the shard.
constexpr int CAND_THREADS = 256;

__global__ void __launch_bounds__(CAND_THREADS) cand_kernel(const int16_t* __restrict__ S, uint32_t ld, uint32_t len,
                                                            uint32_t n0, int max_score, uint64_t* __restrict__ lists,
                                                            CandHdr* __restrict__ hdrs) {
  extern __shared__ __align__(16) uint32_t smem[];
  const int nbins = max_score + 1;
  uint32_t* hist = smem;                                             // nbins
  uint64_t* keys = reinterpret_cast<uint64_t*>(smem + ((nbins + 3) & ~3));  // CAND_CAP
  __shared__ uint32_t seg[CAND_THREADS];
  __shared__ int32_t s_theta, s_count, s_feasible;
  const int k = blockIdx.x;
  const int t = threadIdx.x;
  const int16_t* row = S + (size_t)k * ld;
  for (int b = t; b < nbins; b += CAND_THREADS) hist[b] = 0;
  __syncthreads();
  // pass 1: histogram of feasible scores (16-B loads: 8 scores per lane)
  uint32_t nvec = len / 8;
  for (uint32_t v = t; v < nvec; v += CAND_THREADS) {
    int4 q = reinterpret_cast<const int4*>(row)[v];
    const int16_t* e = reinterpret_cast<const int16_t*>(&q);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (e[j] >= 0) atomicAdd(&hist[e[j]], 1u);
  }
  for (uint32_t i = nvec * 8 + t; i < len; i += CAND_THREADS)
    if (row[i] >= 0) atomicAdd(&hist[row[i]], 1u);
  __syncthreads();
  // threshold: smallest level theta with count(score >= theta) <= CAND_CAP
  int per = (nbins + CAND_THREADS - 1) / CAND_THREADS;
  {
    uint32_t s = 0;
    for (int b = t * per; b < min(nbins, (t + 1) * per); ++b) s += hist[b];
    seg[t] = s;
  }
  __syncthreads();
  if (t == 0) {
    uint32_t total = 0;
    for (int i = 0; i < CAND_THREADS; ++i) total += seg[i];
    uint32_t cum = 0;
    int theta = 0;
    if (total <= (uint32_t)CAND_CAP) {
      cum = total;                                 // every feasible node fits: complete list
    } else {
      theta = nbins;
      bool stop = false;
      for (int i = CAND_THREADS - 1; i >= 0 && !stop; --i) {
        if (cum + seg[i] <= (uint32_t)CAND_CAP) {  // whole segment fits
          cum += seg[i];
          if (i * per < theta) theta = i * per;
          continue;
        }
        for (int b = min(nbins, (i + 1) * per) - 1; b >= i * per; --b) {
          if (cum + hist[b] > (uint32_t)CAND_CAP) break;
          cum += hist[b];
          theta = b;
        }
        stop = true;
      }
    }
    s_theta = theta;
    s_count = 0;
    s_feasible = (int32_t)total;
  }
  __syncthreads();
  const int theta = s_theta;
  // pass 2: compaction of score >= theta
  for (uint32_t v = t; v < nvec; v += CAND_THREADS) {
    int4 q = reinterpret_cast<const int4*>(row)[v];
    const int16_t* e = reinterpret_cast<const int16_t*>(&q);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (e[j] >= 0 && e[j] >= theta) {
        int pos = atomicAdd(&s_count, 1);
        keys[pos] = cand_key(e[j], n0 + v * 8 + j);
      }
    }
  }
  for (uint32_t i = nvec * 8 + t; i < len; i += CAND_THREADS) {
    int16_t e = row[i];
    if (e >= 0 && e >= theta) {
      int pos = atomicAdd(&s_count, 1);
      keys[pos] = cand_key(e, n0 + i);
    }
  }
  __syncthreads();
  const int cnt = s_count;
  for (int i = cnt + t; i < CAND_CAP; i += CAND_THREADS) keys[i] = 0;
  __syncthreads();
  // bitonic sort, descending
  for (int size = 2; size <= CAND_CAP; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = t; i < CAND_CAP; i += CAND_THREADS) {
        int jx = i ^ stride;
        if (jx > i) {
          bool desc = ((i & size) == 0);
          uint64_t a = keys[i], b = keys[jx];
          if (desc ? (a < b) : (a > b)) { keys[i] = b; keys[jx] = a; }
        }
      }
      __syncthreads();
    }
  }
  uint64_t* out = lists + (size_t)k * CAND_CAP;
  for (int i = t; i < cnt; i += CAND_THREADS) out[i] = keys[i];
  if (t == 0) {
    CandHdr h;
    h.count = cnt;
    h.theta = theta;
    h.complete = (cnt == s_feasible) ? 1 : 0;
    h.feasible = s_feasible;
    hdrs[k] = h;
  }
}

// ------------------------------------------------------------------------------------------------
// selectHost tie-break: position (1-based, in feasible order) of the selected node among T max ties.
// Same stream as oracle/oracle.cpp TieBreakRand: R = {1, floor(j/U_0)+1, ...}; answer = max R ∩ [1,T].
__host__ __device__ inline uint64_t mix64(uint64_t x) {
  uint64_t z = x + 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__host__ __device__ inline int64_t tiebreak_position(uint64_t seed, uint64_t seq, int64_t T) {
  uint64_t key = mix64(seed ^ mix64(seq));
  int64_t j = 1;
  for (uint64_t i = 0;; ++i) {
    uint64_t h = mix64(key + i);
    double u = (double)((h >> 11) + 1) * 0x1.0p-53;
    double x = (double)j / u;
    if (!(x < 4.0e18)) break;
    int64_t jn = (int64_t)floor(x) + 1;
    if (jn > T) break;
    j = jn;
  }
  return j;
}

int64_t host_tiebreak_position(uint64_t seed, uint64_t seq, int64_t T) { return tiebreak_position(seed, seq, T); }

// ------------------------------------------------------------------------------------------------
// Sequential commit (one wave). For pod k of the batch: effective scores = candidate lists (snapshot
// at batch start) for clean nodes + exact re-scores (dsc) for nodes earlier pods landed on. Valid while
// the max effective score is >= every incomplete list's threshold; otherwise the batch is cut at k.
constexpr int HASH = 512;

struct __align__(16) DRow {
  int64_t free[7];
  int64_t alloc[2];
  int64_t nzfree[2];
  int64_t la_cap[2];
  int64_t la_free[2];
  int64_t la_pfree[2];
  int32_t free_pods;
  uint32_t dflags;
  uint32_t node;
  uint32_t pad;
};

__device__ __forceinline__ void drow_load(const MirrorView& m, uint32_t i, DRow& d) {
  for (int s = 0; s < 7; ++s) d.free[s] = m.i64[C_FREE_CPU + s][i];
  d.alloc[0] = m.i64[C_ALLOC_CPU][i];
  d.alloc[1] = m.i64[C_ALLOC_MEM][i];
  d.nzfree[0] = m.i64[C_NZFREE_CPU][i];
  d.nzfree[1] = m.i64[C_NZFREE_MEM][i];
  d.la_cap[0] = m.i64[C_LA_CAP_CPU][i];
  d.la_cap[1] = m.i64[C_LA_CAP_MEM][i];
  d.la_free[0] = m.i64[C_LA_FREE_CPU][i];
  d.la_free[1] = m.i64[C_LA_FREE_MEM][i];
  d.la_pfree[0] = m.i64[C_LA_PFREE_CPU][i];
  d.la_pfree[1] = m.i64[C_LA_PFREE_MEM][i];
  d.free_pods = m.i32[C_FREE_PODS][i];
  d.dflags = (uint32_t)m.i32[C_DFLAGS][i];
  d.node = i;
}

__device__ __forceinline__ void drow_to_row(const DRow& d, Row& r) {
  r.free[0] = d.free[0]; r.free[1] = d.free[1]; r.free[2] = d.free[2];
  r.alloc[0] = d.alloc[0]; r.alloc[1] = d.alloc[1];
  r.nzfree[0] = d.nzfree[0]; r.nzfree[1] = d.nzfree[1];
  r.la_cap[0] = d.la_cap[0]; r.la_cap[1] = d.la_cap[1];
  r.la_free[0] = d.la_free[0]; r.la_free[1] = d.la_free[1];
  r.la_pfree[0] = d.la_pfree[0]; r.la_pfree[1] = d.la_pfree[1];
  r.free_pods = d.free_pods; r.dflags = d.dflags; r.node = d.node;
}

// eval_pair reads scalar free columns from the mirror for scalar-requesting pods: in the commit those
// must come from the LDS row, so the commit uses this wrapper with a mirror view onto a 1-row table.
__device__ __forceinline__ int32_t drow_score(const DRow& d, const PodVec& p, const Profile& pf, const MirrorView& m) {
  Row r;
  drow_to_row(d, r);
  PairOut o;
  if (p.scalar_mask || pf.fit_scalar_w_mask) {
    // slow generic path: evaluate against the LDS copy for scalar columns
    o = PairOut{0u, 0, 0};
    if (pf.enabled & 0x1u) {
      if (d.free_pods < 1) o.code |= 0x01u;
      if (!(p.flags & PF_ALL_ZERO)) {
        for (int s = 0; s < 7; ++s) {
          bool chk = s < 3 || (p.scalar_mask & (1u << s));
          if (chk && p.req[s] > d.free[s]) o.code |= (s < 3) ? (0x02u << s) : 0x10u;
        }
      }
    }
    if ((pf.enabled & 0x4u) && !(p.flags & PF_DAEMONSET)) {
      uint32_t bit = (p.flags & PF_PROD) ? DF_LA_FAIL_P : DF_LA_FAIL_NP;
      if (d.dflags & bit) o.code |= 0x20u;
    }
    if (o.code) return -1;
    if (pf.enabled & 0x2u) {
      int32_t ns = 0, ws = 0;
      for (int s = 0; s < 7; ++s) {
        if (!pf.fit_w[s]) continue;
        int64_t preq, cap, fr;
        if (s < 2) { preq = p.nz[s]; cap = d.alloc[s]; fr = d.nzfree[s]; }
        else {
          preq = p.req[s];
          if (s >= 3 && preq == 0) continue;
          cap = m.i64[C_ALLOC_CPU + s][d.node];
          fr = d.free[s];
        }
        if (cap == 0) continue;
        ns += least_requested(fr, preq, cap) * pf.fit_w[s];
        ws += pf.fit_w[s];
      }
      o.fit = ws ? small_div(ns, ws) : 0;
    }
    if ((pf.enabled & 0x8u) && !(d.dflags & DF_LA_ZERO)) {
      bool prod = p.flags & PF_PROD_SCORE;
      int32_t ns = 0;
      if (pf.la_w[0]) ns += least_requested(prod ? d.la_pfree[0] : d.la_free[0], p.est[0], d.la_cap[0]) * pf.la_w[0];
      if (pf.la_w[1]) ns += least_requested(prod ? d.la_pfree[1] : d.la_free[1], p.est[1], d.la_cap[1]) * pf.la_w[1];
      o.la = small_div(ns, pf.la_wsum);
    }
    return total_score(o, pf);
  }
  o = eval_pair<false>(r, p, pf, m);
  return total_score(o, pf);
}

__device__ __forceinline__ int wave_max(int v) {
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}
__device__ __forceinline__ int key_score(uint64_t key) { return (int)(uint32_t)(key >> 32); }
__device__ __forceinline__ uint32_t key_node(uint64_t key) { return ~(uint32_t)key; }

__global__ void __launch_bounds__(64) commit_kernel(CommitArgs a) {
  extern __shared__ __align__(16) unsigned char cm[];
  const int B = a.npods;
  const int lane = threadIdx.x;
  // LDS carve
  PodVec* pods = reinterpret_cast<PodVec*>(cm);                         // B
  DRow* drows = reinterpret_cast<DRow*>(pods + B);                      // B (dirty slots)
  int16_t* dsc = reinterpret_cast<int16_t*>(drows + B);                 // B x B  [pod][slot]
  uint8_t* dof = reinterpret_cast<uint8_t*>(dsc + B * B);               // B x B  old feasibility
  int32_t* hkey = reinterpret_cast<int32_t*>(dof + ((B * B + 15) & ~15));  // HASH
  int32_t* hval = hkey + HASH;                                          // HASH
  uint32_t* ties = reinterpret_cast<uint32_t*>(hval + HASH);            // CAND_CAP * R + B
  const int tie_cap = CAND_CAP * a.nranks + B;
  uint32_t* dties = ties + tie_cap;                                     // B
  __shared__ int s_nd;

  for (int i = lane; i < B; i += 64) pods[i] = a.pods[i];
  for (int i = lane; i < HASH; i += 64) { hkey[i] = -1; hval[i] = -1; }
  if (lane == 0) s_nd = 0;
  __syncthreads();
  const MirrorView& m = a.m;
  int committed = B;

  auto lookup = [&](uint32_t node) -> int {
    uint32_t h = (node * 2654435761u) & (HASH - 1);
    for (int probe = 0; probe < HASH; ++probe) {
      int kk = hkey[h];
      if (kk == (int)node) return hval[h];
      if (kk < 0) return -1;
      h = (h + 1) & (HASH - 1);
    }
    return -1;
  };

  for (int k = 0; k < B; ++k) {
    const int nd = s_nd;
    const PodVec& pk = pods[k];
    // ---- dirty nodes: exact current scores for pod k
    int Md = -1;
    for (int s = lane; s < nd; s += 64) Md = max(Md, (int)dsc[k * B + s]);
    Md = wave_max(Md);
    // ---- clean heads of every shard's list
    int Mnd = -1;
    int first_r[8];
    bool valid = true;
    for (int r = 0; r < a.nranks; ++r) {
      const CandHdr h = a.hdrs[(size_t)r * a.hdr_stride + k];
      const uint64_t* L = a.lists + ((size_t)r * a.list_stride + (size_t)k) * CAND_CAP;
      int first = h.count;
      for (int c = 0; c < h.count; c += 64) {
        int i = c + lane;
        bool clean = false;
        if (i < h.count) clean = lookup(key_node(L[i])) < 0;
        uint64_t bal = __ballot(clean);
        if (bal) { first = c + __ffsll((long long)bal) - 1; break; }
      }
      first_r[r] = first;
      if (first < h.count) Mnd = max(Mnd, key_score(L[first]));
    }
    int M = max(Mnd, Md);
    if (a.forced_node >= 0 && k == 0) {
      // pod 0 resolved by the exact full-row path
    } else {
      for (int r = 0; r < a.nranks; ++r) {
        const CandHdr h = a.hdrs[(size_t)r * a.hdr_stride + k];
        if (!h.complete && M < h.theta) valid = false;
      }
      if (!valid) { committed = k; break; }
    }
    // feasible count: snapshot count, corrected for re-scored nodes
    int F = 0;
    for (int r = 0; r < a.nranks; ++r) F += a.hdrs[(size_t)r * a.hdr_stride + k].feasible;
    {
      int d = 0;
      for (int s = lane; s < nd; s += 64) d += (dsc[k * B + s] >= 0 ? 1 : 0) - (int)dof[k * B + s];
      F += wave_sum(d);
    }
    int64_t T = 0;
    uint32_t winner = 0xffffffffu;
    if (a.forced_node >= 0 && k == 0) {
      winner = (uint32_t)a.forced_node;
      M = a.forced_score;
      T = a.forced_ties;
      F = a.forced_feasible;
    } else if (M >= 0) {
      // ---- clean ties at level M, shard order == node order
      int nt = 0;
      for (int r = 0; r < a.nranks; ++r) {
        const CandHdr h = a.hdrs[(size_t)r * a.hdr_stride + k];
        const uint64_t* L = a.lists + ((size_t)r * a.list_stride + (size_t)k) * CAND_CAP;
        int first = first_r[r];
        if (first >= h.count || key_score(L[first]) != M) continue;
        for (int c = first; c < h.count; c += 64) {
          int i = c + lane;
          bool in = false, clean = false;
          uint32_t node = 0;
          if (i < h.count) {
            uint64_t key = L[i];
            in = key_score(key) == M;
            node = key_node(key);
            clean = in && lookup(node) < 0;
          }
          uint64_t bal = __ballot(clean);
          int pos = __popcll(bal & ((1ull << lane) - 1ull));
          if (clean && nt + pos < tie_cap) ties[nt + pos] = node;
          nt += __popcll(bal);
          uint64_t inb = __ballot(in);
          uint64_t valid_lanes = __ballot(i < h.count);
          if (inb != valid_lanes) break;
        }
      }
      // ---- dirty ties
      int ndt = 0;
      for (int s0 = 0; s0 < nd; s0 += 64) {
        int s = s0 + lane;
        bool in = s < nd && dsc[k * B + s] == M;
        uint64_t bal = __ballot(in);
        int pos = __popcll(bal & ((1ull << lane) - 1ull));
        if (in) dties[ndt + pos] = drows[s].node;
        ndt += __popcll(bal);
      }
      __syncthreads();
      T = nt + ndt;
      int64_t jstar = tiebreak_position(a.seed, a.seq[k], T);   // uniform across lanes
      // ---- j*-th in node order of (clean ties, sorted) U (dirty ties, unsorted)
      // clean tie i: position = i + 1 + #dirty ties with smaller node
      for (int i0 = 0; i0 < nt; i0 += 64) {
        int i = i0 + lane;
        bool hit = false;
        uint32_t node = 0;
        if (i < nt) {
          node = ties[i];
          int less = 0;
          for (int d = 0; d < ndt; ++d) less += dties[d] < node;
          hit = (int64_t)(i + 1 + less) == jstar;
        }
        uint64_t bal = __ballot(hit);
        if (bal) { winner = __shfl(node, __ffsll((long long)bal) - 1); break; }
      }
      if (winner == 0xffffffffu) {
        // dirty tie d: position = #clean ties with smaller node + #dirty ties with smaller node + 1
        for (int d0 = 0; d0 < ndt; d0 += 64) {
          int d = d0 + lane;
          bool hit = false;
          uint32_t node = 0;
          if (d < ndt) {
            node = dties[d];
            int lo = 0, hi = nt;                      // lower_bound in the sorted clean ties
            while (lo < hi) { int mid = (lo + hi) >> 1; if (ties[mid] < node) lo = mid + 1; else hi = mid; }
            int less = lo;
            for (int e = 0; e < ndt; ++e) less += dties[e] < node;
            hit = (int64_t)(less + 1) == jstar;
          }
          uint64_t bal = __ballot(hit);
          if (bal) { winner = __shfl(node, __ffsll((long long)bal) - 1); break; }
        }
      }
      __syncthreads();
    }
    PlacementDev out;
    out.node = (M >= 0) ? (int32_t)winner : -1;
    out.score = M;
    out.ties = (uint32_t)T;
    out.feasible = (uint32_t)F;
    if (M < 0) {
      if (lane == 0) a.out[k] = out;
      continue;
    }
    // ---- assume + Reserve on the winner: update its row (LDS copy), re-score later pods on it
    int slot = lookup(winner);
    bool fresh = slot < 0;
    if (fresh) {
      slot = nd;
      if (lane == 0) {
        drow_load(m, winner, drows[slot]);
        uint32_t h = (winner * 2654435761u) & (HASH - 1);
        while (hkey[h] >= 0) h = (h + 1) & (HASH - 1);
        hkey[h] = (int)winner;
        hval[h] = slot;
        s_nd = nd + 1;
      }
      __syncthreads();
      // old (batch-start) feasibility of the winner for every later pod
      for (int q = k + 1 + lane; q < B; q += 64)
        dof[q * B + slot] = drow_score(drows[slot], pods[q], a.pf, m) >= 0 ? 1 : 0;
      __syncthreads();
    }
    if (lane == 0) {
      DRow& d = drows[slot];
      for (int s = 0; s < 7; ++s) d.free[s] -= pk.req[s];
      d.nzfree[0] -= pk.nz[0];
      d.nzfree[1] -= pk.nz[1];
      d.free_pods -= 1;
      d.la_free[0] -= pk.est[0];
      d.la_free[1] -= pk.est[1];
      if (pk.flags & PF_PROD) {
        d.la_pfree[0] -= pk.est[0];
        d.la_pfree[1] -= pk.est[1];
      }
      a.out[k] = out;
    }
    __syncthreads();
    for (int q = k + 1 + lane; q < B; q += 64) dsc[q * B + slot] = (int16_t)drow_score(drows[slot], pods[q], a.pf, m);
    __syncthreads();
  }
  // write back dirty rows
  __syncthreads();
  const int nd = s_nd;
  for (int s = lane; s < nd; s += 64) {
    const DRow& d = drows[s];
    uint32_t i = d.node;
    for (int c = 0; c < 7; ++c) m.i64[C_FREE_CPU + c][i] = d.free[c];
    m.i64[C_NZFREE_CPU][i] = d.nzfree[0];
    m.i64[C_NZFREE_MEM][i] = d.nzfree[1];
    m.i64[C_LA_FREE_CPU][i] = d.la_free[0];
    m.i64[C_LA_FREE_MEM][i] = d.la_free[1];
    m.i64[C_LA_PFREE_CPU][i] = d.la_pfree[0];
    m.i64[C_LA_PFREE_MEM][i] = d.la_pfree[1];
    m.i32[C_FREE_PODS][i] = d.free_pods;
  }
  if (lane == 0) *a.committed = committed;
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
  // wave reduce (max, count at max, feasible)
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
__global__ void __launch_bounds__(256) scatter_rows_kernel(MirrorView m, const uint32_t* __restrict__ idx,
                                                           const int64_t* __restrict__ rows, uint32_t nrows) {
  uint32_t r = blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  uint32_t i = idx[r];
  const int64_t* src = rows + (size_t)r * ROW_WORDS;
  for (int c = 0; c < NUM_I64_COLS; ++c) m.i64[c][i] = src[c];
  for (int c = 0; c < NUM_I32_COLS; ++c) m.i32[c][i] = (int32_t)src[NUM_I64_COLS + c];
}

// ------------------------------------------------------------------------------------------------
// launchers
hipError_t launch_node_prep(const MirrorView& m, uint32_t n0, uint32_t n1, int64_t now, int32_t filter_expired,
                            int32_t has_exp, int64_t exp_ns, hipStream_t st) {
  if (n1 <= n0) return hipSuccess;
  uint32_t grid = (n1 - n0 + 255) / 256;
  hipLaunchKernelGGL(node_prep_kernel, dim3(grid), dim3(256), 0, st, m, n0, n1, now, filter_expired, has_exp, exp_ns);
  return hipGetLastError();
}

hipError_t launch_eval(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t n0, uint32_t n1,
                       int16_t* S, uint32_t ld, int prod_cols, hipStream_t st) {
  uint32_t len = n1 - n0;
  uint32_t grid = (len + 256 * NPT - 1) / (256 * NPT);
  if (grid == 0) return hipSuccess;
  hipLaunchKernelGGL(eval_kernel, dim3(grid), dim3(256), 0, st, m, pods, npods, pf, n0, n1, S, ld, prod_cols);
  return hipGetLastError();
}

hipError_t launch_eval_full(const MirrorView& m, const PodVec* pods, int npods, const Profile& pf, uint32_t N,
                            int16_t* scores, uint16_t* codes, int16_t* plugin, int prod_cols, hipStream_t st) {
  uint32_t grid = (N + 255) / 256;
  hipLaunchKernelGGL(eval_full_kernel, dim3(grid), dim3(256), 0, st, m, pods, npods, pf, N, scores, codes, plugin,
                     prod_cols);
  return hipGetLastError();
}

size_t cand_smem_bytes(int max_score) {
  return (size_t)(((max_score + 1) + 3) & ~3) * 4 + (size_t)CAND_CAP * 8;
}

hipError_t launch_cand(const int16_t* S, uint32_t ld, uint32_t len, uint32_t n0, int npods, int max_score,
                       uint64_t* lists, CandHdr* hdrs, hipStream_t st) {
  size_t smem = cand_smem_bytes(max_score);
  hipLaunchKernelGGL(cand_kernel, dim3(npods), dim3(CAND_THREADS), smem, st, S, ld, len, n0, max_score, lists, hdrs);
  return hipGetLastError();
}

size_t commit_smem_bytes(int B, int nranks) {
  size_t b = (size_t)B * sizeof(PodVec) + (size_t)B * sizeof(DRow) + (size_t)B * B * 2;
  b += (size_t)((B * B + 15) & ~15);
  b += (size_t)HASH * 8;
  b += (size_t)(CAND_CAP * nranks + B) * 4 + (size_t)B * 4;
  return (b + 15) & ~(size_t)15;
}

hipError_t launch_commit(const CommitArgs& a, hipStream_t st) {
  size_t smem = commit_smem_bytes(a.npods, a.nranks);
  hipLaunchKernelGGL(commit_kernel, dim3(1), dim3(64), smem, st, a);
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
                               hipStream_t st) {
  if (!nrows) return hipSuccess;
  hipLaunchKernelGGL(scatter_rows_kernel, dim3((nrows + 255) / 256), dim3(256), 0, st, m, idx, rows, nrows);
  return hipGetLastError();
}

hipError_t set_kernel_attributes() {
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(commit_kernel),
                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)commit_smem_bytes(MAX_BATCH, MAX_RANKS));
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute(reinterpret_cast<const void*>(cand_kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)cand_smem_bytes(8191));
}

}  // namespace gs
