// gs_eval_dev.h — device code shared by the eval kernels (gs_kernels.hip) and the commit kernels (gs_kernels.hip, gs_commit_spec.hip):
// the node row a pair evaluation reads, the fused Filter + Score of one (pod, node) pair, the selectHost tie-break
// stream, wave helpers and the device-side cpuset Reserve.
//
// Integer semantics follow Go: int64 two's complement, truncating division. The float64 spots of the
// reference (LoadAware filter %, estimator scaling) are host-side per node / per pod; per-pair work here is
// int64 with an exact reciprocal-estimate-plus-correction division (quotients lie in [0,100]).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_cpuset_dev.h"
#include "gs_kernels.h"
#include "gs_numa_dev.h"

namespace gs {

// ------------------------------------------------------------------------------------------------
// exact floor((x*100)/cap) for 0 <= x <= cap, 0 < cap < 2^53
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

// A node row: everything one Filter+Score evaluation reads (scalar-resource columns stay in HBM and are
// read only for pods that request / profiles that weigh scalar resources).
struct Row {
  int64_t free[7];      // Allocatable - Requested per slot (slots 3..6 only in the commit's LDS copy)
  int64_t alloc[2];     // cpu, mem
  int64_t nzfree[2];
  int64_t la_cap[2];
  int64_t la_free[2];
  int64_t la_pfree[2];
  int32_t free_pods;
  uint32_t dflags;
  uint32_t node;        // global index
  uint32_t pad;
  NumaRow nr;           // NodeNUMAResource columns (loaded when the profile enables the plugin)
};
constexpr int ROW_I64 = 17;   // int64 words of Row, in the column order of kRowCol
constexpr int NUMA_I64 = 18;  // NumaRow int64 words: C_ZCAP_CPU0 .. C_NAMP (contiguous columns)
constexpr int NUMA_I32 = 12;  // NumaRow int32 words: C_NFLAGS .. C_ZADJ0+3 (contiguous columns)
static_assert(C_NAMP - C_ZCAP_CPU0 + 1 == NUMA_I64, "NUMA i64 columns contiguous");
static_assert(C_ZADJ0 + 3 - C_NFLAGS + 1 == NUMA_I32, "NUMA i32 columns contiguous");

static __constant__ int kRowCol[ROW_I64] = {C_FREE_CPU,     C_FREE_MEM,    C_FREE_EPH,   C_FREE_BCPU,  C_FREE_BMEM,
                                     C_FREE_MCPU,    C_FREE_MMEM,   C_ALLOC_CPU,  C_ALLOC_MEM,  C_NZFREE_CPU,
                                     C_NZFREE_MEM,   C_LA_CAP_CPU,  C_LA_CAP_MEM, C_LA_FREE_CPU, C_LA_FREE_MEM,
                                     C_LA_PFREE_CPU, C_LA_PFREE_MEM};
// Row words an assume/Reserve changes (written back by the commit kernel)
__device__ __forceinline__ bool row_word_mutable(int j) { return j < 7 || j == 9 || j == 10 || j >= 13; }

__device__ __forceinline__ void load_row(const MirrorView& m, uint32_t i, bool prod_cols, bool numa, Row& r) {
  if (numa) load_numa_row(m, i, r.nr);
  r.free[0] = m.c64(C_FREE_CPU)[i];
  r.free[1] = m.c64(C_FREE_MEM)[i];
  r.free[2] = m.c64(C_FREE_EPH)[i];
  r.alloc[0] = m.c64(C_ALLOC_CPU)[i];
  r.alloc[1] = m.c64(C_ALLOC_MEM)[i];
  r.nzfree[0] = m.c64(C_NZFREE_CPU)[i];
  r.nzfree[1] = m.c64(C_NZFREE_MEM)[i];
  r.la_cap[0] = m.c64(C_LA_CAP_CPU)[i];
  r.la_cap[1] = m.c64(C_LA_CAP_MEM)[i];
  r.la_free[0] = m.c64(C_LA_FREE_CPU)[i];
  r.la_free[1] = m.c64(C_LA_FREE_MEM)[i];
  if (prod_cols) {
    r.la_pfree[0] = m.c64(C_LA_PFREE_CPU)[i];
    r.la_pfree[1] = m.c64(C_LA_PFREE_MEM)[i];
  } else {
    r.la_pfree[0] = r.la_pfree[1] = 0;
  }
  r.free_pods = m.c32(C_FREE_PODS)[i];
  r.dflags = (uint32_t)m.c32(C_DFLAGS)[i];
  r.node = i;
}

struct PairOut {
  uint32_t code;
  int32_t fit, la, numa;
  uint32_t aff;         // NodeNUMAResource Filter-time affinity (NumaOut.aff)
};

// NodeInfo slot views for numa_eval: Allocatable and Allocatable - Requested per resource slot
struct SlotsHbm {
  const Row& r;
  const MirrorView& m;
  __device__ int64_t alloc(int s) const { return s < 2 ? r.alloc[s] : m.c64(C_ALLOC_CPU + s)[r.node]; }
  __device__ int64_t free(int s) const { return s < 3 ? r.free[s] : m.c64(C_FREE_CPU + s)[r.node]; }
};
struct SlotsLds {
  const Row& r;
  const MirrorView& m;
  __device__ int64_t alloc(int s) const { return s < 2 ? r.alloc[s] : m.c64(C_ALLOC_CPU + s)[r.node]; }
  __device__ int64_t free(int s) const { return r.free[s]; }
};

// Filter (Fit + LoadAware) and Score (Fit LeastAllocated + LoadAware) of one pod on one node.
// LDS_SCALARS: scalar free columns come from r.free[3..6] (the commit's LDS copy) instead of HBM.
// NUMA_POLICY_NODES = false: NodeNUMAResource's topology-policy path is compiled out (eval_kernel routes those
// nodes to eval_numa_kernel)
// table: the row's NUMA hint table (commit re-scoring of one row for many pods), else computed from the row.
// GPROV / gh / gh_over: DeviceShare as a second NUMA hint provider (numa_eval; the extension path's GPU pods).
template <bool FULL, bool LDS_SCALARS, bool NUMA_POLICY_NODES = true, bool TABLE = false, bool WAVE = false,
          bool GPROV = false>
__device__ __forceinline__ PairOut eval_pair(const Row& r, const PodVec& p, const Profile& pf, const MirrorView& m,
                                             const HintTable* table = nullptr, uint32_t gh = 0,
                                             bool* gh_over = nullptr) {
  PairOut o{0u, 0, 0, 0, 0u};
  // ---- [upstream] noderesources Fit.Filter -> fitsRequest
  if (pf.enabled & 0x1u) {
    if (r.free_pods < 1) o.code |= 0x01u;                               // len(Pods)+1 > AllowedPodNumber
    if (!(p.flags & PF_ALL_ZERO)) {
      if (p.req[0] > r.free[0]) o.code |= 0x02u;
      if (p.req[1] > r.free[1]) o.code |= 0x04u;
      if (p.req[2] > r.free[2]) o.code |= 0x08u;
      if (p.scalar_mask) {
        for (int s = 3; s < 7; ++s) {
          if (!(p.scalar_mask & (1u << s))) continue;
          int64_t fr = LDS_SCALARS ? r.free[s] : m.c64(C_FREE_CPU + s)[r.node];
          if (p.req[s] > fr) o.code |= 0x10u;
        }
      }
    }
  }
  // ---- LoadAware.Filter (load_aware.go:123-171), usage verdicts precomputed per node
  if ((pf.enabled & 0x4u) && !(p.flags & PF_DAEMONSET)) {
    const bool prod = p.flags & PF_PROD;
    if (r.dflags & (prod ? DF_LA_FAIL_P : DF_LA_FAIL_NP))   // + the reason's resource / aggregated form
      o.code |= 0x20u | ((r.dflags >> (prod ? DF_P_DETAIL_SHIFT : DF_NP_DETAIL_SHIFT)) & 3u) << 10;
  }
  if (!FULL && o.code) return o;
  // ---- NodeNUMAResource Filter (+ Admit) and Score (gs_numa_dev.h)
  if (pf.enabled & 0x30u) {
    NumaOut no;
    if (LDS_SCALARS) no = numa_eval<NUMA_POLICY_NODES, TABLE, WAVE, GPROV>(r.nr, p, pf, SlotsLds{r, m},
                                                                     pf.enabled & 0x10u, pf.enabled & 0x20u, -1,
                                                                     table, gh, gh_over);
    else no = numa_eval<NUMA_POLICY_NODES>(r.nr, p, pf, SlotsHbm{r, m}, pf.enabled & 0x10u, pf.enabled & 0x20u);
    if (pf.enabled & 0x10u) o.code |= no.reason << GS_FAIL_NUMA_SHIFT;
    if (!FULL && o.code) return o;
    o.numa = no.reason ? 0 : no.score;
    o.aff = no.aff;
  }
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
        int64_t cap = m.c64(C_ALLOC_CPU + s)[r.node];
        if (cap == 0) continue;
        int64_t fr = (LDS_SCALARS || s == 2) ? r.free[s] : m.c64(C_FREE_CPU + s)[r.node];
        ns += least_requested(fr, preq, cap) * pf.fit_w[s];
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
  return o.fit * pf.w_fit + o.la * pf.w_la + o.numa * pf.w_numa;
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

// the positions tiebreak_position's walk visits for (seed, seq), ascending (they do not depend on T), for a lane-parallel
// lookup: out[0..TB_N-2] records (INT32_MAX past the walk's end), out[TB_N-1] = the largest T they decide
__host__ __device__ inline void tiebreak_records(uint64_t seed, uint64_t seq, int32_t* out) {
  const uint64_t key = mix64(seed ^ mix64(seq));
  int64_t j = 1;
  int k = 0;
  int32_t lim = INT32_MAX;   // the walk ended: every T
  out[k++] = 1;
  for (uint64_t i = 0;; ++i) {
    if (k == TB_N - 1) { lim = (int32_t)j; break; }   // records full: T up to the last one
    const uint64_t h = mix64(key + i);
    const double u = (double)((h >> 11) + 1) * 0x1.0p-53;
    const double x = (double)j / u;
    if (!(x < 4.0e18)) break;
    const int64_t jn = (int64_t)floor(x) + 1;
    if (jn >= (int64_t)INT32_MAX) { lim = INT32_MAX - 1; break; }   // the next record is past int32
    j = jn;
    out[k++] = (int32_t)j;
  }
  for (; k < TB_N - 1; ++k) out[k] = INT32_MAX;
  out[TB_N - 1] = lim;
}


// ------------------------------------------------------------------------------------------------
// Sequential commit: ONE wave walks the batch's pods in order (no workgroup barriers: LDS traffic of a
// single wave is in order, so phases only need compiler scheduling fences, and global prefetches of the
// next pod's headers stay in flight while the current pod is resolved).
//
// For pod k the effective score of a node is its batch-start score (S, summarized per shard by the listed
// levels) unless an earlier pod of the batch landed on it ("dirty"): dirty rows live in LDS and their
// scores for every later pod are re-evaluated exactly (dso = batch-start score, dsc = current score).
// The max M is valid when it exceeds every shard's highest unlisted score (`next`); otherwise the batch
// is cut at k. Ties at M are ordered by node index across shards (shards are contiguous ranges).
constexpr int NUMA_PPT = 4;   // pods per thread in eval_numa_kernel (full batches): half the row traffic of 2 at the same pass time
constexpr int COMMIT_WAVES = 4, COMMIT_THREADS = 64 * COMMIT_WAVES;   // commit workgroup
constexpr int HASH = 1024;
constexpr int POD_STRIDE = 136;   // LDS bytes per pod vector in the commit kernel (sizeof(PodVec) + 8)
static_assert(POD_STRIDE >= (int)sizeof(PodVec) && POD_STRIDE % 8 == 0, "pod stride");
constexpr int WIN = 2 * MAX_BATCH + 8;
#define WAVE_FENCE() __builtin_amdgcn_wave_barrier()

__device__ __forceinline__ int32_t row_score(const Row& d, const PodVec& p, const Profile& pf, const MirrorView& m,
                                             const HintTable* table = nullptr) {
  return total_score(eval_pair<false, true, true, true>(d, p, pf, m, table), pf);
}

// one pair evaluated by all 64 lanes of a wave (row, pod and table wave-uniform); every lane gets the score
__device__ __forceinline__ int32_t row_score_wave(const Row& d, const PodVec& p, const Profile& pf, const MirrorView& m,
                                                  const HintTable* table) {
  return total_score(eval_pair<false, true, true, true, true>(d, p, pf, m, table), pf);
}

__device__ __forceinline__ int hash_find(const int32_t* hkey, const int32_t* hval, uint32_t node) {
  uint32_t h = (node * 2654435761u) & (HASH - 1);
  for (int probe = 0; probe < HASH; ++probe) {
    int kk = hkey[h];
    if (kk == (int)node) return hval[h];
    if (kk < 0) return -1;
    h = (h + 1) & (HASH - 1);
  }
  return -1;
}

__device__ __forceinline__ const LevelHdr* hdr_ptr(const CommitArgs& a, int r, int k) {
  return reinterpret_cast<const LevelHdr*>(a.xbase + (size_t)r * a.xblock + (size_t)a.bmax * LCAP * 4) + k;
}
__device__ __forceinline__ const uint32_t* list_ptr(const CommitArgs& a, int r, int k) {
  return reinterpret_cast<const uint32_t*>(a.xbase + (size_t)r * a.xblock) + (size_t)k * LCAP;
}

// Wave64 reductions and scan over DPP row operations (no LDS round trip, unlike __shfl_*: ds_bpermute). All 64
// lanes must be active. quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror reduce within a 16-lane row;
// row_bcast15 (rows 1, 3) and row_bcast31 (rows 2, 3) carry the rows into lane 63.
#define GS_DPP(old, v, ctrl, rmask) __builtin_amdgcn_update_dpp((old), (v), (ctrl), (rmask), 0xF, false)
__device__ __forceinline__ int wave_max(int v) {
  constexpr int lo = -2147483647 - 1;
  v = max(v, GS_DPP(lo, v, 0xB1, 0xF));
  v = max(v, GS_DPP(lo, v, 0x4E, 0xF));
  v = max(v, GS_DPP(lo, v, 0x141, 0xF));
  v = max(v, GS_DPP(lo, v, 0x140, 0xF));
  v = max(v, GS_DPP(lo, v, 0x142, 0xA));
  v = max(v, GS_DPP(lo, v, 0x143, 0xC));
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_sum(int v) {
  v += GS_DPP(0, v, 0xB1, 0xF);
  v += GS_DPP(0, v, 0x4E, 0xF);
  v += GS_DPP(0, v, 0x141, 0xF);
  v += GS_DPP(0, v, 0x140, 0xF);
  v += GS_DPP(0, v, 0x142, 0xA);
  v += GS_DPP(0, v, 0x143, 0xC);
  return __builtin_amdgcn_readlane(v, 63);
}
// inclusive prefix sum over lanes: row_shr 1, 2, 4, 8 within rows, then the row carries
__device__ __forceinline__ int wave_or(int v) {
  v |= GS_DPP(0, v, 0xB1, 0xF);
  v |= GS_DPP(0, v, 0x4E, 0xF);
  v |= GS_DPP(0, v, 0x141, 0xF);
  v |= GS_DPP(0, v, 0x140, 0xF);
  v |= GS_DPP(0, v, 0x142, 0xA);
  v |= GS_DPP(0, v, 0x143, 0xC);
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += GS_DPP(0, v, 0x111, 0xF);
  v += GS_DPP(0, v, 0x112, 0xF);
  v += GS_DPP(0, v, 0x114, 0xF);
  v += GS_DPP(0, v, 0x118, 0xF);
  v += GS_DPP(0, v, 0x142, 0xA);
  v += GS_DPP(0, v, 0x143, 0xC);
  return v;
}

// sort n (<= 128) distinct node ids in place, tmp as scratch (one wave)
__device__ __forceinline__ void wave_rank_sort(uint32_t* v, int n, uint32_t* tmp, int lane) {
  for (int i = lane; i < n; i += 64) {
    uint32_t x = v[i];
    int r = 0;
    for (int u = 0; u < n; ++u) r += v[u] < x;
    tmp[r] = x;
  }
  WAVE_FENCE();
  for (int i = lane; i < n; i += 64) v[i] = tmp[i];
  WAVE_FENCE();
}

// The device Reserve selects this pod's cpuset on this row: its topology is in the device scope (topo >= 0), and the
// exclusivity state the selection reads is exact (an exclusive pod on a row marked CM_XSTALE —
// a maxRefCount-2 node whose shared CPUs lost their policy — has its cpuset selected by the host).
__device__ __forceinline__ bool cpuset_on_device(const CpuStateDev& cs, const PodVec& p) {
  const int ep = (p.numa & PN_BIND) ? (int)((p.numa >> PN_EXCL_SHIFT) & 3u) : GS_CPU_EXCLUSIVE_NONE;
  return cs.topo >= 0 && !((cs.meta & CM_XSTALE) && ep != GS_CPU_EXCLUSIVE_NONE);
}

// Device-side cpuset Reserve of one pod on its winner row (one thread): allocateCPUSet with the NUMA split of
// Allocate (resource_manager.go:273-360, gs_cpuset_dev.h), then NodeAllocation.addPodAllocation
// (node_allocation.go:82-110) on the CPU state and the row's available-CPU summaries, as numa_derive
// (gs_numa_host.cpp) would recompute them. false: allocateCPUSet errors (the host fails loudly).
// Arguments live in LDS or registers (zone split by value, cpuset into an LDS array): nothing of the caller's
// frame has its address taken, so the commit kernel keeps its Reserve state out of scratch. The topology (TopoDev,
// read-only) is read from HBM at a wave-uniform address: scalar loads.
#define GS_LDS __attribute__((address_space(3)))
// Not inlined: its register pressure stays out of the commit loop. The LDS operands arrive as address-space-3
// pointers and everything below is inlined here, so every access stays a ds_* instruction (a generic pointer would
// make them flat loads that wait for outstanding global loads).
__device__ __noinline__ bool cpuset_reserve(const TopoDev* __restrict__ tp, GS_LDS CpuStateDev* csp, const PodVec& p,
                                            uint32_t nf, uint32_t zkeys, int64_t zc0, int64_t zc1, int64_t zc2,
                                            int64_t zc3, GS_LDS NumaRow* nrp, GS_LDS uint64_t* cpuset) {
  // every operand is wave-uniform (one Reserve at a time): say so, so that the selection runs on the scalar unit
  auto u32 = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
  auto u64 = [&](int64_t x) {
    return (int64_t)(((uint64_t)u32((uint32_t)((uint64_t)x >> 32)) << 32) | u32((uint32_t)(uint64_t)x));
  };
  tp = (const TopoDev*)(((uint64_t)u32((uint32_t)((uint64_t)tp >> 32)) << 32) | u32((uint32_t)(uint64_t)tp));
  csp = (GS_LDS CpuStateDev*)(size_t)u32((uint32_t)(size_t)csp);
  nrp = (GS_LDS NumaRow*)(size_t)u32((uint32_t)(size_t)nrp);
  cpuset = (GS_LDS uint64_t*)(size_t)u32((uint32_t)(size_t)cpuset);
  nf = u32(nf);
  zkeys = u32(zkeys);
  const TopoDev& t = *tp;   // (the td_* entry points read it through the constant address space)
  CpuStateDev& cs = *(CpuStateDev*)csp;
  NumaRow& nr = *(NumaRow*)nrp;
  const int64_t zcpu[4] = {u64(zc0), u64(zc1), u64(zc2), u64(zc3)};
  // getCPUBindPolicy (util.go:85-103)
  const uint32_t pn = u32(p.numa);
  const int st_req = (pn >> PN_REQ_SHIFT) & 7, nb = (nf >> NF_BIND_SHIFT) & 3;
  int bind = (pn >> PN_PREF_SHIFT) & 7;
  bool required = false;
  if (st_req != BIND_UNSET) { bind = st_req; required = true; }
  else if (nb == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS) { bind = BIND_SPREAD; required = true; }
  else if (nb == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY) { bind = BIND_FULL; required = true; }
  const int ep = (pn & PN_BIND) ? (int)((pn >> PN_EXCL_SHIFT) & 3u) : GS_CPU_EXCLUSIVE_NONE;
  uint64_t R[4];   // the cpuset, packed plane words
  if (!td_allocate_cpuset(t, cs, (int)u32((uint32_t)p.num_cpus), bind, required, ep, zkeys, zcpu, R)) return false;
  const int nz = (nf >> NF_ZONES_SHIFT) & 7;
  nr.alloc_cpus += td_reserve_update(t, cs, R, ep, nz);
  nr.tfree = (uint32_t)td_counts(t, cs, -1);
  for (int z = 0; z < 4; ++z) {
    const int n = td_zone_node(cs, z);
    if (z >= nz || n >= TU32(td_topo(t).nnodes)) continue;   // a zone the topology lacks keeps its zero summaries
    nr.zfree[z] = (uint32_t)td_counts(t, cs, n);
    if (nr.amp > 1.0) {
      const int64_t c = (int64_t)((TU64(cs.zal) >> (16 * z)) & 0xFFFFull) * 1000;
      nr.zadj[z] = (int32_t)(amplify_d(c, nr.amp) - c);
    }
  }
  uint64_t w[4];
  td_to_cpus(t, R, w);
  for (int j = 0; j < 4; ++j) cpuset[j] = w[j];
  return true;
}

}  // namespace gs
