// gs_probe.hip — diagnostics: cycle cost of the commit kernel's per-pair evaluations on real mirror rows
// (gs_debug_pair_probe). Each workgroup (one wave) copies a node row and the pod vectors into LDS the way the
// commit kernel holds them, then times one evaluation with s_memtime.
//   mode 0: one (pod, node) pair by the whole wave (row_score_wave: the selector's re-score of the next pod)
//   mode 1: one node for pods 0..63, one pod per lane (row_score over the row's hint table: the re-scoring waves)
//   mode 2: one (pod, node) pair by the whole wave, lane-parallel evaluation (pair_score_wave)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gs_eval_dev.h"
#define GS_PAIR_PROBE 1
#include "gs_pair_wave.h"

namespace gs {

__device__ __forceinline__ uint64_t probe_stamp() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_waitcnt(0);
  const uint64_t t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int MODE>
__global__ void __launch_bounds__(64) probe_kernel(MirrorView m, Profile pf, const PodVec* __restrict__ pods, int npods,
                                                   const uint32_t* __restrict__ nodes, const int32_t* __restrict__ pod_of,
                                                   int prod_cols, int32_t* __restrict__ scores, uint64_t* __restrict__ cycles) {
  __shared__ Row r;
  __shared__ PodVec pv[64];
  __shared__ HintTable t;
  const int lane = threadIdx.x, i = blockIdx.x;
  const bool numa = (pf.enabled & 0x30u) != 0;
  if (lane == 0) {
    Row x;
    load_row(m, nodes[i], prod_cols, numa, x);
    // the commit's LDS copy carries the scalar free columns too
    for (int s = 3; s < 7; ++s) x.free[s] = m.c64(C_FREE_CPU + s)[nodes[i]];
    r = x;
  }
  for (int q = lane; q < npods && q < 64; q += 64) pv[q] = pods[q];
  __syncthreads();
  int32_t x = 0;
  uint64_t t0 = 0, t1 = 0;
  if (MODE == 0 || MODE == 2) {
    const PodVec& p = pv[pod_of[i]];
    // the second of two evaluations is timed (warm instruction cache, as in the commit loop); cold_cycles: the first
    for (int it = 0; it < 2; ++it) {
      t0 = probe_stamp();
      if (MODE == 0) {
        const Row rr = r;
        x = row_score_wave(rr, p, pf, m, nullptr);
      } else {
        for (int j = lane; j < 8; j += 64) gs_pw_st[j] = 0;
        x = pair_score_wave(r, p, pf, m);
      }
      x = __builtin_amdgcn_readfirstlane(x);
      t1 = probe_stamp();
      if (it == 0 && lane == 0) cycles[gridDim.x + i] = t1 - t0;
    }
    if (lane == 0) scores[i] = x;
    if (MODE == 2)
      for (int j = lane; j < 8; j += 64) cycles[2 * gridDim.x + 8 * i + j] = gs_pw_st[j];
  } else {
    for (int it = 0; it < 2; ++it) {
      t0 = probe_stamp();
      const Row rr = r;
      if (numa && ((rr.nr.nflags >> NF_POLICY_SHIFT) & 3u)) hint_table_fill(t, rr.nr, zone_avail(rr.nr), lane);
      WAVE_FENCE();
      x = lane < npods ? row_score(rr, pv[lane], pf, m, &t) : 0;
      x = __builtin_amdgcn_readfirstlane(wave_max(x));
      t1 = probe_stamp();
      if (it == 0 && lane == 0) cycles[gridDim.x + i] = t1 - t0;
    }
    const Row rr = r;
    scores[(size_t)i * 64 + lane] = lane < npods ? row_score(rr, pv[lane], pf, m, &t) : 0;
  }
  if (lane == 0) cycles[i] = t1 - t0 + (x == 0x7fffffff ? 1 : 0);
}

hipError_t launch_probe(int mode, const MirrorView& m, const Profile& pf, const PodVec* pods, int npods,
                        const uint32_t* nodes, const int32_t* pod_of, uint32_t n, int prod_cols, int32_t* scores,
                        uint64_t* cycles, hipStream_t st) {
  if (mode == 0)
    hipLaunchKernelGGL(probe_kernel<0>, dim3(n), dim3(64), 0, st, m, pf, pods, npods, nodes, pod_of, prod_cols, scores, cycles);
  else if (mode == 1)
    hipLaunchKernelGGL(probe_kernel<1>, dim3(n), dim3(64), 0, st, m, pf, pods, npods, nodes, pod_of, prod_cols, scores, cycles);
  else
    hipLaunchKernelGGL(probe_kernel<2>, dim3(n), dim3(64), 0, st, m, pf, pods, npods, nodes, pod_of, prod_cols, scores, cycles);
  return hipGetLastError();
}

// The device's topology-manager Merge (gs_numa_dev.h merge_hint_lists, the code every NUMA-policy pair evaluation runs)
// on given inputs, one case per thread: the policy_test.go vectors driven through the device merge directly.
__global__ void __launch_bounds__(64) merge_probe_kernel(const gs_merge_case* __restrict__ cs, int n,
                                                         gs_merge_result* __restrict__ out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const gs_merge_case c = cs[i];
  auto score_at = [&](int mi) -> int32_t { return c.score[mi]; };
  bool aff_has = false, over = false;
  uint32_t aff = 0;
  bool admit;
  if (c.gpu_hints) {   // both providers: the extension path's general merge (merge_hint_lists_gen)
    HintList L[5];
    const int nl = gen_lists(c.totc, c.lc, c.totm, c.lm, ord_valid(c.nz), c.nil_hints != 0, c.has_cpu != 0,
                             c.has_mem != 0, c.tot_c_any != 0, c.tot_m_any != 0, c.gpu_hints, L);
    admit = merge_hint_lists_gen(L, nl, c.nz, c.policy, score_at, aff_has, aff, over);
  } else {
    admit = merge_hint_lists(c.totc, c.lc, c.totm, c.lm, c.nz, c.policy, c.nil_hints != 0, c.has_cpu != 0,
                             c.has_mem != 0, c.tot_c_any != 0, c.tot_m_any != 0, score_at, aff_has, aff);
  }
  out[i] = gs_merge_result{admit ? 1 : 0, aff_has ? 1 : 0, aff, over ? 1 : 0};
}

hipError_t launch_merge_probe(const gs_merge_case* cases, int n, gs_merge_result* out, hipStream_t st) {
  hipLaunchKernelGGL(merge_probe_kernel, dim3((n + 63) / 64), dim3(64), 0, st, cases, n, out);
  return hipGetLastError();
}

}  // namespace gs
