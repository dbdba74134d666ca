// merge_ptr_probe.hip — reproducer of the round-4 "miscompile" in the two-provider merge (gs_numa_dev.h
// merge_hint_lists_gen): with GS_MERGE_PTR_SELECT the pass's entry sets are read through a pointer selecting one of two
// private arrays (the round-4 form; the library reads a copy). The SAME source runs on the host (checked clean under
// ASan + UBSan by san_merge, and against the oracle's permutation scan) and on the GPU, over the same random list
// sets; any difference between the two is the device compiler's. Built twice by scripts/sanitize/gpu_probe.sh: with
// -DGS_MERGE_PTR_SELECT (the round-4 form) and without (the library's form, the control).
// Usage: merge_ptr_probe <cases> (prints the mismatch count, rc 0).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../koordinator_amd/csrc/gs_kernels.h"
#include "../../koordinator_amd/csrc/gs_numa_dev.h"

using namespace gs;

__host__ __device__ inline gs_merge_result run_case(const gs_merge_case& c) {
  HintList L[5];
  const int nl = gen_lists(c.totc, c.lc, c.totm, c.lm, ord_valid(c.nz), c.nil_hints != 0, c.has_cpu != 0,
                           c.has_mem != 0, c.tot_c_any != 0, c.tot_m_any != 0, c.gpu_hints, L);
  auto score_at = [&](int mi) -> int32_t { return c.score[mi]; };
  bool aff_has = false, over = false;
  uint32_t aff = 0;
  const bool admit = merge_hint_lists_gen(L, nl, c.nz, c.policy, score_at, aff_has, aff, over);
  return gs_merge_result{admit ? 1 : 0, aff_has ? 1 : 0, aff_has ? aff : 0u, over ? 1 : 0};
}

__global__ void probe(const gs_merge_case* cs, int n, gs_merge_result* out) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i < n) out[i] = run_case(cs[i]);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 100000;
  std::mt19937_64 rng(20260);
  auto U = [&](int lo, int hi) { return lo + (int)(rng() % (uint64_t)(hi - lo + 1)); };
  std::vector<gs_merge_case> cs(n);
  for (auto& c : cs) {   // list sets of the providers' shapes (as san_merge / test_numa_merge_device.py draw them)
    c = gs_merge_case{};
    c.nz = U(1, 4);
    const uint32_t valid = ord_valid(c.nz);
    const int pols[3] = {GS_NUMA_POLICY_BEST_EFFORT, GS_NUMA_POLICY_RESTRICTED, GS_NUMA_POLICY_SINGLE_NUMA_NODE};
    c.policy = pols[U(0, 2)];
    for (int i = 0; i < 15; ++i) c.score[i] = U(0, 100);
    c.nil_hints = U(0, 19) == 0;
    auto pick = [&]() { return (uint32_t)rng() & valid; };
    for (int r = 0; r < 2; ++r) {
      const bool has = U(0, 99) < 85;
      uint32_t l = pick(), tot = l | pick();
      if (U(0, 9) == 0) l = 0;
      if (!has) l = tot = 0;
      if (r == 0) { c.lc = l; c.totc = tot; c.has_cpu = has; c.tot_c_any = tot != 0; }
      else { c.lm = l; c.totm = tot; c.has_mem = has; c.tot_m_any = tot != 0; }
    }
    const uint32_t gl = U(0, 9) == 0 ? 0u : pick();
    int hi = c.nz;
    for (int i = 0; i < 15; ++i) if (gl >> i & 1u) hi = std::min(hi, __builtin_popcount(ord_mask(i)));
    c.gpu_hints = gl | ((uint32_t)U(1, hi) << 16) | ((uint32_t)U(2, 3) << 20);
  }
  std::vector<gs_merge_result> host(n), dev(n);
  for (int i = 0; i < n; ++i) host[i] = run_case(cs[i]);
  gs_merge_case* d_c = nullptr;
  gs_merge_result* d_o = nullptr;
  if (hipMalloc(&d_c, sizeof(gs_merge_case) * n) != hipSuccess || hipMalloc(&d_o, sizeof(gs_merge_result) * n) != hipSuccess)
    return 2;
  (void)hipMemcpy(d_c, cs.data(), sizeof(gs_merge_case) * n, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3((n + 63) / 64), dim3(64), 0, 0, d_c, n, d_o);
  if (hipDeviceSynchronize() != hipSuccess) return 3;
  (void)hipMemcpy(dev.data(), d_o, sizeof(gs_merge_result) * n, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    const auto& a = host[i];
    const auto& b = dev[i];
    if (a.admit != b.admit || a.aff_has != b.aff_has || a.aff != b.aff || a.pad != b.pad) {
      if (bad < 5)
        printf("case %d (nz %d policy %d gpu %#x): host admit %d aff %d/%#x, device admit %d aff %d/%#x\n", i, cs[i].nz,
               cs[i].policy, cs[i].gpu_hints, a.admit, a.aff_has, a.aff, b.admit, b.aff_has, b.aff);
      ++bad;
    }
  }
#ifdef GS_MERGE_PTR_SELECT
  const char* form = "pointer-select (round-4) form";
#else
  const char* form = "copy (library) form";
#endif
  printf("%s: %d of %d cases differ between the host and the gfx950 build of the same source\n", form, bad, n);
  (void)hipFree(d_c);
  (void)hipFree(d_o);
  return 0;
}
