// san_merge.cpp — the two-provider topology-manager merge (gs_numa_dev.h merge_hint_lists_gen, the code the extension
// path's policy-node evaluation runs on the GPU) compiled for the HOST under AddressSanitizer + UBSan, against the
// oracle's permutation scan (oracle/numa.cpp policy_merge_filtered, mergeFilteredHints with hint scores), on random
// list sets of the shapes the hint providers produce (the generator of tests/test_numa_merge_device.py::_gen_case).
//
// Why: round 4 found the GPU result wrong until "a pointer selecting between two private arrays" (the pass's entry
// sets s0 / s1) was replaced by a copy, and called it a miscompile. Out-of-bounds indexing or other undefined behaviour
// in the function would look the same; this run settles it for the code as it is.
//
// Built by scripts/sanitize/run.sh with amdclang++ (hipcc) host-only: -x hip --offload-host-only, the sanitizers on
// the host compilation (-Xarch_host). Usage: san_merge <seed> <cases>
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../koordinator_amd/csrc/gs_kernels.h"
#include "../../koordinator_amd/csrc/gs_numa_dev.h"

extern "C" int or_policy_merge_scored(int policy, uint64_t numa_mask, int nlists, const int32_t* lens,
                                      const uint8_t* has_mask, const uint64_t* masks, const uint8_t* preferred,
                                      const int64_t* scores, uint8_t* out_has_mask, uint64_t* out_mask,
                                      uint8_t* out_preferred);

using namespace gs;

namespace {
constexpr uint64_t kOrd4 = 0xFEDB7CA69538421ull;   // position -> mask (gs_numa_dev.h ord_mask)
int ordm(int i) { return (int)((kOrd4 >> (4 * i)) & 15u); }

struct H { bool has; uint64_t mask; bool pref; int64_t score; };
}  // namespace

int main(int argc, char** argv) {
  if (argc != 3) { fprintf(stderr, "usage: san_merge <seed> <cases>\n"); return 2; }
  std::mt19937_64 rng(strtoull(argv[1], nullptr, 0));
  const long ncases = atol(argv[2]);
  auto U = [&](int lo, int hi) { return lo + (int)(rng() % (uint64_t)(hi - lo + 1)); };
  auto R = [&]() { return (double)(rng() >> 11) * (1.0 / 9007199254740992.0); };
  long bad = 0, over = 0;
  for (long k = 0; k < ncases; ++k) {
    gs_merge_case c{};
    const int nz = U(1, 4);
    std::vector<int> valid;
    for (int i = 0; i < 15; ++i)
      if (ordm(i) < (1 << nz)) valid.push_back(i);
    c.nz = nz;
    const int pols[3] = {GS_NUMA_POLICY_BEST_EFFORT, GS_NUMA_POLICY_RESTRICTED, GS_NUMA_POLICY_SINGLE_NUMA_NODE};
    c.policy = pols[U(0, 2)];
    for (int i = 0; i < 15; ++i) c.score[i] = U(0, 100);
    c.nil_hints = R() < 0.05;
    auto pick = [&]() {
      uint32_t m = 0;
      for (int i : valid) if (R() < 0.5) m |= 1u << i;
      return m;
    };
    for (int res = 0; res < 2; ++res) {
      const bool has = R() < 0.85;
      uint32_t l = pick(), tot = l | pick();
      if (R() < 0.1) l = 0;
      if (!has) l = tot = 0;
      if (res == 0) { c.lc = l; c.totc = tot; c.has_cpu = has; c.tot_c_any = tot != 0; }
      else { c.lm = l; c.totm = tot; c.has_mem = has; c.tot_m_any = tot != 0; }
    }
    const int r = U(2, 3);
    const uint32_t gl = R() < 0.1 ? 0u : pick();
    int gmin_hi = nz;
    for (int i = 0; i < 15; ++i)
      if (gl >> i & 1u) gmin_hi = std::min(gmin_hi, __builtin_popcount(ordm(i)));
    const int gmin = U(1, gmin_hi);
    c.gpu_hints = gl | ((uint32_t)gmin << 16) | ((uint32_t)r << 20);
    // the reference-shaped lists (filterProvidersHints): NodeNUMAResource's cpu, memory; then r identical GPU lists
    std::vector<std::vector<H>> lists;
    if (!c.nil_hints) {
      const uint32_t ls[2] = {c.lc, c.lm}, ts[2] = {c.totc, c.totm};
      const int hs[2] = {c.has_cpu, c.has_mem};
      for (int q = 0; q < 2; ++q) {
        if (!hs[q] || !ts[q]) continue;
        if (!ls[q]) { lists.push_back({H{false, 0, false, 0}}); continue; }
        int smin = 9;
        for (int i = 0; i < 15; ++i) if (ts[q] >> i & 1u) smin = std::min(smin, __builtin_popcount(ordm(i)));
        std::vector<H> l;
        for (int i = 0; i < 15; ++i)
          if (ls[q] >> i & 1u) l.push_back(H{true, (uint64_t)ordm(i), __builtin_popcount(ordm(i)) == smin, c.score[i]});
        lists.push_back(l);
      }
    }
    if (lists.empty()) lists.push_back({H{false, 0, true, 0}});
    std::vector<H> g;
    for (int i = 0; i < 15; ++i)
      if (gl >> i & 1u) g.push_back(H{true, (uint64_t)ordm(i), __builtin_popcount(ordm(i)) == gmin, 0});
    if (g.empty()) g.push_back(H{false, 0, false, 0});
    for (int q = 0; q < r; ++q) lists.push_back(g);
    std::vector<int32_t> lens;
    std::vector<uint8_t> has, pref;
    std::vector<uint64_t> masks;
    std::vector<int64_t> scores;
    for (auto& l : lists) {
      lens.push_back((int32_t)l.size());
      for (auto& h : l) { has.push_back(h.has); masks.push_back(h.mask); pref.push_back(h.pref); scores.push_back(h.score); }
    }
    uint8_t oh = 0, op = 0;
    uint64_t om = 0;
    const int want_admit = or_policy_merge_scored(c.policy, (1ull << nz) - 1, (int)lists.size(), lens.data(), has.data(),
                                                  masks.data(), pref.data(), scores.data(), &oh, &om, &op);
    // the device merge, as the probe kernel runs it (gs_probe.hip merge_probe_kernel)
    HintList L[5];
    const int nl = gen_lists(c.totc, c.lc, c.totm, c.lm, ord_valid(c.nz), c.nil_hints != 0, c.has_cpu != 0,
                             c.has_mem != 0, c.tot_c_any != 0, c.tot_m_any != 0, c.gpu_hints, L);
    auto score_at = [&](int mi) -> int32_t { return c.score[mi]; };
    bool aff_has = false, ov = false;
    uint32_t aff = 0;
    const bool admit = merge_hint_lists_gen(L, nl, c.nz, c.policy, score_at, aff_has, aff, ov);
    if (ov) { ++over; continue; }
    const bool same = admit == (want_admit != 0) && aff_has == (oh != 0) && (!aff_has || aff == (uint32_t)om);
    if (!same && bad++ < 5)
      fprintf(stderr, "case %ld: nz %d policy %d lists %d: device admit %d aff %d/%#x, oracle admit %d aff %d/%#" PRIx64 "\n",
              k, nz, c.policy, nl, admit, aff_has, aff, want_admit, oh, om);
  }
  printf("merge: %ld random two-provider list sets, %ld mismatches, %ld over the search bound\n", ncases, bad, over);
  return bad || over ? 1 : 0;
}
