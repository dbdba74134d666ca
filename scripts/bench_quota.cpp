// bench_quota.cpp — host throughput of the ElasticQuota gate (gs_quota_refresh_runtime, gs_quota_prefilter) as a
// cgo caller would drive it: one refresh per quota / request change, one PreFilter per pod. Seeded random forest
// (splitmix64), 3 dimensions, depth <= 4.
//   g++ -O2 -std=c++17 -o /tmp/bench_quota scripts/bench_quota.cpp -Lkoordinator_amd -lgpuscore \
//       -Wl,-rpath,$PWD/koordinator_amd && /tmp/bench_quota 2000 1000000
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/gpuscore.h"

static uint64_t s = 0x6b6f6f7264ull;
static uint64_t next() {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static int64_t rnd(int64_t n) { return (int64_t)(next() % (uint64_t)n); }

int main(int argc, char** argv) {
  const uint32_t q = argc > 1 ? atoi(argv[1]) : 2000;
  const uint32_t pods = argc > 2 ? atoi(argv[2]) : 1000000;
  std::vector<gs_quota_group> g(q);
  std::vector<uint32_t> depth(q, 0);
  for (uint32_t i = 0; i < q; ++i) {
    gs_quota_group& x = g[i];
    x = gs_quota_group{};
    x.parent = -1;
    if (i > 8) {
      const uint32_t p = (uint32_t)rnd(i);
      if (depth[p] < 3) { x.parent = (int32_t)p; depth[i] = depth[p] + 1; }
    }
    x.allow_lent = rnd(10) < 7;
    x.max_mask = x.min_mask = 0x7;
    for (int d = 0; d < 3; ++d) {
      x.max[d] = 1000000 + rnd(1000000);
      x.min[d] = rnd(x.max[d] / 4);
      x.shared_weight[d] = x.max[d];
      x.request[d] = rnd(200000);
      x.used[d] = rnd(x.request[d] + 1);
    }
  }
  int64_t total[GS_QUOTA_DIMS] = {500000000, 500000000, 500000000};
  std::vector<int64_t> rt(size_t(q) * GS_QUOTA_DIMS);
  std::vector<uint32_t> mask(q);
  const int refreshes = 200;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < refreshes; ++r) {
    g[r % q].request[0] += 1;
    if (gs_quota_refresh_runtime(g.data(), q, total, rt.data(), nullptr, mask.data()) != 0) return 1;
  }
  auto t1 = std::chrono::steady_clock::now();
  uint64_t admitted = 0;
  int64_t req[GS_QUOTA_DIMS] = {};
  gs_quota_status st;
  for (uint32_t p = 0; p < pods; ++p) {
    req[0] = rnd(8000);
    req[1] = rnd(16000);
    req[2] = rnd(2);
    if (gs_quota_prefilter(g.data(), q, rt.data(), mask.data(), (int32_t)rnd(q), req, 0x7,
                           GS_QUOTA_RUNTIME | GS_QUOTA_CHECK_PARENT | (p & 1 ? GS_QUOTA_NON_PREEMPTIBLE : 0),
                           &st) != 0)
      return 1;
    admitted += st.code == GS_QUOTA_ADMIT;
  }
  auto t2 = std::chrono::steady_clock::now();
  const double rs = std::chrono::duration<double>(t1 - t0).count() / refreshes;
  const double ps = std::chrono::duration<double>(t2 - t1).count();
  printf("{\"quotas\": %u, \"refresh_runtime_us\": %.1f, \"prefilter_pods_per_s\": %.3g, \"admitted_frac\": %.3f}\n",
         q, rs * 1e6, pods / ps, (double)admitted / pods);
  return 0;
}
