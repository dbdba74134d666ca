// san_host.cpp — the CPU code of this repository under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5
// "Race detection / sanitizers"; scripts/sanitize/run.sh builds and runs it; g++ -fsanitize=address,undefined).
//
// Linked from the sources as they are (nothing copied): the oracle (oracle/oracle.cpp, numa.cpp: test
// infrastructure), and the host library sources that need no HIP runtime — the ingest decoders (gs_ingest.cpp), the
// ElasticQuota gate (gs_quota.cpp), the Coscheduling manager (gs_gang.cpp), the reason strings (gs_reasons.cpp) and
// the NodeNUMAResource host restatement with the device cpuset selection compiled for the host
// (gs_numa_host.cpp + gs_cpuset_dev.h, whose self-test compares the two). The device-only merge is in san_merge.cpp.
//
//   san_host replay <file.bin> <expect-hex>   oracle call script recorded by record.py; FNV-1a of the placements
//   san_host cpuset <seed> <iters>            gsx_cpuset_selftest (device takeCPUs vs the host restatement)
//   san_host ingest <corpus>                  every decoder on the corpus and on truncations / byte mutations of it
//   san_host quota <seed> <forests>           random quota forests: refresh, prefilter, reserve, admit / settle
//   san_host gang <seed> <sequences>          random Coscheduling event sequences over the C-ABI
#include <cinttypes>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/gpuscore.h"
#include "../../oracle/oracle.h"

extern "C" int gsx_cpuset_selftest(uint64_t seed, int iters, char* msg, size_t len);

namespace {

int fails = 0;
#define CHECK(cond, ...)                      \
  do {                                        \
    if (!(cond)) {                            \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);           \
      fprintf(stderr, "\n");                  \
      ++fails;                                \
    }                                         \
  } while (0)

uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  return h;
}

// ---------------------------------------------------------------------------------------------- oracle replay
struct Arr {
  bool null = true;
  std::vector<unsigned char> b;
  template <class T> const T* p() const { return null ? nullptr : reinterpret_cast<const T*>(b.data()); }
  template <class T> uint32_t n() const { return (uint32_t)(b.size() / sizeof(T)); }
};

bool read_rec(FILE* f, uint32_t* op, std::vector<Arr>* arrs) {
  uint32_t h[2];
  if (fread(h, 4, 2, f) != 2) return false;
  *op = h[0];
  arrs->assign(h[1], Arr{});
  for (auto& a : *arrs) {
    uint64_t n = 0;
    if (fread(&n, 8, 1, f) != 1) return false;
    if (n == ~0ull) continue;
    a.null = false;
    a.b.resize(n);
    if (n && fread(a.b.data(), 1, n, f) != n) return false;
  }
  return true;
}

int replay(const char* path, const char* expect) {
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "cannot open %s\n", path); return 2; }
  or_cluster* c = nullptr;
  uint64_t h = 1469598103934665603ull;
  uint32_t op;
  std::vector<Arr> a;
  size_t calls = 0, decisions = 0;
  while (read_rec(f, &op, &a)) {
    ++calls;
    int rc = 0;
    switch (op) {
      case 1: c = or_create(a[0].p<gs_config>()); CHECK(c, "or_create"); break;
      case 2: rc = or_set_now(c, *a[0].p<int64_t>()); break;
      case 3: rc = or_nodes_upsert(c, a[0].p<uint32_t>(), a[1].p<gs_node>(), a[1].n<gs_node>()); break;
      case 4:
        rc = or_node_metrics_upsert(c, a[0].p<uint32_t>(), a[1].p<gs_node_metric>(), a[1].n<gs_node_metric>(),
                                    a[2].p<gs_pod_metric>(), a[3].p<uint32_t>());
        break;
      case 5: rc = or_pods_assign(c, a[0].p<uint32_t>(), a[1].p<gs_pod>(), a[2].p<int64_t>(), a[1].n<gs_pod>()); break;
      case 6: {
        int32_t id = -1;
        rc = or_topology_register(c, a[0].p<gs_cpu_topology>(), &id);
        break;
      }
      case 7: rc = or_nodes_numa_upsert(c, a[0].p<uint32_t>(), a[1].p<gs_node_numa>(), a[1].n<gs_node_numa>()); break;
      case 8:
        rc = or_numa_allocations_update(c, a[0].p<uint32_t>(), a[1].p<gs_pod_allocation>(), a[1].n<gs_pod_allocation>());
        break;
      case 9: {
        const uint32_t n = a[0].n<gs_pod>();
        std::vector<gs_placement> out(n);
        rc = or_schedule(c, a[0].p<gs_pod>(), n, a[1].p<uint64_t>(), out.data(), (int)*a[2].p<int64_t>());
        h = fnv(h, out.data(), out.size() * sizeof(gs_placement));
        decisions += n;
        break;
      }
      case 10: {
        const uint32_t n = a[0].n<gs_pod>();
        // (the node count is not in the script: evaluate rows are sized from the cluster's config)
        std::vector<int16_t> sc((size_t)n * 100000), pl((size_t)n * 100000 * GS_NUM_PLUGINS);
        std::vector<uint16_t> cd((size_t)n * 100000);
        rc = or_evaluate(c, a[0].p<gs_pod>(), n, sc.data(), cd.data(), pl.data());
        break;
      }
      case 11: rc = or_ext_configure(c, a[0].p<gs_ext_args>()); break;
      case 12: rc = or_node_devices_upsert(c, a[0].p<uint32_t>(), a[1].p<gs_node_devices>(), a[1].n<gs_node_devices>()); break;
      case 13: rc = or_reservations_upsert(c, a[0].p<gs_reservation>(), a[0].n<gs_reservation>()); break;
      case 14: {
        const uint32_t n = a[0].n<gs_pod>();
        std::vector<gs_placement> out(n);
        std::vector<gs_ext_placement> xo(n);
        rc = or_schedule_ext(c, a[0].p<gs_pod>(), a[1].p<gs_pod_ext>(), n, a[2].p<uint64_t>(), out.data(), xo.data());
        h = fnv(h, out.data(), out.size() * sizeof(gs_placement));
        h = fnv(h, xo.data(), xo.size() * sizeof(gs_ext_placement));
        decisions += n;
        break;
      }
      default: CHECK(false, "unknown op %u", op);
    }
    CHECK(rc >= 0, "%s: op %u returned %d", path, op, rc);
  }
  fclose(f);
  if (c) or_destroy(c);
  char got[32];
  snprintf(got, sizeof got, "%016" PRIx64, h);
  CHECK(std::strcmp(got, expect) == 0, "%s: placements %s, the unsanitized oracle's %s", path, got, expect);
  printf("replay %s: %zu calls, %zu decisions, placements %s\n", path, calls, decisions, got);
  return 0;
}

// ---------------------------------------------------------------------------------------------- ingest
void decode_all(int kind, const std::string& k, const std::string& v) {
  gs_node node{};
  gs_node_numa numa{};
  gs_pod pod{};
  gs_kv kv{k.c_str(), v.c_str()};
  uint64_t w[GS_CPU_WORDS];
  int64_t a = 0, b = 0;
  int32_t nr = 0;
  switch (kind) {
    case 1: (void)gs_decode_quantity(v.c_str(), &a, &b); break;
    case 2: (void)gs_decode_cpuset(v.c_str(), w); break;
    case 3:
      (void)gs_decode_node_annotations(&kv, 1, &node, &numa);
      node.allocatable[0] = 64000;
      node.allocatable[1] = 256LL << 30;
      (void)gs_node_reservation_trim(&kv, 1, &node);
      (void)gs_node_reserved_cpus(&kv, 1, w, &nr);
      (void)gs_decode_nrt_reserved_cpus(&kv, 1, w);
      break;
    case 4: (void)gs_decode_resource_spec(v.c_str(), &pod); break;
    case 5: {
      static gs_cpu_topology t;
      (void)gs_decode_cpu_topology(v.c_str(), &t);
      break;
    }
    case 6:
      (void)gs_decode_node_labels(&kv, 1, v.c_str(), v.c_str(), &numa);
      (void)gs_decode_node_labels(&kv, 1, nullptr, nullptr, &numa);
      break;
  }
}

int ingest(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) { fprintf(stderr, "cannot open %s\n", path); return 2; }
  std::mt19937_64 rng(7);
  size_t inputs = 0, runs = 0;
  uint32_t h[3];
  while (fread(h, 4, 3, f) == 3) {
    std::string k(h[1], '\0'), v(h[2], '\0');
    if ((h[1] && fread(&k[0], 1, h[1], f) != h[1]) || (h[2] && fread(&v[0], 1, h[2], f) != h[2])) break;
    ++inputs;
    decode_all((int)h[0], k, v);
    ++runs;
    for (size_t l = 0; l < v.size() && l < 400; ++l) {   // every truncation
      decode_all((int)h[0], k, v.substr(0, l));
      ++runs;
    }
    const char alpha[] = "{}[]\":,.-+eE0123456789 \\uaxyz";
    for (int m = 0; m < 64 && !v.empty(); ++m) {   // byte mutations (deletions, substitutions, insertions)
      std::string x = v;
      const int nm = 1 + (int)(rng() % 3);
      for (int j = 0; j < nm && !x.empty(); ++j) {
        const size_t at = rng() % x.size();
        const int what = (int)(rng() % 3);
        const char ch = alpha[rng() % (sizeof alpha - 1)];
        if (what == 0) x.erase(at, 1);
        else if (what == 1) x[at] = ch;
        else x.insert(x.begin() + (long)at, ch);
      }
      decode_all((int)h[0], k, x);
      ++runs;
    }
  }
  fclose(f);
  printf("ingest: %zu corpus inputs, %zu decoder runs\n", inputs, runs);
  CHECK(inputs > 0, "empty corpus");
  return 0;
}

// ---------------------------------------------------------------------------------------------- quota
int quota(uint64_t seed, int forests) {
  std::mt19937_64 rng(seed);
  auto U = [&](int64_t lo, int64_t hi) { return lo + (int64_t)(rng() % (uint64_t)(hi - lo + 1)); };
  size_t pods = 0;
  for (int it = 0; it < forests; ++it) {
    const uint32_t n = (uint32_t)U(1, 40);
    std::vector<gs_quota_group> g(n);
    for (uint32_t i = 0; i < n; ++i) {
      gs_quota_group& q = g[i];
      std::memset(&q, 0, sizeof q);
      q.parent = (i == 0 || U(0, 3) == 0) ? -1 : (int32_t)U(0, i - 1);
      q.allow_lent = (uint32_t)U(0, 1);
      q.max_mask = (uint32_t)U(0, (1 << GS_QUOTA_DIMS) - 1);
      q.min_mask = q.max_mask & (uint32_t)U(0, (1 << GS_QUOTA_DIMS) - 1);
      for (int d = 0; d < GS_QUOTA_DIMS; ++d) {
        q.max[d] = U(0, 1000000);
        q.min[d] = U(0, q.max[d]);
        q.shared_weight[d] = U(0, 1) ? q.max[d] : U(1, 1000);
        q.request[d] = U(0, 200000);
        q.used[d] = U(0, q.request[d]);
        q.non_preemptible_used[d] = U(0, q.used[d]);
      }
    }
    int64_t total[GS_QUOTA_DIMS];
    for (int d = 0; d < GS_QUOTA_DIMS; ++d) total[d] = U(0, 5000000);
    std::vector<int64_t> rt((size_t)n * GS_QUOTA_DIMS), lr((size_t)n * GS_QUOTA_DIMS);
    std::vector<uint32_t> rm(n);
    int rc = gs_quota_refresh_runtime(g.data(), n, total, rt.data(), lr.data(), rm.data());
    CHECK(rc == GS_OK, "refresh rc %d", rc);
    const uint32_t cnt = (uint32_t)U(1, 64);
    std::vector<int32_t> qi(cnt);
    std::vector<int64_t> req((size_t)cnt * GS_QUOTA_DIMS);
    std::vector<uint32_t> rmask(cnt), fl(cnt);
    for (uint32_t j = 0; j < cnt; ++j) {
      qi[j] = (int32_t)U(-1, n - 1);
      rmask[j] = (uint32_t)U(0, (1 << GS_QUOTA_DIMS) - 1);
      fl[j] = (uint32_t)U(0, 7);
      for (int d = 0; d < GS_QUOTA_DIMS; ++d) req[(size_t)j * GS_QUOTA_DIMS + d] = U(0, 100000);
      gs_quota_status st{};
      rc = gs_quota_prefilter(g.data(), n, rt.data(), rm.data(), qi[j], &req[(size_t)j * GS_QUOTA_DIMS], rmask[j], fl[j], &st);
      CHECK(rc == GS_OK, "prefilter rc %d", rc);
    }
    std::vector<gs_quota_status> st(cnt);
    uint32_t done = 0;
    for (uint32_t at = 0; at < cnt; at += done) {
      rc = gs_quota_admit_batch(g.data(), n, rt.data(), rm.data(), qi.data() + at, req.data() + (size_t)at * GS_QUOTA_DIMS,
                                rmask.data() + at, fl.data() + at, cnt - at, st.data() + at, &done);
      CHECK(rc == GS_OK && done > 0, "admit_batch rc %d consumed %u", rc, done);
      if (rc != GS_OK || !done) break;
      std::vector<int32_t> placed(done);
      for (uint32_t j = 0; j < done; ++j) placed[j] = U(0, 3) ? (int32_t)U(0, 99) : -1;
      rc = gs_quota_settle_batch(g.data(), n, rt.data(), rm.data(), qi.data() + at, req.data() + (size_t)at * GS_QUOTA_DIMS,
                                 rmask.data() + at, fl.data() + at, done, placed.data(), st.data() + at);
      CHECK(rc == GS_OK, "settle_batch rc %d", rc);
      pods += done;
    }
    for (uint32_t j = 0; j < cnt; ++j)
      if (qi[j] >= 0) (void)gs_quota_reserve(g.data(), n, qi[j], &req[(size_t)j * GS_QUOTA_DIMS], fl[j], U(0, 1) ? 1 : -1);
  }
  printf("quota: %d forests, %zu pods through admit / settle\n", forests, pods);
  return 0;
}

// ---------------------------------------------------------------------------------------------- gang
int gang(uint64_t seed, int seqs) {
  std::mt19937_64 rng(seed);
  auto U = [&](int64_t lo, int64_t hi) { return lo + (int64_t)(rng() % (uint64_t)(hi - lo + 1)); };
  size_t events = 0;
  std::vector<uint64_t> buf(8);
  for (int s = 0; s < seqs; ++s) {
    gs_gang_args ga{};
    ga.default_timeout_ns = 600000000000LL;
    gs_gang_mgr* m = nullptr;
    CHECK(gs_gang_mgr_create(&ga, &m) == GS_OK && m, "gang create");
    if (!m) return 1;
    const int ng = (int)U(1, 6);
    int64_t now = 1000;
    for (int e = 0; e < 300; ++e, ++events) {
      const uint64_t gid = (uint64_t)U(1, ng), uid = (uint64_t)U(1, 40);
      uint32_t nout = 0;
      int64_t wait = 0;
      int rc = 0;
      now += U(0, 5) * 1000000000LL;
      switch (U(0, 10)) {
        case 0: {
          gs_gang_spec sp{};
          sp.gang_id = gid;
          sp.min_member = (int32_t)U(-1, 6);
          sp.total_children = (int32_t)U(-1, 8);
          sp.mode = (int32_t)U(-1, 1);
          sp.match_policy = (int32_t)U(-1, 2);
          sp.wait_time_ns = U(-1, 3) * 1000000000LL;
          sp.create_time_ns = now;
          sp.group_n = (uint32_t)U(0, 3);
          for (uint32_t k = 0; k < sp.group_n; ++k) sp.group[k] = (uint64_t)U(1, ng);
          rc = gs_gang_podgroup_upsert(m, &sp);
          break;
        }
        case 1: rc = gs_gang_podgroup_delete(m, gid); break;
        case 2: case 3: {
          gs_gang_spec an{};
          an.gang_id = gid;
          an.min_member = (int32_t)U(1, 4);
          an.total_children = -1;
          an.mode = -1;
          an.match_policy = -1;
          an.wait_time_ns = -1;
          an.create_time_ns = now;
          rc = gs_gang_pod_add(m, gid, uid, (int)U(0, 1), U(0, 1) ? &an : nullptr);
          break;
        }
        case 4: rc = gs_gang_pod_delete(m, gid, uid); break;
        case 5: rc = gs_gang_prefilter(m, gid, uid, (int)U(0, 1)); break;
        case 6:
          rc = gs_gang_permit(m, gid, uid, now, &wait, buf.data(), (uint32_t)buf.size(), &nout);
          if (rc == GS_EINVAL) { buf.resize(nout + 1); rc = 0; }
          break;
        case 7:
          rc = gs_gang_post_filter(m, gid, uid, buf.data(), (uint32_t)buf.size(), &nout);
          if (rc == GS_EINVAL) { buf.resize(nout + 1); rc = 0; }
          break;
        case 8:
          rc = gs_gang_unreserve(m, gid, uid, buf.data(), (uint32_t)buf.size(), &nout);
          if (rc == GS_EINVAL) { buf.resize(nout + 1); rc = 0; }
          break;
        case 9:
          rc = gs_gang_expire(m, now, buf.data(), (uint32_t)buf.size(), &nout);
          if (rc == GS_EINVAL) { buf.resize(nout + 1); rc = 0; }
          break;
        default: {
          rc = gs_gang_post_bind(m, gid, uid);
          gs_gang_info inf{};
          (void)gs_gang_get(m, gid, &inf);
          break;
        }
      }
      (void)rc;   // codes are checked against the restatement by tests/test_gang.py; here: memory and UB only
    }
    gs_gang_mgr* cl = nullptr;
    if (gs_gang_mgr_clone(m, &cl) == GS_OK && cl) {
      (void)gs_gang_mgr_assign(cl, m);
      gs_gang_mgr_destroy(cl);
    }
    gs_gang_mgr_destroy(m);
  }
  printf("gang: %d sequences, %zu events\n", seqs, events);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: san_host replay|cpuset|ingest|quota|gang ...\n"); return 2; }
  const std::string what = argv[1];
  int rc = 2;
  if (what == "replay" && argc == 4) rc = replay(argv[2], argv[3]);
  else if (what == "cpuset" && argc == 4) {
    char msg[512] = {0};
    const int bad = gsx_cpuset_selftest(strtoull(argv[2], nullptr, 0), atoi(argv[3]), msg, sizeof msg);
    CHECK(bad == 0, "cpuset self-test: %s", msg);
    printf("cpuset: seed %s, %s cases, %d mismatches\n", argv[2], argv[3], bad);
    rc = 0;
  } else if (what == "ingest" && argc == 3) rc = ingest(argv[2]);
  else if (what == "quota" && argc == 4) rc = quota(strtoull(argv[2], nullptr, 0), atoi(argv[3]));
  else if (what == "gang" && argc == 4) rc = gang(strtoull(argv[2], nullptr, 0), atoi(argv[3]));
  if (rc) return rc;
  return fails ? 1 : 0;
}
