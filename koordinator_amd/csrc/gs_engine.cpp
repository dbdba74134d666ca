// gs_engine.cpp — libgpuscore host side: the C-ABI of include/gpuscore.h over the HIP kernels.
//
// Owns the host mirror of the scheduler state the hot path reads (NodeInfo rows, NodeMetrics, the
// LoadAware podAssignCache) and its HBM structure-of-arrays image. Per-node derived columns (LoadAware
// usage verdicts, estimated usage, free capacities) are recomputed on the host only for rows an event
// touched and scattered to HBM; pod placements made by gs_schedule are applied on the device by the
// commit kernel and replayed on the host mirror, so no row crosses PCIe for them.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <atomic>

#include "../../include/gpuscore.h"
#include "gs_ext.h"
#include "gs_kernels.h"
#include "gs_numa_host.h"

using namespace gs;

namespace {

constexpr int64_t kDefaultMilliCPURequest = 250;              // loadaware/estimator/default_estimator.go:36
constexpr int64_t kDefaultMemoryRequest = 200LL * 1024 * 1024; // loadaware/estimator/default_estimator.go:38
constexpr int64_t kDefaultReportIntervalNs = 60LL * 1000000000LL;
constexpr int64_t kZeroTime = INT64_MIN;
constexpr int64_t kMaxExact = 1LL << 53;                      // value bound for the exact int64 score paths

struct Assigned {
  int64_t ts;
  gs_pod pod;
};

struct HostNode {
  gs_node node{};
  bool valid = false;
  gs_node_metric metric{};
  std::vector<gs_pod_metric> pms;
  std::unordered_map<uint64_t, Assigned> assigned;   // podAssignCache.podInfoItems[node]
};

struct Vec2 {
  int64_t v[2] = {0, 0};
  uint32_t mask = 0;
  bool has(int r) const { return mask & (1u << r); }
  int64_t get(int r) const { return has(r) ? v[r] : 0; }
  void add(int r, int64_t x) { v[r] = get(r) + x; mask |= 1u << r; }
};

Vec2 usage_of(const gs_usage& u) {
  Vec2 o;
  if (u.mask & GS_USAGE_CPU) { o.v[0] = u.cpu_milli; o.mask |= 1; }
  if (u.mask & GS_USAGE_MEMORY) { o.v[1] = u.memory; o.mask |= 2; }
  if (u.mask & GS_USAGE_OTHER) o.mask |= GS_USAGE_OTHER;
  return o;
}

}  // namespace

// ---- asynchronous submissions (gs_schedule_submit / gs_schedule_wait): a worker thread runs schedule_stream over
// the submitted runs in order, taking the next run while the current one's last batch is in flight
struct AsyncRun {
  std::vector<gs_pod> pods;
  std::vector<uint64_t> seq;
  gs_placement* out = nullptr;
  uint64_t ticket = 0;
  int rc = 1;   // 1: not complete
  std::string err;
};
struct AsyncQueue {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<std::shared_ptr<AsyncRun>> pending;                  // submitted, not yet taken by the worker
  std::unordered_map<uint64_t, std::shared_ptr<AsyncRun>> runs;   // submitted, not yet waited for
  uint64_t next_ticket = 1;
  bool busy = false, stop = false;
};


// In-process device transport (gs_comm_init_local): the ranks are threads of one process. Per exchange each rank
// publishes its send block and the event recorded after its tag, the threads meet (host barrier, no GPU wait), every
// rank enqueues on its stream a wait on each rank's event and the device-to-device copy of its block, publishes the
// event after its copies, and after a second meeting waits on every rank's copies event on its stream: the collective
// is complete on a rank's stream only once every rank has read its block, as with ncclAllGather, and the host never
// waits for the GPU. A rank that does not arrive within GS_LOCAL_WAIT_S (60 s) fails the call with GS_ECOMM.
struct gs_local_group {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  std::vector<const uint8_t*> send;
  std::vector<size_t> bytes;
  std::vector<hipEvent_t> ready, done;
  // true: every rank arrived; false: the wait expired or the group is broken (a rank failed)
  bool meet(double limit_s) {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    const bool ok = cv.wait_for(lk, std::chrono::duration<double>(limit_s), [&] { return gen != g || broken; });
    if (!ok || broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

struct gs_ctx {
  std::unordered_set<uint64_t> ext_reserved;   // pods placed with an extension-path Reserve (gs_schedule_ext)
  gs_config cfg{};
  std::string err;
  std::unique_ptr<AsyncQueue> aq;   // gs_schedule_submit's worker (created by the first submission)
  uint32_t N = 0, npad = 0;
  hipStream_t st = nullptr;
  hipStream_t st2 = nullptr;                // side stream: eval_kernel beside eval_numa_kernel
  hipStream_t st_ev = nullptr;              // eval passes: a batch's eval runs beside the previous batch's commit
  hipStream_t st_rb = nullptr;              // a batch's placement readback, off the stream the next batch runs on
  uint32_t window_k = 0;                    // node sampling: numFeasibleNodesToFind(N) (0 = every node)
  uint32_t next_start = 0;                  // [upstream] Scheduler.nextStartNodeIndex
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  std::vector<hipEvent_t> x_ev;             // RCCL all-gather start / end events not yet accounted (exchange_ms)
  int x_pending = 0;
  // device mirror
  int64_t* d_i64 = nullptr;
  int32_t* d_i32 = nullptr;
  MirrorView mv{};
  // batch buffers
  int B = MAX_BATCH;
  PodVec* d_pods = nullptr;
  uint64_t* d_seq = nullptr;
  int16_t* d_S = nullptr;
  uint32_t ld = 0;
  uint8_t* d_xchg_send = nullptr;   // local lists + headers (contiguous, all-gathered)
  uint8_t* d_xchg_recv = nullptr;   // R blocks
  uint8_t* d_xmerged = nullptr;     // several ranks, speculative commit: the R blocks' levels merged into one block
  size_t xchg_bytes = 0;
  int lstride = LCAP;               // listed nodes per pod in the local / exchanged blocks (XCAP: several ranks, spec)
  PlacementDev* d_out = nullptr;
  int32_t* d_committed = nullptr;
  int32_t* d_tb = nullptr;          // speculative commit: tie-break records of the batch's pods
  RowStat* d_rowstat = nullptr;
  int32_t* d_sel = nullptr;
  uint32_t* d_stage_idx = nullptr;
  int64_t* d_stage_rows = nullptr;
  uint32_t stage_cap = 0;
  // pinned host buffers
  PodVec* h_pods = nullptr;
  uint64_t* h_seq = nullptr;
  PlacementDev* h_out = nullptr;
  int32_t* h_committed = nullptr;
  uint32_t* h_stage_idx = nullptr;
  int64_t* h_stage_rows = nullptr;
  uint8_t* h_xchg_send = nullptr;
  uint8_t* h_xchg_recv = nullptr;
  hipEvent_t ev[8] = {};
  // double-buffered per-batch buffers (slot 0 = the fields above when bound): the next batch is enqueued
  // speculatively before the current one is read back (gs_schedule)
  struct Slot {
    int16_t* d_S = nullptr;         // score rows and Filter-time affinities of the slot's batch
    uint8_t* d_aff = nullptr;
    hipEvent_t ev_go = nullptr, ev_evdone = nullptr;
    PodVec* d_pods = nullptr;
    uint64_t* d_seq = nullptr;
    PlacementDev* d_out = nullptr;
    int32_t* d_committed = nullptr;
    PodVec* h_pods = nullptr;
    uint64_t* h_seq = nullptr;
    PlacementDev* h_out = nullptr;
    int32_t* h_committed = nullptr;
    hipEvent_t ev[6] = {};
    bool untimed = false;           // the batch recorded no timing events (a short direct batch)
    uint8_t* d_lst = nullptr;       // overlapped cand (one shard): the slot's lists + headers, and its histograms
    uint32_t* d_hist = nullptr;
  } slot[2];
  bool cand_overlap = false;        // GS_CAND_OVERLAP (default on): cand beside the previous commit, fix_levels after it
  uint8_t* d_lst = nullptr;         // the bound slot's (cand_overlap)
  uint32_t* d_hist = nullptr;
  uint32_t* d_cscratch = nullptr;   // launch_cand's short-batch split (slice histograms, slice offsets)
  int cur_slot = 0;
  // host mirror
  std::vector<HostNode> nodes;
  std::vector<uint8_t> row_dirty;
  std::vector<uint32_t> dirty_list;
  std::unordered_map<uint64_t, uint32_t> uid_node;
  std::unordered_map<uint64_t, int> metric_names;
  int64_t now = 0;
  bool prep_stale = true;
  Profile pf{};
  int max_score = 0;
  // sharding
  int nranks = 1, rank = 0;
  uint32_t n0 = 0, n1 = 0;          // the node range the levels, fixes and commit see (all nodes: one rank, scores)
  // Several ranks exchange either their score rows (sgather, the default: every rank evaluates its shard [e0, e1), the
  // all-gather makes the full rows, and the one-shard pipeline runs on every rank) or their candidate levels
  // (GS_XCHG=levels: n0/n1 = the shard, merged level lists, the multi-shard commit)
  bool sgather = false;
  uint32_t e0 = 0, e1 = 0;          // the node range this rank evaluates
  uint32_t sx_per = 0, sx_pld = 0;  // nodes per shard, the block's row stride
  size_t sx_bytes = 0;              // one rank's score block (tag included)
  uint8_t* d_sx_send = nullptr;     // [B x pld int16 | B x pld u8 | ... | XTag]
  uint8_t* d_sx_recv = nullptr;     // R blocks
  uint8_t* h_sx_send = nullptr;     // host-callback transport
  uint8_t* h_sx_recv = nullptr;
  uint32_t n_valid = 0;   // nodes upserted at least once (ready())
  ncclComm_t comm = nullptr;
  gs_allgather_fn cb = nullptr;
  void* cb_user = nullptr;
  gs_local_group* lg = nullptr;     // in-process device transport (tests: ranks as threads)
  hipEvent_t lg_ready = nullptr, lg_done = nullptr;
  // exchange sequence (XTag): every exchange's block carries (site, seq, batch, rank); all ranks check all tags
  std::atomic<uint64_t> xseq{0};    // exchanges so far
  std::atomic<uint64_t> xbatch{0};  // batch passes launched so far (launch_batch)
  int32_t* d_xerr = nullptr;        // merge_levels_kernel's verdict on the level blocks' tags
  uint8_t* d_xsmall = nullptr;      // small exchanges (row stats, selection): [own block | R blocks] of XSMALL bytes
  uint8_t* h_xsmall = nullptr;      // their R blocks read back
  int64_t dbg_xskew_rank = -1;      // GS_DEBUG_XCHG_SKEW=rank:batch (tests): that rank skips one sequence number there
  uint64_t dbg_xskew_batch = 0;
  // GS_WATCHDOG_S=<seconds> (diagnostics): a thread reports on stderr any host wait of the scheduling path that lasts
  // longer, naming the wait (Where markers), the batch pass and the exchange count
  std::atomic<const char*> where{nullptr};
  std::atomic<int64_t> where_t{0};
  std::thread watchdog;
  std::atomic<bool> wd_stop{false};
  gs_stats stats{};
  uint64_t* d_stamps = nullptr;   // GS_COMMIT_STAMPS=1: commit-kernel phase cycle sums
  uint64_t stats_all_pods = 0;     // pods placed by gs_schedule over the context's life (stamp averages)
  // GS_HOST_TIMING=1: host time per batch of schedule_stream, by phase (printed by gs_destroy)
  bool host_timing = false;
  double ht_wait = 0, ht_apply = 0, ht_stage = 0, ht_launch = 0, ht_max_busy = 0;
  uint64_t ht_batches = 0, ht_busy_hist[8] = {};
  // ... and of gs_schedule_ext: per extension pod (records, flushes, the device chain up to the host's wake-up, the
  // Reserves) and per plain run (the whole gs_schedule call)
  double hx_prep = 0, hx_flush = 0, hx_gpu = 0, hx_reserve = 0, hx_plain = 0;
  uint64_t hx_pods = 0, hx_runs = 0;
  // NodeNUMAResource: per-node TopologyOptions + NodeAllocation mirror, registered CPU topologies
  std::vector<NumaNode> numa;
  std::vector<std::shared_ptr<TopoClass>> topos;
  std::shared_ptr<TopoClass> empty_topo = std::make_shared<TopoClass>();
  std::unordered_map<uint64_t, uint32_t> numa_uid_node;   // pods holding a NodeAllocation record
  bool numa_on = false;
  // the shard's nodes with a NUMA topology policy (eval_numa_kernel's work list), rebuilt when policies change
  uint32_t* d_numa_idx = nullptr;
  uint32_t numa_n = 0;
  MirrorView slab_mv{nullptr, nullptr, 0};   // the eval pass's dense copy of the NUMA-policy rows (gather_numa_kernel)
  uint32_t slab_cap = 0;
  bool numa_idx_stale = true;
  // the extension path's list over [n0, n1) (all nodes under the score-row exchange, where the batch path's list covers
  // the rank's shard only): its own buffer, so pods alternating between the two paths rebuild neither
  uint32_t* d_xnuma_idx = nullptr;
  uint32_t xnuma_n = 0;
  bool xnuma_stale = true;
  uint32_t numa_idx_lo = 0, numa_idx_hi = 0;   // the node range d_numa_idx lists (the batch path's shard [e0, e1))
  int64_t prep_now = INT64_MIN;             // `now` of the last full node_prep pass
  // registered topologies in bit-plane form (the commit kernel's cpuset Reserve), and the host re-check of
  // every device-chosen cpuset (GS_VERIFY_CPUSET=1)
  TopoDev* d_topos = nullptr;
  uint8_t* d_aff = nullptr;       // [pod][ld] Filter-time NUMA affinity of policy nodes (eval -> commit Reserve)
  bool verify_cpuset = false;
  // Reservation + DeviceShare (gs_ext.hip): host mirror of the nodes' GPU devices and of the reservation cache
  gs_ext_args ext{};
  std::vector<gs_node_devices> devs;             // per node (has_device = 0: no Device object)
  std::vector<uint8_t> dev_dirty;
  std::vector<uint32_t> dev_dirty_list;
  std::map<uint64_t, gs_reservation> rsv;        // reservationCache by uid (uid order = the harness's iteration order)
  std::vector<std::vector<uint64_t>> rsv_node;   // uids per node, ascending
  std::unordered_map<uint64_t, std::vector<uint64_t>> rsv_owner;   // owner key -> uids
  DevNode* d_dev = nullptr;
  DevNode* h_dev_stage = nullptr;   // ext_flush_devices staging (pinned / device): images, then node indices
  DevNode* d_dev_stage = nullptr;
  ExtPod* d_xpod = nullptr;
  ExtRec* d_xrec = nullptr;
  ExtRes* d_xres = nullptr;
  int32_t* d_xtot = nullptr;
  int16_t* d_xds = nullptr;
  int16_t* d_xrs = nullptr;
  int32_t* d_xnom = nullptr;
  int32_t* d_xT = nullptr;
  ExtOut* d_xout = nullptr;
  ExtPod* h_xpod = nullptr;          // (the host half of d_xin's first section)
  unsigned char* h_xin = nullptr;    // one extension pod's inputs, staged for ONE copy: ExtPod | PodVec | ExtRec[] |
  unsigned char* d_xin = nullptr;    // ExtRes[] (pinned host / device, ext_stage_layout)
  PodVec* d_xpv = nullptr;
  size_t xin_off_rec = 0, xin_off_res = 0, xin_bytes = 0;
  ExtOut* h_xout = nullptr;
  int32_t* h_xnom = nullptr;
  std::vector<ExtRec> xrec;
  std::vector<ExtRes> xres;
  std::vector<uint64_t> xres_uid;
  uint32_t xrec_cap = 0, xres_cap = 0;
};

int quiesce(gs_ctx* c);   // the async submissions' worker is idle (gs_schedule_submit)

namespace {
int64_t mono_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// marks a host wait of the scheduling path (the watchdog names it when it lasts)
struct Where {
  gs_ctx* c;
  const char* prev;
  int64_t prev_t;
  Where(gs_ctx* cc, const char* site) : c(cc), prev(cc->where.load()), prev_t(cc->where_t.load()) {
    c->where_t.store(mono_ns());
    c->where.store(site);
  }
  ~Where() {
    c->where.store(prev);
    c->where_t.store(prev_t);
  }
};
// Host waits of the scheduling path: poll the event / stream (spin, then yield, then short sleeps) instead of HIP's
// blocking synchronisation. Several processes sharing one GPU (the C4 rehearsal) showed a rank parked for 10-100 s
// inside hipStreamSynchronize / hipEventSynchronize while every stream and event of that rank had long completed (the
// watchdog's queries), i.e. a lost wake-up of the blocking wait. A poll sees the completion at once;
// bounded: past GS_WAIT_LIMIT_S (default 600 s) the call fails with GS_EDEVICE naming the wait. GS_WAIT_BLOCKING=1:
// HIP's blocking calls (experiments).
bool wait_blocking() {
  static const bool b = getenv("GS_WAIT_BLOCKING") && getenv("GS_WAIT_BLOCKING")[0] == '1';
  return b;
}
template <class Query>
hipError_t poll_until(Query&& query, double limit_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t it = 0;; ++it) {
    const hipError_t e = query();
    if (e != hipErrorNotReady) return e;
    if (it < 2000) {
      __builtin_ia32_pause();
    } else if (it < 20000) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
      if ((it & 1023) == 0 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > limit_s)
        return hipErrorLaunchTimeOut;   // (the wait exceeded its bound: reported as GS_EDEVICE)
    }
  }
}
double wait_limit_s() {
  static const double lim = getenv("GS_WAIT_LIMIT_S") ? atof(getenv("GS_WAIT_LIMIT_S")) : 600.0;
  return lim > 0 ? lim : 600.0;
}
hipError_t host_wait_event(hipEvent_t ev) {
  if (wait_blocking()) return hipEventSynchronize(ev);
  return poll_until([&] { return hipEventQuery(ev); }, wait_limit_s());
}
hipError_t host_wait_stream(hipStream_t st) {
  if (wait_blocking()) return hipStreamSynchronize(st);
  return poll_until([&] { return hipStreamQuery(st); }, wait_limit_s());
}

void watchdog_loop(gs_ctx* c, double limit_s) {
  (void)hipSetDevice(c->cfg.device);
  const char* reported = nullptr;
  int64_t reported_t = 0;
  while (!c->wd_stop.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(250));
    const char* w = c->where.load();
    const int64_t t = c->where_t.load();
    if (!w || (w == reported && t == reported_t)) continue;
    const double s = (mono_ns() - t) * 1e-9;
    if (s < limit_s) continue;
    // which device work is still pending: the streams, and per batch slot its eval-pass end (evdone), commit end
    // (ev[4]) and readback end (ev[5]) (0 = complete, 1 = pending)
    auto q = [](hipError_t e) { return e == hipSuccess ? 0 : e == hipErrorNotReady ? 1 : 9; };
    fprintf(stderr, "gpuscore watchdog: rank %d of %d blocked %.1f s in %s (batch pass %llu, exchange %llu); pending: "
            "st %d st_ev %d st2 %d st_rb %d | slot 0 evdone %d ev4 %d ev5 %d | slot 1 evdone %d ev4 %d ev5 %d (bound %d)\n",
            c->rank, c->nranks, s, w, (unsigned long long)c->xbatch, (unsigned long long)c->xseq, q(hipStreamQuery(c->st)),
            q(hipStreamQuery(c->st_ev)), q(hipStreamQuery(c->st2)), q(hipStreamQuery(c->st_rb)),
            q(hipEventQuery(c->slot[0].ev_evdone)), q(hipEventQuery(c->slot[0].ev[4])), q(hipEventQuery(c->slot[0].ev[5])),
            q(hipEventQuery(c->slot[1].ev_evdone)), q(hipEventQuery(c->slot[1].ev[4])), q(hipEventQuery(c->slot[1].ev[5])),
            c->cur_slot);
    fflush(stderr);
    reported = w;
    reported_t = t;
  }
}
}  // namespace
void async_stop(gs_ctx* c);

namespace {

int fail(gs_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return code;
}

#define HIP_TRY(c, expr)                                                                    \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess) return fail((c), GS_EDEVICE, "%s: %s", #expr, hipGetErrorString(_e)); \
  } while (0)

// ---- DefaultEstimator (loadaware/estimator/default_estimator.go:57-108) ------------------------
int translate(int32_t prio, int r) {   // extension.TranslateResourceNameByPriorityClass
  if (prio == GS_PRIO_PROD || prio == GS_PRIO_NONE) return r;
  if (prio == GS_PRIO_BATCH) return r == 0 ? GS_RES_BATCH_CPU : GS_RES_BATCH_MEMORY;
  if (prio == GS_PRIO_MID) return r == 0 ? GS_RES_MID_CPU : GS_RES_MID_MEMORY;
  return -1;
}

int64_t estimate_resource(const gs_pod& p, int real, int64_t sf) {
  int64_t lim = real >= 0 ? p.limits[real] : 0, req = real >= 0 ? p.requests[real] : 0;
  int64_t q = req;
  if (lim > req) { sf = 100; q = lim; }
  if (q == 0) {
    if (real == GS_RES_CPU || real == GS_RES_BATCH_CPU) return kDefaultMilliCPURequest;
    if (real == GS_RES_MEMORY || real == GS_RES_BATCH_MEMORY) return kDefaultMemoryRequest;
    return 0;
  }
  int64_t e = (int64_t)std::round((double)q * (double)sf / 100);
  if (lim > 0 && e > lim) e = lim;
  return e;
}

Vec2 estimate_pod(const gs_loadaware_args& a, const gs_pod& p) {
  Vec2 o;
  for (int r = 0; r < 2; ++r) {
    if (!(a.resource_weights_mask & (1u << r))) continue;
    int64_t sf = (a.estimated_scaling_factors_mask & (1u << r)) ? a.estimated_scaling_factors[r] : 0;
    o.add(r, estimate_resource(p, translate(p.priority_class, r), sf));
  }
  return o;
}

int64_t estimate_node(const gs_node& n, int r) {   // EstimateNode (default_estimator.go:110-129)
  return (n.raw_allocatable_mask & (1u << r)) ? n.raw_allocatable[r] : n.allocatable[r];
}

// ---- LoadAware node-side derivations (loadaware/load_aware.go, helper.go) -----------------------
bool target_agg(const gs_node_metric& m, int64_t dur, int32_t type, Vec2* out) {   // helper.go:58-90
  if (!m.has_node_metric || m.n_aggregated <= 0 || type < 0 || type >= GS_NUM_AGG_TYPES) return false;
  int n = std::min(m.n_aggregated, GS_MAX_AGG_USAGES);
  if (dur == 0) {
    int64_t maxd = 0;
    int mi = 0;
    for (int i = 0; i < n; ++i)
      if (m.aggregated[i].duration_ns > maxd) { maxd = m.aggregated[i].duration_ns; mi = i; }
    if (m.aggregated[mi].type_mask & (1u << type)) {
      Vec2 u = usage_of(m.aggregated[mi].usage[type]);
      if (u.mask) { *out = u; return true; }
    }
    return false;
  }
  for (int i = 0; i < n; ++i) {
    if (m.aggregated[i].duration_ns != dur || !(m.aggregated[i].type_mask & (1u << type))) continue;
    Vec2 u = usage_of(m.aggregated[i].usage[type]);
    if (u.mask) { *out = u; return true; }
  }
  return false;
}

struct Thr {
  int64_t v[2] = {0, 0};
  uint32_t mask = 0;
};

// 0: within the thresholds; else 1 + the first exceeding resource in the order cpu, memory
int usage_exceeds(const Thr& th, const Vec2& used, const gs_node& n) {
  for (int r = 0; r < 2; ++r) {
    if (!(th.mask & (1u << r)) || th.v[r] == 0) continue;
    int64_t total = estimate_node(n, r);
    if (total == 0) continue;
    int64_t u = used.get(r);
    double mu = (double)(r == 0 ? u : u * 1000), mt = (double)(r == 0 ? total : total * 1000);
    int64_t pct = (int64_t)std::round(mu / mt * 100);   // load_aware.go:214,248
    if (pct >= th.v[r]) return 1 + r;
  }
  return 0;
}

struct LaDerived {
  uint32_t sflags = 0;
  int64_t used_np[2] = {0, 0};
  int64_t used_p[2] = {0, 0};
};

LaDerived derive_loadaware(const gs_loadaware_args& a, const HostNode& hn) {
  LaDerived d;
  const gs_node& n = hn.node;
  const gs_node_metric& m = hn.metric;
  // Score-side usage is derived even without a NodeMetric (Score then returns 0 anyway): the value is
  // what the row must hold once a metric appears, and what device-side Reserve deltas accumulate into.
  if (m.exists) d.sflags |= SF_METRIC;
  if (m.exists && m.has_update_time) d.sflags |= SF_UPDATE_TIME;
  // ---- Filter profile (helper.go:102-140)
  Thr usage{{a.usage_thresholds[0], a.usage_thresholds[1]}, a.usage_thresholds_mask};
  Thr prod{{a.prod_usage_thresholds[0], a.prod_usage_thresholds[1]}, a.prod_usage_thresholds_mask};
  bool has_agg = false;
  Thr agg;
  int32_t agg_type = GS_AGG_NONE;
  int64_t agg_dur = 0;
  if (n.custom_flags & GS_NODE_CUSTOM_THRESHOLDS) {
    if (n.custom_usage_mask) usage = Thr{{n.custom_usage_thresholds[0], n.custom_usage_thresholds[1]}, n.custom_usage_mask};
    if (n.custom_prod_usage_mask)
      prod = Thr{{n.custom_prod_usage_thresholds[0], n.custom_prod_usage_thresholds[1]}, n.custom_prod_usage_mask};
    if ((n.custom_flags & GS_NODE_CUSTOM_AGGREGATED) && n.custom_agg_usage_mask && n.custom_agg_type != GS_AGG_NONE) {
      has_agg = true;
      agg = Thr{{n.custom_agg_usage_thresholds[0], n.custom_agg_usage_thresholds[1]}, n.custom_agg_usage_mask};
      agg_type = n.custom_agg_type;
      agg_dur = n.custom_agg_duration_ns;
    }
  }
  if (!has_agg && a.has_aggregated && a.agg_usage_thresholds_mask && a.agg_usage_type != GS_AGG_NONE) {
    has_agg = true;
    agg = Thr{{a.agg_usage_thresholds[0], a.agg_usage_thresholds[1]}, a.agg_usage_thresholds_mask};
    agg_type = a.agg_usage_type;
    agg_dur = a.agg_usage_duration_ns;
  }
  // non-prod verdict: filterNodeUsage (load_aware.go:173-224)
  const Thr& th = has_agg ? agg : usage;
  if (m.exists && th.mask && m.has_node_metric) {
    Vec2 u;
    bool have = has_agg ? target_agg(m, agg_dur, agg_type, &u) : (u = usage_of(m.node_usage), true);
    const int ex = have ? usage_exceeds(th, u, n) : 0;
    if (ex) d.sflags |= SF_FAIL_NP | (ex == 2 ? SF_NP_MEM : 0u) | (has_agg ? SF_NP_AGG : 0u);
  }
  // prod verdict: filterProdUsage (load_aware.go:226-254)
  if (prod.mask) {
    d.sflags |= SF_PROD_THR;
    if (m.exists && !hn.pms.empty()) {
      std::unordered_map<uint64_t, Vec2> pm;
      for (const auto& e : hn.pms)
        if (e.in_lister && e.priority_class == GS_PRIO_PROD) pm[e.name_key] = usage_of(e.usage);
      Vec2 sum;
      for (const auto& kv : pm)
        for (int r = 0; r < 2; ++r)
          if (kv.second.has(r)) sum.add(r, kv.second.v[r]);
      const int ex = usage_exceeds(prod, sum, n);
      if (ex) d.sflags |= SF_FAIL_P | (ex == 2 ? SF_P_MEM : 0u);
    }
  }
  // ---- Score-side usage (load_aware.go:291-327, 337-376), for both prodPod modes
  int64_t update = m.has_update_time ? m.update_time_ns : kZeroTime;
  int64_t interval = m.has_report_interval ? m.report_interval_s * 1000000000LL : kDefaultReportIntervalNs;
  bool score_agg = a.has_aggregated && a.agg_score_type != GS_AGG_NONE;
  Vec2 score_usage;
  bool have_score_usage = false;
  if (score_agg) have_score_usage = target_agg(m, a.agg_score_duration_ns, a.agg_score_type, &score_usage);
  bool agg_missing = score_agg && !have_score_usage;
  for (int mode = 0; mode < 2; ++mode) {
    bool prod_mode = mode == 1;
    std::unordered_map<uint64_t, Vec2> pm;
    for (const auto& e : hn.pms) {
      if (!e.in_lister) continue;
      if (prod_mode && e.priority_class != GS_PRIO_PROD) continue;
      pm[e.name_key] = usage_of(e.usage);
    }
    Vec2 used;
    std::unordered_map<uint64_t, bool> estimated;
    for (const auto& kv : hn.assigned) {
      const Assigned& as = kv.second;
      if (prod_mode && as.pod.priority_class != GS_PRIO_PROD) continue;
      auto it = pm.find(as.pod.name_key);
      Vec2 pu;
      if (it != pm.end()) pu = it->second;
      bool est_it = pu.mask == 0 || as.ts > update || (as.ts < update && update - as.ts < interval) || agg_missing;
      if (!est_it) continue;
      Vec2 e = estimate_pod(a, as.pod);
      for (int r = 0; r < 2; ++r) {
        if (!e.has(r)) continue;
        int64_t v = e.v[r];
        if (pu.has(r) && pu.v[r] > v) v = pu.v[r];
        used.add(r, v);
      }
      estimated[as.pod.name_key] = true;
    }
    Vec2 actual, est_actual;
    for (const auto& kv : pm) {
      Vec2& dst = estimated.count(kv.first) ? est_actual : actual;
      for (int r = 0; r < 2; ++r)
        if (kv.second.has(r)) dst.add(r, kv.second.v[r]);
    }
    if (prod_mode) {
      for (int r = 0; r < 2; ++r) used.add(r, actual.get(r));
    } else if (m.has_node_metric) {
      Vec2 nu;
      bool have = score_agg ? have_score_usage : true;
      if (score_agg) nu = score_usage;
      else nu = usage_of(m.node_usage);
      if (have) {
        for (int r = 0; r < 2; ++r) {
          if (!nu.has(r)) continue;
          int64_t q = nu.v[r], e = est_actual.get(r);
          if (e != 0 && q >= e) q -= e;
          used.add(r, q);
        }
      }
    }
    int64_t* dst = prod_mode ? d.used_p : d.used_np;
    dst[0] = used.get(0);
    dst[1] = used.get(1);
  }
  return d;
}

gs_node reservation_view(const gs_ctx* c, uint32_t i, uint64_t owner);

void derive_row(const gs_ctx* c, uint32_t i, int64_t* row) {
  const HostNode& hn = c->nodes[i];
  // NodeInfo as a pod that matches none of the node's reservations sees it (reservation/transformer.go:266-292)
  const gs_node n = reservation_view(c, i, 0);
  for (int s = 0; s < 7; ++s) {
    row[C_FREE_CPU + s] = n.allocatable[s] - n.requested[s];
    row[C_ALLOC_CPU + s] = n.allocatable[s];
  }
  row[C_NZFREE_CPU] = n.allocatable[0] - n.nonzero_requested[0];
  row[C_NZFREE_MEM] = n.allocatable[1] - n.nonzero_requested[1];
  LaDerived d = derive_loadaware(c->cfg.loadaware, hn);
  for (int r = 0; r < 2; ++r) {
    int64_t cap = estimate_node(n, r);
    row[C_LA_CAP_CPU + r] = cap;
    row[C_LA_FREE_CPU + r] = cap - d.used_np[r];
    row[C_LA_PFREE_CPU + r] = cap - d.used_p[r];
  }
  row[C_UPDATE_TIME] = hn.metric.has_update_time ? hn.metric.update_time_ns : 0;
  int64_t fp = n.allowed_pod_number - n.pod_count;
  fp = std::max<int64_t>(INT32_MIN, std::min<int64_t>(INT32_MAX, fp));
  row[NUM_I64_COLS + C_FREE_PODS] = fp;
  row[NUM_I64_COLS + C_SFLAGS] = (int64_t)(d.sflags | (hn.valid ? SF_VALID : 0));
  row[NUM_I64_COLS + C_DFLAGS] = 0;
}

// ---- Reservation restore (reservation/transformer.go:50-292) on the host mirror ----------------------------------
// A reservation enters a pod's NodeInfo in BeforePreFilter: available ones (IsAvailable, no parse error, not an
// allocate-once reservation already used) that the pod matches are removed with their reserve pod (RemovePod); the
// others with assigned pods are "unmatched" and trimmed to their remaining resources (updateNodeInfoRequested).
bool rsv_usable(const gs_reservation& r) { return r.available && !(r.allocate_once && r.assigned_pods > 0); }
bool rsv_matches(const gs_reservation& r, uint64_t owner) {
  return owner != 0 && !r.unschedulable && r.owner_key == owner && rsv_usable(r);
}

// one-container pod requests -> (Requested delta per slot, NonZeroRequested delta): [upstream] calculateResource with
// schedutil.GetNonzeroRequests (100m / 200Mi for an absent cpu / memory key)
void rsv_request_delta(const int64_t* v, uint32_t mask, int64_t sign, int64_t* req, int64_t* nz) {
  for (int s = 0; s < GS_NUM_RES; ++s)
    if (mask >> s & 1u) req[s] += sign * v[s];
  nz[0] += sign * ((mask & 1u) ? v[0] : 100);
  nz[1] += sign * ((mask & 2u) ? v[1] : 200LL * 1024 * 1024);
}
// SubtractWithNonNegativeResult(Allocatable, Allocated): values and keys
uint32_t rsv_remained(const gs_reservation& r, int64_t* rem) {
  const uint32_t keys = r.allocatable_mask | r.allocated_mask;
  for (int s = 0; s < GS_NUM_RES; ++s) {
    const int64_t a = (r.allocatable_mask >> s & 1u) ? r.allocatable[s] : 0;
    const int64_t u = (r.allocated_mask >> s & 1u) ? r.allocated[s] : 0;
    rem[s] = (keys >> s & 1u) ? std::max<int64_t>(0, a - u) : 0;
  }
  return keys;
}
bool all_zero(const int64_t* v) {
  for (int s = 0; s < GS_NUM_RES; ++s)
    if (v[s]) return false;
  return true;
}
// restoreUnmatchedReservations on a NodeInfo copy
void rsv_trim_unmatched(const gs_reservation& r, gs_node& n) {
  rsv_request_delta(r.allocatable, r.allocatable_mask, -1, n.requested, n.nonzero_requested);
  int64_t rem[GS_NUM_RES];
  const uint32_t keys = rsv_remained(r, rem);
  if (!all_zero(rem)) rsv_request_delta(rem, keys, +1, n.requested, n.nonzero_requested);
}

// NodeInfo of node i as a pod with owner key `owner` sees it after the unmatched trim (podRequested; the matched
// reservations are not removed here)
gs_node reservation_view(const gs_ctx* c, uint32_t i, uint64_t owner) {
  gs_node n = c->nodes[i].node;
  if (c->rsv_node.empty() || !(c->ext.enabled & GS_EXT_RESERVATION)) return n;
  for (uint64_t uid : c->rsv_node[i]) {
    const gs_reservation& r = c->rsv.at(uid);
    if (!rsv_usable(r) || rsv_matches(r, owner) || r.assigned_pods <= 0) continue;
    rsv_trim_unmatched(r, n);
  }
  return n;
}

void derive_row_numa(const gs_ctx* c, uint32_t i, int64_t* row) {
  numa_derive(c->numa[i], c->cfg.numa.numa_scoring_type == GS_SCORING_MOST_ALLOCATED, row, row + NUM_I64_COLS);
}

bool in_range(int64_t v) { return v > -kMaxExact && v < kMaxExact; }

int validate_node(gs_ctx* c, const gs_node& n) {
  for (int s = 0; s < GS_NUM_RES; ++s)
    if (!in_range(n.allocatable[s]) || !in_range(n.requested[s]) || n.allocatable[s] < 0)
      return fail(c, GS_EUNSUPPORTED, "node resource slot %d outside the exact range [0, 2^53)", s);
  if (!in_range(n.nonzero_requested[0]) || !in_range(n.nonzero_requested[1]) || !in_range(n.raw_allocatable[0]) ||
      !in_range(n.raw_allocatable[1]) || n.raw_allocatable[0] < 0 || n.raw_allocatable[1] < 0)
    return fail(c, GS_EUNSUPPORTED, "node quantity outside the exact range [0, 2^53)");
  if (n.allocatable[GS_RES_RESERVED] || n.requested[GS_RES_RESERVED])
    return fail(c, GS_EINVAL, "resource slot 7 is reserved");
  return GS_OK;
}

PodVec prep_pod(const gs_ctx* c, const gs_pod& p) {
  PodVec v{};
  for (int s = 0; s < 7; ++s) v.req[s] = p.requests[s];
  v.nz[0] = p.nonzero_requests[0];
  v.nz[1] = p.nonzero_requests[1];
  Vec2 e = estimate_pod(c->cfg.loadaware, p);
  v.est[0] = e.get(0);
  v.est[1] = e.get(1);
  uint32_t f = 0;
  if (p.flags & GS_POD_DAEMONSET) f |= PF_DAEMONSET;
  if (p.priority_class == GS_PRIO_PROD) {
    f |= PF_PROD;
    if (c->cfg.loadaware.score_according_prod_usage) f |= PF_PROD_SCORE;
  }
  uint32_t scalar = p.request_mask & GS_SCALAR_RES_MASK;
  if (p.requests[0] == 0 && p.requests[1] == 0 && p.requests[2] == 0 && scalar == 0) f |= PF_ALL_ZERO;
  v.flags = f;
  v.scalar_mask = scalar;
  // NodeNUMAResource PreFilter (nodenumaresource/plugin.go:219-269)
  uint32_t keys = p.request_mask & 0x7Fu;
  v.req_keys = keys;
  bool zero = true;
  for (int s = 0; s < 7; ++s)
    if ((keys >> s & 1) && p.requests[s] != 0) zero = false;
  uint32_t pn = 0;
  int64_t cpu = (keys & 1u) ? p.requests[GS_RES_CPU] : 0;
  v.num_cpus = (int32_t)(cpu / 1000);
  if (zero) {
    pn |= PN_SKIP;
  } else if ((p.qos_class == GS_QOS_LSE || p.qos_class == GS_QOS_LSR) && p.priority_class == GS_PRIO_PROD) {
    const int def = c->cfg.numa.default_cpu_bind_policy;
    int bind = p.preferred_cpu_bind_policy;
    if (bind == GS_CPU_BIND_UNSET || bind == GS_CPU_BIND_DEFAULT) bind = def;
    int required = p.required_cpu_bind_policy;
    if (required == GS_CPU_BIND_DEFAULT) required = def;
    if (required != GS_CPU_BIND_UNSET) bind = required;
    if (bind == GS_CPU_BIND_FULL_PCPUS || bind == GS_CPU_BIND_SPREAD_BY_PCPUS) {
      if (cpu % 1000 != 0) pn |= PN_PREFAIL;
      else if (cpu > 0)
        pn |= PN_BIND | ((uint32_t)required << PN_REQ_SHIFT) | ((uint32_t)bind << PN_PREF_SHIFT) |
              ((uint32_t)p.preferred_cpu_exclusive_policy << PN_EXCL_SHIFT);
    }
  }
  v.numa = pn;
  return v;
}

// a pod the device path takes (msg: why not); no context state written (gs_schedule_submit runs it beside the worker)
int validate_pod_msg(bool numa_on, const gs_pod& p, char* msg, size_t len) {
  for (int s = 0; s < GS_NUM_RES; ++s)
    if (!in_range(p.requests[s]) || p.requests[s] < 0 || !in_range(p.limits[s]) || p.limits[s] < 0) {
      snprintf(msg, len, "pod resource slot %d outside the exact range [0, 2^53)", s);
      return GS_EUNSUPPORTED;
    }
  if (p.requests[GS_RES_RESERVED] || (p.request_mask & 0x80u)) {
    snprintf(msg, len, "resource slot 7 is reserved");
    return GS_EINVAL;
  }
  if (numa_on) {
    for (int s = 2; s < 7; ++s)
      if ((p.request_mask >> s & 1) && p.requests[s] == 0) {
        snprintf(msg, len, "NodeNUMAResource: a zero-valued request key other than cpu/memory (slot %d) is not "
                 "supported on the device path", s);
        return GS_EUNSUPPORTED;
      }
    if (p.required_cpu_bind_policy < 0 || p.required_cpu_bind_policy > 4 || p.preferred_cpu_bind_policy < 0 ||
        p.preferred_cpu_bind_policy > 4 || p.preferred_cpu_exclusive_policy < 0 || p.preferred_cpu_exclusive_policy > 2) {
      snprintf(msg, len, "pod cpu bind / exclusive policy out of range");
      return GS_EINVAL;
    }
  }
  return GS_OK;
}

int validate_pod(gs_ctx* c, const gs_pod& p) {
  char msg[256];
  const int rc = validate_pod_msg(c->numa_on, p, msg, sizeof msg);
  return rc ? fail(c, rc, "%s", msg) : GS_OK;
}

void mark_dirty(gs_ctx* c, uint32_t i) {
  if (!c->row_dirty[i]) {
    c->row_dirty[i] = 1;
    c->dirty_list.push_back(i);
  }
}

int flush_rows(gs_ctx* c) {
  if (c->dirty_list.empty()) return GS_OK;
  size_t done = 0;
  while (done < c->dirty_list.size()) {
    uint32_t n = (uint32_t)std::min<size_t>(c->stage_cap, c->dirty_list.size() - done);
    // staging buffers are reused: the previous scatter must have consumed them
    Where w_(c, "flush_rows: previous scatter");
    HIP_TRY(c, host_wait_stream(c->st));
    // one staged block, one copy: the n rows, then their node indices
    uint32_t* h_idx = reinterpret_cast<uint32_t*>(c->h_stage_rows + (size_t)n * ROW_WORDS);
    for (uint32_t j = 0; j < n; ++j) {
      uint32_t i = c->dirty_list[done + j];
      h_idx[j] = i;
      derive_row(c, i, c->h_stage_rows + (size_t)j * ROW_WORDS);
      derive_row_numa(c, i, c->h_stage_rows + (size_t)j * ROW_WORDS);
      c->row_dirty[i] = 0;
    }
    HIP_TRY(c, hipMemcpyAsync(c->d_stage_rows, c->h_stage_rows, (size_t)n * (ROW_WORDS * 8 + 4), hipMemcpyHostToDevice,
                              c->st));
    const uint32_t* d_idx = reinterpret_cast<const uint32_t*>(c->d_stage_rows + (size_t)n * ROW_WORDS);
    // with the rows' LoadAware verdicts at `now` (node_prep, fused into the scatter), unless a full pass is due anyway
    if (!c->prep_stale && c->prep_now == c->now) {
      const gs_loadaware_args& la = c->cfg.loadaware;
      const ScatterPrep sp{c->now, la.filter_expired_node_metrics, la.has_node_metric_expiration,
                           la.has_node_metric_expiration ? la.node_metric_expiration_seconds * 1000000000LL : 0};
      HIP_TRY(c, launch_scatter_rows(c->mv, d_idx, c->d_stage_rows, n, c->st, &sp));
    } else {
      HIP_TRY(c, launch_scatter_rows(c->mv, d_idx, c->d_stage_rows, n, c->st));
    }

    c->stats.delta_rows += n;
    c->stats.delta_bytes += (uint64_t)n * (4 + ROW_WORDS * 8);
    done += n;
  }
  c->dirty_list.clear();
  if (c->prep_now != c->now) c->prep_stale = true;
  return GS_OK;
}

int node_prep(gs_ctx* c) {
  const gs_loadaware_args& a = c->cfg.loadaware;
  int64_t exp_ns = a.has_node_metric_expiration ? a.node_metric_expiration_seconds * 1000000000LL : 0;
  HIP_TRY(c, launch_node_prep(c->mv, 0, c->N, c->now, a.filter_expired_node_metrics, a.has_node_metric_expiration,
                              exp_ns, c->st));
  c->prep_stale = false;
  c->prep_now = c->now;
  return GS_OK;
}

// every node upserted at least once (nodes never become invalid again: a count, not a scan of the N host rows — at
// 100k nodes the scan cost ~0.1 ms per gs_schedule call, i.e. per short plain run on the C5 extension path)
int ready(gs_ctx* c) {
  if (c->n_valid == c->N) return GS_OK;
  for (uint32_t i = 0; i < c->N; ++i)
    if (!c->nodes[i].valid) return fail(c, GS_ESTATE, "node %u was never upserted", i);
  return GS_OK;
}

double ev_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();   // (an event without timing: not sticky for the next launch's check)
    return 0;
  }
  return ms;
}

// exchange_ms of RCCL all-gathers: completion time from events around each collective on the stream, added up once
// a collective's end event has completed (finish_batch); the pairs of a speculative batch still in flight stay pending
void flush_exchange_times(gs_ctx* c) {
  int keep = 0;
  for (int i = 0; i < c->x_pending; ++i) {
    hipEvent_t a = c->x_ev[2 * i], b = c->x_ev[2 * i + 1];
    if (hipEventQuery(b) == hipSuccess) {
      c->stats.exchange_ms += ev_ms(a, b);
    } else {   // still in flight: keep the pair (moved to the front)
      std::swap(c->x_ev[2 * keep], c->x_ev[2 * i]);
      std::swap(c->x_ev[2 * keep + 1], c->x_ev[2 * i + 1]);
      ++keep;
    }
  }
  c->x_pending = keep;
}

constexpr size_t XSMALL = 64;   // small exchange block: payload <= 32 B, XTag at 32

const char* xsite_name(uint32_t s) {
  return s == XSITE_LEVELS ? "levels" : s == XSITE_ROWSTAT ? "row stats" : s == XSITE_SELECT ? "selection"
       : s == XSITE_SCORES ? "score rows" : s == XSITE_RUNS ? "run boundary" : "?";
}

// The R received blocks' tags against the tag this rank sent: every rank checks all of them, so a divergence fails
// on every rank at the same exchange.
int check_tags(gs_ctx* c, const uint8_t* blocks, size_t bytes, const XTag& mine) {
  for (int r = 0; r < c->nranks; ++r) {
    XTag t;
    std::memcpy(&t, blocks + (size_t)r * bytes + bytes - sizeof(XTag), sizeof t);
    if (t.magic != XTAG_MAGIC || t.site != mine.site || t.seq != mine.seq || t.batch != mine.batch || t.rank != r ||
        t.bytes != mine.bytes)
      return fail(c, GS_ECOMM,
                  "exchange sequence diverged: rank %d is at exchange %llu (%s, batch %llu), rank %d sent exchange %llu "
                  "(%s, batch %llu, %u bytes, magic %#x)",
                  c->rank, (unsigned long long)mine.seq, xsite_name(mine.site), (unsigned long long)mine.batch, r,
                  (unsigned long long)t.seq, xsite_name(t.site), (unsigned long long)t.batch, t.bytes, t.magic);
  }
  return GS_OK;
}

// One all-gather of `bytes`-byte blocks (each ending in an XTag, filled here) from d_send into R blocks at d_recv.
// RCCL: stream-ordered, the tag written on the stream before the collective; the receiver checks the tags (the level
// blocks on the device in merge_levels_kernel, the small ones on the host). Callback: host-synchronous, checked here.
int exchange(gs_ctx* c, uint32_t site, uint8_t* d_send, uint8_t* d_recv, size_t bytes, XTag* sent = nullptr,
             hipStream_t xs = nullptr) {
  auto t0 = std::chrono::steady_clock::now();
  if (!xs) xs = c->st;
  // the host-callback transport's staging: the score blocks have their own buffers
  uint8_t* h_send = site == XSITE_SCORES ? c->h_sx_send : c->h_xchg_send;
  uint8_t* h_recv = site == XSITE_SCORES ? c->h_sx_recv : c->h_xchg_recv;
  const size_t h_cap = site == XSITE_SCORES ? c->sx_bytes : c->xchg_bytes;
  if (bytes < sizeof(XTag) || bytes % 8) return fail(c, GS_EINVAL, "exchange block of %zu bytes", bytes);
  XTag tag{XTAG_MAGIC, site, ++c->xseq, c->xbatch, c->rank, (uint32_t)bytes};
  if (c->rank == c->dbg_xskew_rank && c->xbatch == c->dbg_xskew_batch && (site == XSITE_LEVELS || site == XSITE_SCORES))
    tag.seq = ++c->xseq;
  if (sent) *sent = tag;
  if (c->comm) {
    HIP_TRY(c, launch_write_tag(d_send + bytes - sizeof(XTag), tag, xs));
    if (c->x_pending * 2 + 2 > (int)c->x_ev.size()) {
      for (int k = 0; k < 2; ++k) {
        hipEvent_t ev;
        HIP_TRY(c, hipEventCreate(&ev));
        c->x_ev.push_back(ev);
      }
    }
    HIP_TRY(c, hipEventRecord(c->x_ev[2 * c->x_pending], xs));
    ncclResult_t r = ncclAllGather(d_send, d_recv, bytes, ncclUint8, c->comm, xs);
    if (r != ncclSuccess) return fail(c, GS_ECOMM, "ncclAllGather: %s", ncclGetErrorString(r));
    HIP_TRY(c, hipEventRecord(c->x_ev[2 * c->x_pending + 1], xs));
    ++c->x_pending;
    return GS_OK;
  } else if (c->lg) {
    gs_local_group& g = *c->lg;
    static const double limit = getenv("GS_LOCAL_WAIT_S") ? atof(getenv("GS_LOCAL_WAIT_S")) : 60.0;
    HIP_TRY(c, launch_write_tag(d_send + bytes - sizeof(XTag), tag, xs));
    if (c->x_pending * 2 + 2 > (int)c->x_ev.size()) {
      for (int k = 0; k < 2; ++k) {
        hipEvent_t ev;
        HIP_TRY(c, hipEventCreate(&ev));
        c->x_ev.push_back(ev);
      }
    }
    HIP_TRY(c, hipEventRecord(c->x_ev[2 * c->x_pending], xs));
    HIP_TRY(c, hipEventRecord(c->lg_ready, xs));
    {
      std::lock_guard<std::mutex> lk(g.mu);
      g.send[c->rank] = d_send;
      g.bytes[c->rank] = bytes;
      g.ready[c->rank] = c->lg_ready;
    }
    bool met;
    {
      Where w_(c, "exchange (local transport): the ranks' send blocks");
      met = g.meet(limit);
    }
    if (!met)
      return fail(c, GS_ECOMM, "local transport: a rank did not reach exchange %llu (%s, batch %llu) within %.0f s",
                  (unsigned long long)tag.seq, xsite_name(site), (unsigned long long)tag.batch, limit);
    bool same = true;
    for (int s = 0; s < c->nranks; ++s) same = same && g.bytes[s] == bytes;
    if (same)
      for (int s = 0; s < c->nranks; ++s) {
        HIP_TRY(c, hipStreamWaitEvent(xs, g.ready[s], 0));
        HIP_TRY(c, hipMemcpyAsync(d_recv + (size_t)s * bytes, g.send[s], bytes, hipMemcpyDeviceToDevice, xs));
      }
    HIP_TRY(c, hipEventRecord(c->lg_done, xs));
    {
      std::lock_guard<std::mutex> lk(g.mu);
      g.done[c->rank] = c->lg_done;
    }
    {
      Where w_(c, "exchange (local transport): the ranks' copies");
      met = g.meet(limit);
    }
    if (!met)
      return fail(c, GS_ECOMM, "local transport: a rank did not finish exchange %llu (%s, batch %llu) within %.0f s",
                  (unsigned long long)tag.seq, xsite_name(site), (unsigned long long)tag.batch, limit);
    if (!same) return fail(c, GS_ECOMM, "local transport: the ranks' blocks of exchange %llu differ in size",
                           (unsigned long long)tag.seq);
    for (int s = 0; s < c->nranks; ++s)
      if (s != c->rank) HIP_TRY(c, hipStreamWaitEvent(xs, g.done[s], 0));
    HIP_TRY(c, hipEventRecord(c->x_ev[2 * c->x_pending + 1], xs));
    ++c->x_pending;
    return GS_OK;
  } else if (c->cb) {
    if (bytes > h_cap || !h_send) return fail(c, GS_EINVAL, "exchange payload too large");
    Where w_(c, site == XSITE_LEVELS   ? "exchange (levels): stream before the callback"
                : site == XSITE_SCORES ? "exchange (score rows): stream before the callback"
                                       : "exchange (small): stream before the callback");
    HIP_TRY(c, hipMemcpyAsync(h_send, d_send, bytes - sizeof(XTag), hipMemcpyDeviceToHost, xs));
    HIP_TRY(c, host_wait_stream(xs));
    c->where.store("exchange: allgather callback");
    std::memcpy(h_send + bytes - sizeof(XTag), &tag, sizeof tag);
    if (c->cb(c->cb_user, h_send, h_recv, bytes) != 0) return fail(c, GS_ECOMM, "allgather callback failed");
    if (int rc = check_tags(c, h_recv, bytes, tag)) return rc;
    HIP_TRY(c, hipMemcpyAsync(d_recv, h_recv, bytes * c->nranks, hipMemcpyHostToDevice, xs));
  } else {
    return fail(c, GS_ESTATE, "multi-rank context without a communicator");
  }
  c->stats.exchange_ms +=
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return GS_OK;
}

// A small exchange (payload <= 32 B at d_payload, device) and its R payloads read back to host_out (R x payload bytes).
// xs: the stream (default st); a host payload (d_payload == nullptr) is taken from host_in.
int exchange_small(gs_ctx* c, uint32_t site, const void* d_payload, size_t payload, void* host_out,
                   hipStream_t xs = nullptr, const void* host_in = nullptr) {
  static_assert(XSMALL >= 32 + sizeof(XTag), "small exchange block");
  if (payload > XSMALL - sizeof(XTag)) return fail(c, GS_EINVAL, "small exchange payload too large");
  if (!xs) xs = c->st;
  if (d_payload) {
    HIP_TRY(c, hipMemcpyAsync(c->d_xsmall, d_payload, payload, hipMemcpyDeviceToDevice, xs));
  } else {   // (h_xsmall is free between small exchanges: staged through it, in stream order)
    std::memcpy(c->h_xsmall, host_in, payload);
    HIP_TRY(c, hipMemcpyAsync(c->d_xsmall, c->h_xsmall, payload, hipMemcpyHostToDevice, xs));
  }
  XTag tag{};
  if (int rc = exchange(c, site, c->d_xsmall, c->d_xsmall + XSMALL, XSMALL, &tag, xs)) return rc;
  HIP_TRY(c, hipMemcpyAsync(c->h_xsmall, c->d_xsmall + XSMALL, XSMALL * c->nranks, hipMemcpyDeviceToHost, xs));
  Where w_(c, "exchange_small: read back");
  HIP_TRY(c, host_wait_stream(xs));
  if (int rc = check_tags(c, c->h_xsmall, XSMALL, tag)) return rc;
  for (int r = 0; r < c->nranks; ++r)
    std::memcpy(static_cast<uint8_t*>(host_out) + (size_t)r * payload, c->h_xsmall + (size_t)r * XSMALL, payload);
  return GS_OK;
}

bool special_pod(const gs_ctx* c, const gs_pod& p) {
  // Placements whose LoadAware effect is not "+EstimatePod" on the chosen row: the pod UID already sits
  // in an assign cache, a PodMetric with the pod's name exists, or the pod is terminated (assign skips it).
  if (p.flags & GS_POD_TERMINATED) return true;
  if (c->uid_node.count(p.uid)) return true;
  if (c->metric_names.count(p.name_key)) return true;
  if (c->numa_on && c->numa_uid_node.count(p.uid)) return true;   // Update() would release its old allocation
  return false;
}

// NodeNUMAResource Reserve (nodenumaresource/plugin.go:375-422) replayed on the host mirror: NUMA resources
// along the device-chosen affinity (already applied to HBM by the commit kernel), and for cpuset pods the
// cpuset selection itself (resourceManager.Allocate -> allocateCPUSet -> takeCPUs).
int numa_reserve(gs_ctx* c, const gs_pod& p, const PodVec& v, const PlacementDev& pd) {
  if (!c->numa_on || pd.node < 0) return GS_OK;
  if (v.numa & (PN_SKIP | PN_PREFAIL)) return GS_OK;
  NumaNode& nn = c->numa[pd.node];
  const bool rb = pd.flags & GS_PLACED_CPUSET;
  if (!rb && nn.cfg.numa_topology_policy == GS_NUMA_POLICY_NONE) return GS_OK;
  PodAllocRec rec;
  rec.uid = p.uid;
  rec.excl = (v.numa & PN_BIND) ? p.preferred_cpu_exclusive_policy : GS_CPU_EXCLUSIVE_NONE;
  for (int z = 0; z < GS_MAX_NUMA; ++z) {
    if (!(pd.zkeys >> z & 1) && !(pd.zkeys >> (4 + z) & 1)) continue;
    gs_numa_zone a{};
    a.node_id = nn.cfg.zones[z].node_id;
    if (pd.zkeys >> z & 1) { a.mask |= GS_USAGE_CPU; a.cpu_milli = pd.zcpu[z]; }
    if (pd.zkeys >> (4 + z) & 1) { a.mask |= GS_USAGE_MEMORY; a.memory = pd.zmem[z]; }
    rec.numa.push_back(a);
  }
  if (pd.flags & PL_RESERVE_FAILED)
    return fail(c, GS_ESTATE, "NodeNUMAResource Reserve failed on the device for node %d after a feasible Filter",
                pd.node);
  const bool on_device = pd.flags & PL_DEVICE_CPUSET;   // the commit kernel chose the cpuset and updated the row
  if (rb && (!on_device || c->verify_cpuset)) {
    // getCPUBindPolicy (util.go:85-103) and GetNUMAAllocateStrategy (util.go:35-41)
    int req = (v.numa >> PN_REQ_SHIFT) & 7, pref = (v.numa >> PN_PREF_SHIFT) & 7;
    int bind = pref;
    bool required = false;
    if (req != GS_CPU_BIND_UNSET) { bind = req; required = true; }
    else if (nn.cfg.node_cpu_bind_policy == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS) { bind = GS_CPU_BIND_SPREAD_BY_PCPUS; required = true; }
    else if (nn.cfg.node_cpu_bind_policy == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY) { bind = GS_CPU_BIND_FULL_PCPUS; required = true; }
    int strategy = nn.cfg.numa_allocate_strategy;
    if (strategy == GS_NUMA_ALLOC_UNSET)
      strategy = c->cfg.numa.numa_scoring_type == GS_SCORING_MOST_ALLOCATED ? GS_NUMA_ALLOC_MOST_ALLOCATED
                                                                          : GS_NUMA_ALLOC_LEAST_ALLOCATED;
    if (!numa_allocate_cpuset(nn, v.num_cpus, bind, required, rec.excl, strategy, rec.numa, &rec.cpus))
      return fail(c, GS_ESTATE, "NodeNUMAResource Reserve: cpuset allocation failed on node %d after a feasible Filter",
                  pd.node);
    if (on_device && std::memcmp(rec.cpus.w, pd.cpuset, sizeof(pd.cpuset)) != 0)
      return fail(c, GS_ESTATE, "NodeNUMAResource Reserve: device cpuset differs from the host takeCPUs on node %d",
                  pd.node);
  }
  if (on_device)
    for (int w = 0; w < GS_CPU_WORDS; ++w) rec.cpus.w[w] = pd.cpuset[w];
  if (!nn.topo_valid()) return GS_OK;   // resourceManager.Update skips nodes without a valid CPU topology
  numa_release(nn, rec.uid);
  numa_add(nn, rec);
  c->numa_uid_node[rec.uid] = (uint32_t)pd.node;
  if (rb && !on_device) mark_dirty(c, (uint32_t)pd.node);
  return GS_OK;
}

void apply_placement(gs_ctx* c, const gs_pod& p, int32_t node, bool special) {
  if (node < 0) return;
  HostNode& hn = c->nodes[node];
  for (int s = 0; s < GS_NUM_RES; ++s) hn.node.requested[s] += p.requests[s];
  hn.node.nonzero_requested[0] += p.nonzero_requests[0];
  hn.node.nonzero_requested[1] += p.nonzero_requests[1];
  hn.node.pod_count += 1;
  if (!(p.flags & GS_POD_TERMINATED)) {
    hn.assigned[p.uid] = Assigned{c->now, p};
    c->uid_node[p.uid] = (uint32_t)node;
  }
  if (special) mark_dirty(c, (uint32_t)node);
}

void index_metric_names(gs_ctx* c, const HostNode& hn, int delta) {
  for (const auto& e : hn.pms) {
    auto it = c->metric_names.find(e.name_key);
    if (delta > 0) {
      c->metric_names[e.name_key] += 1;
    } else if (it != c->metric_names.end()) {
      if (--it->second <= 0) c->metric_names.erase(it);
    }
  }
}

int compute_profile(gs_ctx* c) {
  const gs_config& cfg = c->cfg;
  Profile& pf = c->pf;
  pf = Profile{};
  pf.enabled = cfg.enabled & 0x3Fu;
  c->numa_on = (pf.enabled & (GS_ENABLE_NUMA_FILTER | GS_ENABLE_NUMA_SCORE)) != 0;
  pf.w_numa = (int32_t)cfg.plugin_weights[GS_PLUGIN_NUMA];
  for (int s = 0; s < 7; ++s) {
    int64_t w = cfg.numa.resource_weights[s];
    if (w < 0 || w > 100) return fail(c, GS_EINVAL, "NodeNUMAResource weight of slot %d not in [0, 100]", s);
    pf.numa_w[s] = (int32_t)w;
  }
  pf.numa_most = cfg.numa.scoring_type == GS_SCORING_MOST_ALLOCATED;
  pf.numa_hint_most = cfg.numa.numa_scoring_type == GS_SCORING_MOST_ALLOCATED;
  {
    int d = cfg.numa.default_cpu_bind_policy;   // validation.ValidateNodeNUMAResourceArgs (validation_pluginargs.go:156-172)
    if (d != GS_CPU_BIND_UNSET && d != GS_CPU_BIND_FULL_PCPUS && d != GS_CPU_BIND_SPREAD_BY_PCPUS)
      return fail(c, GS_EINVAL, "defaultCPUBindPolicy must specified CPU bind policy FullPCPUs or SpreadByPCPUs");
  }
  pf.w_fit = (int32_t)cfg.plugin_weights[GS_PLUGIN_FIT];
  pf.w_la = (int32_t)cfg.plugin_weights[GS_PLUGIN_LOADAWARE];
  for (int r = 0; r < 2; ++r) {
    if (cfg.loadaware.resource_weights_mask & (1u << r)) pf.la_w[r] = (int32_t)cfg.loadaware.resource_weights[r];
    pf.la_wsum += pf.la_w[r];
  }
  for (int s = 0; s < 7; ++s) {
    int64_t w = cfg.fit.resource_weights[s];
    if (w < 0 || w > 100) return fail(c, GS_EINVAL, "NodeResourcesFit weight of slot %d not in (0, 100]", s);
    pf.fit_w[s] = (int32_t)w;
    if (s >= 2 && w) pf.fit_scalar_w_mask |= 1u << s;
  }
  if (cfg.fit.resource_weights[7]) return fail(c, GS_EINVAL, "resource slot 7 is reserved");
  if ((pf.enabled & GS_ENABLE_LA_SCORE) && pf.la_wsum == 0)
    return fail(c, GS_EINVAL, "LoadAwareScheduling scoring needs at least one resource weight");
  int64_t ms = 0;
  if (pf.enabled & GS_ENABLE_FIT_SCORE) ms += 100 * cfg.plugin_weights[GS_PLUGIN_FIT];
  if (pf.enabled & GS_ENABLE_LA_SCORE) ms += 100 * cfg.plugin_weights[GS_PLUGIN_LOADAWARE];
  if (pf.enabled & GS_ENABLE_NUMA_SCORE) ms += 100 * cfg.plugin_weights[GS_PLUGIN_NUMA];
  if (cfg.plugin_weights[0] < 0 || cfg.plugin_weights[1] < 0 || cfg.plugin_weights[2] < 0 || ms > MAX_SCORE_LIMIT)
    return fail(c, GS_EUNSUPPORTED, "profile score weights must keep the max total score <= %d (got %lld)",
                MAX_SCORE_LIMIT, (long long)ms);
  c->max_score = (int)ms;
  return GS_OK;
}

// GS_XCHG=levels (read at every comm init): the per-shard candidate levels instead of the score rows
bool xchg_levels() { return getenv("GS_XCHG") && std::strcmp(getenv("GS_XCHG"), "levels") == 0; }

void set_shard(gs_ctx* c) {
  uint32_t per = (c->N + c->nranks - 1) / c->nranks;
  c->e0 = std::min(c->N, per * (uint32_t)c->rank);
  c->e1 = std::min(c->N, c->e0 + per);
  c->sgather = c->nranks > 1 && !xchg_levels();
  c->n0 = c->sgather ? 0 : c->e0;
  c->n1 = c->sgather ? c->N : c->e1;
  c->sx_per = per;
  c->sx_pld = (per + 1023) / 1024 * 1024;
  c->stats.shard_begin = c->e0;
  c->stats.shard_end = c->e1;
}

// ranks whose candidate levels the commit merges: 1 unless the ranks exchange level lists (GS_XCHG=levels)
int lvl_ranks(const gs_ctx* c) { return c->sgather ? 1 : c->nranks; }

// one rank's exchange block: [B x lstride listed node ids | B LevelHdr | B LevelExt | ... | XTag], padded to 256 B (the
// tag in the block's last 32 bytes)
size_t lists_bytes(int B, int lstride) { return (size_t)B * lstride * 4; }
size_t xchg_block_bytes(int B, int lstride) {
  size_t raw = lists_bytes(B, lstride) + (size_t)B * (sizeof(LevelHdr) + sizeof(LevelExt)) + sizeof(XTag);
  return (raw + 255) / 256 * 256;
}

int alloc_exchange(gs_ctx* c) {
  // the speculative commit merges the shards' lists: XCAP listed nodes per (pod, shard) are enough for a pod at batch
  // position k (k + 1 per shard), and the all-gathered block is 8x smaller; the other kernels read LCAP-wide blocks
  // (score rows: every rank runs the one-shard pipeline over all nodes, LCAP-wide local lists)
  c->lstride = !c->sgather && commit_spec_selected(c->window_k) ? XCAP : LCAP;
  c->xchg_bytes = xchg_block_bytes(c->B, c->lstride);
  if (c->d_xchg_recv) { (void)hipFree(c->d_xchg_recv); c->d_xchg_recv = nullptr; }
  if (c->h_xchg_recv) { (void)hipHostFree(c->h_xchg_recv); c->h_xchg_recv = nullptr; }
  HIP_TRY(c, hipMalloc(&c->d_xchg_recv, c->xchg_bytes * c->nranks + 64));
  HIP_TRY(c, hipHostMalloc(&c->h_xchg_recv, c->xchg_bytes * c->nranks + 64, hipHostMallocDefault));
  if (c->d_xmerged) { (void)hipFree(c->d_xmerged); c->d_xmerged = nullptr; }
  HIP_TRY(c, hipMalloc(&c->d_xmerged, xchg_block_bytes(c->B, LCAP) + 64));
  if (!c->d_xerr) HIP_TRY(c, hipMalloc(&c->d_xerr, 2 * XERR_BYTES));   // one per batch slot (score rows)
  HIP_TRY(c, hipMemset(c->d_xerr, 0, 2 * XERR_BYTES));
  if (c->d_sx_send) { (void)hipFree(c->d_sx_send); c->d_sx_send = nullptr; }
  if (c->d_sx_recv) { (void)hipFree(c->d_sx_recv); c->d_sx_recv = nullptr; }
  if (c->h_sx_send) { (void)hipHostFree(c->h_sx_send); c->h_sx_send = nullptr; }
  if (c->h_sx_recv) { (void)hipHostFree(c->h_sx_recv); c->h_sx_recv = nullptr; }
  c->sx_bytes = 0;
  if (c->sgather) {
    c->sx_bytes = ((size_t)c->B * c->sx_pld * 3 + sizeof(XTag) + 255) / 256 * 256;
    HIP_TRY(c, hipMalloc(&c->d_sx_send, c->sx_bytes * 2));               // one per batch slot
    HIP_TRY(c, hipMalloc(&c->d_sx_recv, c->sx_bytes * c->nranks * 2));
    if (c->cb) {
      HIP_TRY(c, hipHostMalloc(&c->h_sx_send, c->sx_bytes, hipHostMallocDefault));
      HIP_TRY(c, hipHostMalloc(&c->h_sx_recv, c->sx_bytes * c->nranks, hipHostMallocDefault));
    }
  }
  if (!c->d_xsmall) HIP_TRY(c, hipMalloc(&c->d_xsmall, XSMALL * (1 + MAX_RANKS)));
  if (!c->h_xsmall) HIP_TRY(c, hipHostMalloc(&c->h_xsmall, XSMALL * MAX_RANKS, hipHostMallocDefault));
  if (const char* sk = getenv("GS_DEBUG_XCHG_SKEW")) {   // "rank:batch" (tests of the sequence check)
    long r = -1;
    unsigned long long b = 0;
    if (sscanf(sk, "%ld:%llu", &r, &b) == 2) { c->dbg_xskew_rank = r; c->dbg_xskew_batch = b; }
  }
  return GS_OK;
}


void bind_slot(gs_ctx* c, int s) {
  const gs_ctx::Slot& x = c->slot[s];
  c->d_S = x.d_S; c->d_aff = x.d_aff;
  c->d_pods = x.d_pods; c->d_seq = x.d_seq; c->d_out = x.d_out; c->d_committed = x.d_committed;
  c->h_pods = x.h_pods; c->h_seq = x.h_seq; c->h_out = x.h_out; c->h_committed = x.h_committed;
  for (int i = 0; i < 6; ++i) c->ev[i] = x.ev[i];
  c->d_lst = x.d_lst; c->d_hist = x.d_hist;
  c->cur_slot = s;
}

constexpr int GS_REDO = 1;   // internal: re-run the batch (its score rows were overwritten by a speculative pass)
constexpr size_t COMMITTED_BYTES = 32;   // committed[0..7] (the commit kernels write [0..4]); the placements follow

// The candidate levels of a one-shard pass without node sampling are built on st_ev right after the eval pass (beside
// the previous batch's commit, on the stale rows it lands on), then fixed up on st once that commit is done
// (GS_FUSED_PATCH=0, the separate patch kernel: not overlapped)
// A batch with no speculative pass before it, of at most GS_DIRECT_B pods (default 32; 0: none), on one shard: its
// upload, eval pass and levels go on st in order instead of through st_ev. st_ev then waits for that eval pass and its
// levels (launch_batch): a speculative pass enqueued after it on st_ev shares the NUMA slab, st2 and the fork / join
// events with it, so it starts only once they are done. Short runs (the plain pods between C5's extension pods) lose
// two queue hops per batch.
bool direct_batch(const gs_ctx* c, int b, bool speculative) {
  static const int max_b = getenv("GS_DIRECT_B") ? atoi(getenv("GS_DIRECT_B")) : 32;
  return !speculative && b <= max_b && lvl_ranks(c) == 1;
}

bool cand_overlapped(const gs_ctx* c) {
  static const bool separate = getenv("GS_FUSED_PATCH") && getenv("GS_FUSED_PATCH")[0] == '0';
  return c->cand_overlap && lvl_ranks(c) == 1 && !c->window_k && c->d_lst && !separate;
}

CommitArgs commit_args(gs_ctx* c, int b) {
  CommitArgs a{};
  a.m = c->mv;
  a.pods = c->d_pods;
  a.seq = c->d_seq;
  a.npods = b;
  a.nranks = lvl_ranks(c);
  a.shard_size = (c->N + a.nranks - 1) / a.nranks;
  // several ranks: the speculative commit reads the merged levels, the pipelined / lockstep kernels every rank block
  a.xbase = a.nranks == 1 ? (cand_overlapped(c) ? c->d_lst : c->d_xchg_send)
                            : commit_spec_selected(c->window_k) ? c->d_xmerged : c->d_xchg_recv;
  a.xblock = c->xchg_bytes;
  a.bmax = c->B;
  a.pf = c->pf;
  a.seed = c->cfg.seed;
  a.forced_node = -1;
  a.out = c->d_out;
  a.committed = c->d_committed;
  a.stamps = c->d_stamps;
  a.topos = c->d_topos;
  a.aff = c->d_aff;
  a.ld = c->ld;
  a.own0 = c->n0;
  a.own1 = c->n1;
  a.S = a.nranks == 1 ? c->d_S : nullptr;
  a.S_own = c->d_S;
  a.window_k = c->window_k;
  a.start = c->next_start;
  a.nnodes = c->N;
  static const bool nospec = getenv("GS_SPEC_WAIT") && getenv("GS_SPEC_WAIT")[0] == '1';
  // GS_SPEC_PRIO (experiments): issue priorities of the roles, bits 4-5 Reserve, 6-7 re-scoring, 8-9 verify
  static const uint32_t prio = getenv("GS_SPEC_PRIO") ? (uint32_t)strtoul(getenv("GS_SPEC_PRIO"), nullptr, 0) & 0x3f0u : 0u;
  // GS_SPEC_LAG (experiments): decisions ahead of the verifier, 1..12 (bits 12-15; 0: the kernel's SP_LAG)
  static const uint32_t lag = getenv("GS_SPEC_LAG") ? (uint32_t)std::min(12L, std::max(0L, atol(getenv("GS_SPEC_LAG")))) : 0u;
  // the split selector (one shard; a prep wave decides ahead over a snapshot, wave 0 applies the landings after it),
  // bit 16: the default (GS_SPEC_SPLIT=0: the single selector wave); GS_SPEC_SPLIT=2 (experiments): and the decided
  // pods verified by the re-scoring / Reserve waves (bit 17)
  static const int split = getenv("GS_SPEC_SPLIT") ? atoi(getenv("GS_SPEC_SPLIT")) : 1;
  // GS_SPEC_AHEAD=2 (experiments): the prep wave may run two pods ahead (bit 18)
  static const bool ahead2 = getenv("GS_SPEC_AHEAD") && getenv("GS_SPEC_AHEAD")[0] == '2';
  // GS_SPEC_SPLIT=3 (experiments): shared verification by the prep wave while it waits (bits 17 and 19)
  a.dbg = (nospec ? 1u : 0u) | prio | lag << 12 | (split >= 1 ? 1u << 16 : 0u) | (split >= 2 ? 1u << 17 : 0u) |
          (ahead2 ? 1u << 18 : 0u) | (split >= 3 ? 1u << 19 : 0u);
  a.tb = c->d_tb;
  // (score rows: the batch slot's verdict of unpack_scores_kernel; levels: merge_levels_kernel's)
  a.xerr = c->sgather ? c->d_xerr + (XERR_BYTES / 4) * c->cur_slot : c->nranks > 1 ? c->d_xerr : nullptr;
  return a;
}

// Enqueue one device pass over pods [0, b) of the bound slot's staged batch, and its read-back; no host wait.
// The eval pass runs on st_ev, the rest on st. prev != nullptr: a speculative pass behind the batch that wrote `prev`
// (its placements prev_out, prev_b pods): its eval pass runs beside that batch's commit, on the mirror as it was
// before it, and the rows that batch landed on are re-evaluated on st once it committed (patch_kernel); its commit
// kernel does nothing unless that batch committed every pod and needs no host-side Reserve (prev[1] == 1).
int launch_batch(gs_ctx* c, int b, const int32_t* prev, const PlacementDev* prev_out = nullptr, int prev_b = 0) {
  static const bool separate = getenv("GS_FUSED_PATCH") && getenv("GS_FUSED_PATCH")[0] == '0';
  const bool ovl = cand_overlapped(c);
  uint8_t* lblk = ovl ? c->d_lst : c->d_xchg_send;
  uint32_t* d_lists = reinterpret_cast<uint32_t*>(lblk);
  LevelHdr* d_hdrs = reinterpret_cast<LevelHdr*>(lblk + lists_bytes(c->B, c->lstride));
  LevelExt* d_ext = reinterpret_cast<LevelExt*>(lblk + lists_bytes(c->B, c->lstride) + (size_t)c->B * sizeof(LevelHdr));
  int prod_cols = 0;
  for (int i = 0; i < b; ++i) prod_cols |= (c->h_pods[i].flags & PF_PROD_SCORE) ? 1 : 0;
  uint32_t len = c->n1 - c->n0;
  if (c->numa_on && (c->numa_idx_stale || c->numa_idx_lo != c->e0 || c->numa_idx_hi != c->e1)) {
    std::vector<uint32_t> idx;   // the policy nodes this rank evaluates
    for (uint32_t n = c->e0; n < c->e1; ++n)
      if (c->numa[n].cfg.numa_topology_policy != GS_NUMA_POLICY_NONE) idx.push_back(n);
    if (c->d_numa_idx) {
      HIP_TRY(c, host_wait_stream(c->st));
      HIP_TRY(c, host_wait_stream(c->st_ev));
      (void)hipFree(c->d_numa_idx);
      c->d_numa_idx = nullptr;
    }
    c->numa_n = (uint32_t)idx.size();
    if (c->numa_n) {
      HIP_TRY(c, hipMalloc(&c->d_numa_idx, 4 * idx.size()));
      HIP_TRY(c, hipMemcpy(c->d_numa_idx, idx.data(), 4 * idx.size(), hipMemcpyHostToDevice));
    }
    static const bool no_slab = getenv("GS_NUMA_SLAB") && getenv("GS_NUMA_SLAB")[0] == '0';
    if (!no_slab && c->numa_n > c->slab_cap) {   // columns of numa_n entries (rounded), the mirror's numbering
      HIP_TRY(c, host_wait_stream(c->st_ev));
      if (c->slab_mv.i64) (void)hipFree(c->slab_mv.i64);
      if (c->slab_mv.i32) (void)hipFree(c->slab_mv.i32);
      c->slab_mv = MirrorView{nullptr, nullptr, 0};
      c->slab_cap = (c->numa_n + 1023) & ~1023u;
      HIP_TRY(c, hipMalloc(&c->slab_mv.i64, (size_t)NUM_I64_COLS * c->slab_cap * 8));
      HIP_TRY(c, hipMalloc(&c->slab_mv.i32, (size_t)NUM_I32_COLS * c->slab_cap * 4));
      c->slab_mv.npad = c->slab_cap;
    }
    c->numa_idx_stale = false;
    c->numa_idx_lo = c->e0;
    c->numa_idx_hi = c->e1;
  }
  const gs_ctx::Slot& sl = c->slot[c->cur_slot];
  // a short batch with no pass beside it: upload, eval and levels in order on st (no queue hops)
  const bool direct = direct_batch(c, b, prev != nullptr);
  hipStream_t se = direct ? c->st : c->st_ev;
  // A direct batch read back on st records no timing events: three HIP calls less per short plain run (C5 at 100k nodes,
  // medians of 7 alternations: 23.6k against 21.8k pods/s); its eval and levels intervals are not counted in the stats,
  // the commit's comes from the kernel. GS_DIRECT_TIMING=1: timed as the other batches.
  static const bool direct_untimed = !(getenv("GS_DIRECT_TIMING") && getenv("GS_DIRECT_TIMING")[0] == '1');
  const bool untimed = direct_untimed && direct && b < 32;
  c->slot[c->cur_slot].untimed = untimed;
  if (!untimed) HIP_TRY(c, hipEventRecord(c->ev[0], se));
  if (c->sgather) {
    // several ranks, score rows: this rank's shard into its block of the all-gather (rows of sx_pld entries), then the
    // R blocks into the full-width rows S / aff: every rank continues with the one-shard pipeline over all nodes
    const uint32_t pld = c->sx_pld;
    uint8_t* blk = c->d_sx_send + c->sx_bytes * c->cur_slot;
    uint8_t* rcv = c->d_sx_recv + c->sx_bytes * c->nranks * c->cur_slot;
    HIP_TRY(c, launch_eval(c->mv, c->d_pods, b, c->pf, c->e0, c->e1, reinterpret_cast<int16_t*>(blk), pld, prod_cols,
                           c->d_numa_idx, c->numa_n, blk + (size_t)b * pld * 2, se, c->st2, c->ev_fork, c->ev_join,
                           c->slab_mv.i64 ? &c->slab_mv : nullptr));
    if (!untimed) HIP_TRY(c, hipEventRecord(c->ev[1], se));
    const size_t bytes = ((size_t)b * pld * 3 + sizeof(XTag) + 255) / 256 * 256;
    if (int rc = exchange(c, XSITE_SCORES, blk, rcv, bytes, nullptr, se)) return rc;
    HIP_TRY(c, launch_unpack_scores(rcv, bytes, c->nranks, b, c->sx_per, pld, c->N, c->d_S, c->d_aff, c->ld,
                                    c->d_xerr + (XERR_BYTES / 4) * c->cur_slot, se));
  } else {
    HIP_TRY(c, launch_eval(c->mv, c->d_pods, b, c->pf, c->n0, c->n1, c->d_S, c->ld, prod_cols, c->d_numa_idx, c->numa_n,
                           c->d_aff, se, c->st2, c->ev_fork, c->ev_join, c->slab_mv.i64 ? &c->slab_mv : nullptr));
    if (!untimed) HIP_TRY(c, hipEventRecord(c->ev[1], se));
  }
  const bool fix = ovl && prev && prev_b > 0;
  if (ovl) {
    // levels on st_ev beside the previous batch's commit: the rows it lands on are stale here (listed with a margin of
    // prev_b nodes, histogram kept), fixed up on st below once it committed
    CandPatch cp{};
    cp.extra = fix ? prev_b : 0;
    cp.hist = fix ? c->d_hist : nullptr;
    HIP_TRY(c, launch_cand(c->d_S, c->ld, len, c->n0, b, c->max_score, c->lstride, d_lists, d_hdrs, d_ext, se, &cp,
                           c->d_cscratch));
  }
  if (!direct) {
    HIP_TRY(c, hipEventRecord(sl.ev_evdone, c->st_ev));
    HIP_TRY(c, hipStreamWaitEvent(c->st, sl.ev_evdone, 0));
  } else {   // the next speculative pass on st_ev (gather into the shared slab, eval) after this one
    HIP_TRY(c, hipEventRecord(sl.ev_evdone, c->st));
    HIP_TRY(c, hipStreamWaitEvent(c->st_ev, sl.ev_evdone, 0));
  }
  if (fix) {
    CandPatch cp{c->mv, c->d_pods, c->pf, c->n0, c->n1, prod_cols, 0, c->d_aff, prev_out, prev};
    cp.extra = prev_b;
    cp.hist = c->d_hist;
    HIP_TRY(c, launch_fix_levels(c->d_S, c->ld, b, c->max_score, c->lstride, d_lists, d_hdrs, d_ext, cp, c->st));
  }
  // the rows the previous batch landed on, re-evaluated on their committed state: inside cand_kernel (block k patches
  // pod k's row before its histogram; one launch less on the commit chain), or by patch_kernel under node sampling
  // (no candidate levels) or GS_FUSED_PATCH=0
  const bool fused = prev && prev_b > 0 && !c->window_k && !separate;
  if (!ovl && prev && !fused)
    HIP_TRY(c, launch_patch(c->mv, c->d_pods, b, c->pf, c->n0, c->n1, c->d_S, c->ld, prod_cols, c->d_aff, prev_out,
                            prev, prev_b, c->st));
  if (!c->window_k && !ovl) {   // node sampling selects over the rotation window, not the candidate levels
    CandPatch cp{c->mv, c->d_pods, c->pf, c->n0, c->n1, prod_cols, 1, c->d_aff, prev_out, prev};
    HIP_TRY(c, launch_cand(c->d_S, c->ld, len, c->n0, b, c->max_score, c->lstride, d_lists, d_hdrs, d_ext, c->st,
                           fused ? &cp : nullptr, c->d_cscratch));
  }
  // no timing markers between the levels and the commit kernel (each one held the commit's dispatch ~13 us): the
  // commit's duration comes from the kernel itself (committed[4]), the levels' interval is the rest up to ev[4]
  if (lvl_ranks(c) > 1) {
    int rc = exchange(c, XSITE_LEVELS, c->d_xchg_send, c->d_xchg_recv, c->xchg_bytes);
    if (rc) return rc;
    if (!commit_spec_selected(c->window_k)) return fail(c, GS_EUNSUPPORTED, "several ranks need the speculative commit");
    HIP_TRY(c, launch_merge_levels(c->d_xchg_recv, c->xchg_bytes, c->nranks, b, c->B, c->lstride, c->d_xmerged,
                                   c->d_xerr, c->st));
  }
  CommitArgs a = commit_args(c, b);
  a.prev = prev;
  ++c->xbatch;
  HIP_TRY(c, launch_commit(a, c->st));
  if (!untimed) HIP_TRY(c, hipEventRecord(c->ev[4], c->st));
  // full batches: readback on its own stream, so that the speculative next batch's patch / cand start right after the
  // commit (the slot's buffers are rewritten only after finish_batch has waited for ev[5]). Short batches (the host
  // waits on each one) keep it in order on st: the extra queue hop costs more than it hides there.
  hipStream_t rb = b >= 32 ? c->st_rb : c->st;
  if (rb != c->st) HIP_TRY(c, hipStreamWaitEvent(rb, c->ev[4], 0));
  // Two copies, not one over the adjacent committed words and placements: with one merged copy, 4 processes sharing the
  // GPU (the C4 rehearsal) stalled for 10-100 s at a time, every rank's commit and next eval pass pending (DESIGN §8;
  // GS_MERGE_RB=1 restores the merged copy for that experiment)
  // A direct batch reads back in two copies as well: the merged form measured within noise there and its
  // stall with several processes on one GPU is not understood (GS_DIRECT_MERGE_RB=1, experiments: one copy)
  static const bool merge_rb = getenv("GS_MERGE_RB") && getenv("GS_MERGE_RB")[0] == '1';
  static const bool merge_direct = getenv("GS_DIRECT_MERGE_RB") && getenv("GS_DIRECT_MERGE_RB")[0] == '1';
  if (merge_rb || (direct && merge_direct && rb == c->st)) {
    HIP_TRY(c, hipMemcpyAsync(c->h_committed, c->d_committed, COMMITTED_BYTES + sizeof(PlacementDev) * b,
                              hipMemcpyDeviceToHost, rb));
  } else {
    HIP_TRY(c, hipMemcpyAsync(c->h_committed, c->d_committed, COMMITTED_BYTES, hipMemcpyDeviceToHost, rb));
    HIP_TRY(c, hipMemcpyAsync(c->h_out, c->d_out, sizeof(PlacementDev) * b, hipMemcpyDeviceToHost, rb));
  }
  HIP_TRY(c, hipEventRecord(c->ev[5], rb));
  return GS_OK;
}

// Wait for the bound slot's batch; when it committed nothing, resolve its pod 0 by the exact full-row path
// (several shards). clobbered: a speculative pass has overwritten the score rows and lists since -> GS_REDO.
int finish_batch(gs_ctx* c, int b, bool clobbered, int* committed_out) {
  uint32_t len = c->n1 - c->n0;
  {
    Where w_(c, "finish_batch: the batch's readback event");
    HIP_TRY(c, host_wait_event(c->ev[5]));
  }
  flush_exchange_times(c);
  const bool untimed = c->slot[c->cur_slot].untimed;
  if (!untimed) c->stats.eval_ms += ev_ms(c->ev[0], c->ev[1]);
  {   // commit kernel: its own duration (s_memrealtime, 100 MHz) in committed[4]; levels: the rest from the eval's end
    const double cm = (double)(uint32_t)c->h_committed[4] * 1e-5;
    c->stats.commit_ms += cm;
    if (!untimed) c->stats.cand_ms += std::max(0.0, ev_ms(c->ev[1], c->ev[4]) - cm);
  }
  c->stats.eval_launches += 1;
  c->stats.eval_pairs += (uint64_t)b * (c->e1 - c->e0);
  c->stats.batches += 1;
  int committed = c->h_committed[0];
  if (committed < 0) return fail(c, GS_ESTATE, "commit pass of a batch was voided unexpectedly");
  if (c->h_committed[3] == COMMIT_ERR_XTAG) {   // the level exchange paired different exchanges of the ranks
    // the first mismatching exchange's tags, as merge_levels_kernel kept them
    std::vector<uint8_t> xe(XERR_BYTES);
    HIP_TRY(c, host_wait_stream(c->st));
    HIP_TRY(c, hipMemcpy(xe.data(), c->d_xerr + (c->sgather ? (XERR_BYTES / 4) * c->cur_slot : 0), xe.size(),
                         hipMemcpyDeviceToHost));
    const uint8_t* tags = xe.data() + 4 * XERR_TAGS;
    XTag mine;
    std::memcpy(&mine, tags + (size_t)c->rank * sizeof(XTag), sizeof mine);
    if (int rc = check_tags(c, tags, sizeof(XTag), mine)) return rc;
    return fail(c, GS_ECOMM, "exchange sequence diverged at a %s exchange (device check)",
                c->sgather ? "score-row" : "level");
  }
  if (c->h_committed[3])
    return fail(c, GS_EDEVICE, "commit kernel: a pipeline wait expired (internal error, site %d)", c->h_committed[3]);
  if (c->window_k) {
    if (committed == 0) return fail(c, GS_ESTATE, "node-sampling commit made no progress");
    c->next_start = (uint32_t)c->h_committed[2];
    c->stats.next_start_node_index = c->next_start;
  }
  if (committed == 0 && clobbered) return GS_REDO;
  if (committed == 0) {
    CommitArgs a = commit_args(c, b);
    // exact full-row path for pod 0: (max, ties, feasible) of every shard's row, global selection
    HIP_TRY(c, launch_row_stats(c->d_S, len, c->d_rowstat, c->st));
    const int lr = lvl_ranks(c);
    std::vector<RowStat> rs(lr);
    if (lr > 1) {
      int rc = exchange_small(c, XSITE_ROWSTAT, c->d_rowstat, sizeof(RowStat), rs.data());
      if (rc) return rc;
    } else {
      HIP_TRY(c, hipMemcpyAsync(rs.data(), c->d_rowstat, sizeof(RowStat), hipMemcpyDeviceToHost, c->st));
    }
    HIP_TRY(c, host_wait_stream(c->st));
    int M = -1;
    int64_t T = 0, F = 0;
    for (const auto& r : rs) {
      F += r.feasible;
      if (r.max_score > M) { M = r.max_score; T = r.ties; }
      else if (r.max_score == M && M >= 0) T += r.ties;
    }
    if (M < 0) {
      c->h_out[0] = PlacementDev{-1, (uint32_t)F, 0, 0, GS_PLACED_SLOWPATH, 0, 0, {0, 0, 0, 0}, {0, 0, 0, 0}};
      *committed_out = 1;
      return GS_OK;
    }
    int64_t jstar = host_tiebreak_position(c->cfg.seed, c->h_seq[0], T);
    int owner = -1;
    int64_t before = 0;
    for (int r = 0; r < lr; ++r) {
      if (rs[r].max_score != M) continue;
      if (jstar <= before + rs[r].ties) { owner = r; break; }
      before += rs[r].ties;
    }
    int32_t winner = -1;
    if (owner == (lr > 1 ? c->rank : 0)) {
      HIP_TRY(c, launch_row_select(c->d_S, len, M, jstar - before, c->n0, c->d_sel, c->st));
    } else {
      HIP_TRY(c, hipMemsetAsync(c->d_sel, 0xff, 4, c->st));
    }
    if (lr > 1) {
      std::vector<int32_t> w(lr);
      int rc = exchange_small(c, XSITE_SELECT, c->d_sel, 4, w.data());
      if (rc) return rc;
      winner = w[owner];
    } else {
      HIP_TRY(c, hipMemcpyAsync(&winner, c->d_sel, 4, hipMemcpyDeviceToHost, c->st));
      HIP_TRY(c, host_wait_stream(c->st));
    }
    if (winner < 0) return fail(c, GS_ESTATE, "exact path could not locate tie %lld", (long long)jstar);
    a.forced_node = winner;
    a.forced_score = M;
    a.forced_ties = T;
    a.forced_feasible = (int32_t)F;
    HIP_TRY(c, hipEventRecord(c->ev[3], c->st));
    HIP_TRY(c, launch_commit(a, c->st));
    HIP_TRY(c, hipEventRecord(c->ev[4], c->st));
    HIP_TRY(c, hipMemcpyAsync(c->h_committed, c->d_committed, COMMITTED_BYTES, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(c, host_wait_stream(c->st));
    c->stats.commit_ms += ev_ms(c->ev[3], c->ev[4]);
    committed = c->h_committed[0];
    if (committed < 1) return fail(c, GS_ESTATE, "forced commit made no progress");
    HIP_TRY(c, hipMemcpyAsync(c->h_out, c->d_out, sizeof(PlacementDev) * committed, hipMemcpyDeviceToHost, c->st));
    HIP_TRY(c, host_wait_stream(c->st));
  }
  flush_exchange_times(c);
  if (committed < b) {
    c->stats.cuts += 1;
    static const bool dbg = getenv("GS_DEBUG_CUTS") && getenv("GS_DEBUG_CUTS")[0] == '1';
    if (dbg) {
      const PlacementDev& x = c->h_out[committed];
      fprintf(stderr, "gpuscore: batch of %d ended after %d pods (code %#x) [%d run %u M %lld Mc %lld Md %lld T %u Tc %d new %u old %u jp %lld nd %lld pend %lld]\n",
              b, committed, c->h_committed[2], x.node, x.feasible, (long long)(x.score & 0xfffff),
              (long long)((x.score >> 20) & 0xfffff), (long long)(x.score >> 40), x.ties, (int)x.flags, x.zkeys, x.pad,
              (long long)x.zcpu[0], (long long)x.zcpu[1], (long long)x.zcpu[2]);
      fprintf(stderr, "   old slot %lld node %llu hash %lld S %d dso %d\n", (long long)x.cpuset[0],
              (unsigned long long)x.cpuset[1], (long long)x.cpuset[2], (int)(x.cpuset[3] >> 32), (int)(int32_t)x.cpuset[3]);
    }
  }
  *committed_out = committed;
  return GS_OK;
}

// ---- Reservation + DeviceShare: one extension pod (gs_ext.hip) ------------------------------------------------

// GetPodDeviceRequests for the GPU type (deviceshare/utils.go:147-252): ValidateDeviceRequest + ConvertDeviceRequest.
// 0: ok (mask 0 = no GPU request), -1: invalid (PreFilter UnschedulableAndUnresolvable)
int gpu_request_of(const gs_pod_ext& e, int64_t req[3], uint32_t* mask) {
  req[0] = req[1] = req[2] = 0;
  *mask = 0;
  const uint32_t m = e.gpu_request_mask & 0x1Fu;
  if (!m) return 0;
  for (int n : {GS_GPU_NAME_KOORD_GPU, GS_GPU_NAME_CORE, GS_GPU_NAME_MEMORY_RATIO})   // ValidatePercentageResource
    if ((m >> n & 1u) && e.gpu_requests[n] > 100 && e.gpu_requests[n] % 100 != 0) return -1;
  const int64_t* q = e.gpu_requests;
  switch (m) {   // ValidDeviceResourceCombinations -> ResourceCombinationsMapper
    case 1u << GS_GPU_NAME_NVIDIA: req[0] = req[1] = q[GS_GPU_NAME_NVIDIA] * 100; *mask = 3; return 0;
    case 1u << GS_GPU_NAME_KOORD_GPU: req[0] = req[1] = q[GS_GPU_NAME_KOORD_GPU]; *mask = 3; return 0;
    case 1u << GS_GPU_NAME_MEMORY: req[2] = q[GS_GPU_NAME_MEMORY]; *mask = 4; return 0;
    case 1u << GS_GPU_NAME_MEMORY_RATIO: req[1] = q[GS_GPU_NAME_MEMORY_RATIO]; *mask = 2; return 0;
    case (1u << GS_GPU_NAME_CORE) | (1u << GS_GPU_NAME_MEMORY):
      req[0] = q[GS_GPU_NAME_CORE]; req[2] = q[GS_GPU_NAME_MEMORY]; *mask = 5; return 0;
    case (1u << GS_GPU_NAME_CORE) | (1u << GS_GPU_NAME_MEMORY_RATIO):
      req[0] = q[GS_GPU_NAME_CORE]; req[1] = q[GS_GPU_NAME_MEMORY_RATIO]; *mask = 3; return 0;
    default: return -1;
  }
}

// The HBM image of node i's Device object; a GPU's Topology.NodeID becomes a slot of the node's NUMA zones (the zone
// masks the topology manager merges), GZ_FOREIGN when it is none of them.
DevNode dev_image(const gs_ctx* c, uint32_t i) {
  const gs_node_devices& d = c->devs[i];
  const gs_node_numa* nn = c->numa_on ? &c->numa[i].cfg : nullptr;
  DevNode o{};
  o.has_device = d.has_device;
  o.num_gpus = d.has_device ? d.num_gpus : 0;
  for (int n = 0; n < GS_NUM_GPU_NAMES; ++n) o.fit_free[n] = d.allocatable[n] - d.requested[n];
  for (int x = 0; x < GS_MAX_XRES; ++x) o.fit_free[GS_NUM_GPU_NAMES + x] = d.xres_allocatable[x] - d.xres_requested[x];
  for (int g = 0; g < o.num_gpus; ++g) {
    o.g[g].minor = d.gpus[g].minor;
    o.g[g].has_info = d.gpus[g].has_info ? 1 : 0;
    o.g[g].zone = GZ_NONE;
    if (d.gpus[g].numa_node >= 0) {
      o.g[g].zone = GZ_FOREIGN;
      for (int z = 0; nn && z < nn->num_zones; ++z)
        if (nn->zones[z].node_id == d.gpus[g].numa_node) o.g[g].zone = (int16_t)z;
    }
    for (int r = 0; r < 3; ++r) {
      o.g[g].total[r] = d.gpus[g].total[r];
      o.g[g].free[r] = std::max<int64_t>(0, d.gpus[g].total[r] - d.gpus[g].used[r]);
    }
  }
  return o;
}

int ext_alloc(gs_ctx* c) {
  if (c->d_dev) return GS_OK;
  HIP_TRY(c, hipMalloc(&c->d_dev, sizeof(DevNode) * std::max<uint32_t>(1, c->N)));
  std::vector<DevNode> img(c->N);
  for (uint32_t i = 0; i < c->N; ++i) img[i] = dev_image(c, i);
  HIP_TRY(c, hipMemcpy(c->d_dev, img.data(), sizeof(DevNode) * c->N, hipMemcpyHostToDevice));
  c->dev_dirty_list.clear();
  std::fill(c->dev_dirty.begin(), c->dev_dirty.end(), 0);
  HIP_TRY(c, hipMalloc(&c->d_xtot, 4 * (size_t)c->ld));
  HIP_TRY(c, hipMalloc(&c->d_xT, 4 * ext_select_scratch_words(c->ld)));
  HIP_TRY(c, hipMalloc(&c->d_xds, 2 * (size_t)c->ld));
  HIP_TRY(c, hipMalloc(&c->d_xrs, 2 * (size_t)c->ld));
  HIP_TRY(c, hipMalloc(&c->d_xout, sizeof(ExtOut)));
  HIP_TRY(c, hipHostMalloc(&c->h_xout, sizeof(ExtOut), hipHostMallocDefault));   // written by ext_finish_kernel
  return GS_OK;
}

// The extension pod's input block (pinned host + device, one H2D copy per pod) and the nomination arrays, for at
// least nrec matched records and nres matched reservations.
int ext_stage_reserve(gs_ctx* c, uint32_t nrec, uint32_t nres) {
  if (c->h_xin && nrec <= c->xrec_cap && nres <= c->xres_cap) return GS_OK;
  c->xrec_cap = std::max<uint32_t>({64, c->xrec_cap, nrec * 2});
  c->xres_cap = std::max<uint32_t>({64, c->xres_cap, nres * 2});
  auto al = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t off_pv = al(sizeof(ExtPod));
  c->xin_off_rec = off_pv + al(sizeof(PodVec));
  c->xin_off_res = c->xin_off_rec + al(sizeof(ExtRec) * c->xrec_cap);
  c->xin_bytes = c->xin_off_res + sizeof(ExtRes) * c->xres_cap;
  HIP_TRY(c, host_wait_stream(c->st));
  if (c->h_xin) (void)hipHostFree(c->h_xin);
  if (c->d_xin) (void)hipFree(c->d_xin);
  if (c->d_xnom) (void)hipFree(c->d_xnom);
  if (c->h_xnom) (void)hipHostFree(c->h_xnom);
  HIP_TRY(c, hipHostMalloc(&c->h_xin, c->xin_bytes, hipHostMallocDefault));
  HIP_TRY(c, hipMalloc(&c->d_xin, c->xin_bytes));
  HIP_TRY(c, hipMalloc(&c->d_xnom, 4 * c->xrec_cap));
  HIP_TRY(c, hipHostMalloc(&c->h_xnom, 4 * c->xrec_cap, hipHostMallocDefault));   // written by ext_finish_kernel
  c->h_xpod = reinterpret_cast<ExtPod*>(c->h_xin);
  c->d_xpod = reinterpret_cast<ExtPod*>(c->d_xin);
  c->d_xpv = reinterpret_cast<PodVec*>(c->d_xin + off_pv);
  c->d_xrec = reinterpret_cast<ExtRec*>(c->d_xin + c->xin_off_rec);
  c->d_xres = reinterpret_cast<ExtRes*>(c->d_xin + c->xin_off_res);
  return GS_OK;
}

// the dirty nodes' Device images: staged in pinned memory, one copy and one scatter per EXT_DEV_STAGE nodes
int ext_flush_devices(gs_ctx* c) {
  if (c->dev_dirty_list.empty()) return GS_OK;
  if (!c->d_dev) return ext_alloc(c);
  if (!c->h_dev_stage) {   // n images, then their node indices: one copy
    HIP_TRY(c, hipHostMalloc(&c->h_dev_stage, (sizeof(DevNode) + 4) * EXT_DEV_STAGE, hipHostMallocDefault));
    HIP_TRY(c, hipMalloc(&c->d_dev_stage, (sizeof(DevNode) + 4) * EXT_DEV_STAGE));
  }
  for (size_t done = 0; done < c->dev_dirty_list.size();) {
    const uint32_t n = (uint32_t)std::min<size_t>(EXT_DEV_STAGE, c->dev_dirty_list.size() - done);
    HIP_TRY(c, host_wait_stream(c->st));   // the previous scatter has consumed the staging buffers
    uint32_t* h_idx = reinterpret_cast<uint32_t*>(c->h_dev_stage + n);
    for (uint32_t j = 0; j < n; ++j) {
      const uint32_t i = c->dev_dirty_list[done + j];
      c->h_dev_stage[j] = dev_image(c, i);
      h_idx[j] = i;
      c->dev_dirty[i] = 0;
    }
    HIP_TRY(c, hipMemcpyAsync(c->d_dev_stage, c->h_dev_stage, (sizeof(DevNode) + 4) * n, hipMemcpyHostToDevice, c->st));
    HIP_TRY(c, launch_scatter_devnodes(c->d_dev, reinterpret_cast<const uint32_t*>(c->d_dev_stage + n), c->d_dev_stage,
                                       n, c->st));
    done += n;
  }
  c->dev_dirty_list.clear();
  return GS_OK;
}

void dev_mark(gs_ctx* c, uint32_t i) {
  if (!c->dev_dirty[i]) { c->dev_dirty[i] = 1; c->dev_dirty_list.push_back(i); }
}

// the pod's matched reservations grouped by node (node order, uid order within a node)
void matched_of(const gs_ctx* c, uint64_t owner, std::vector<std::pair<uint32_t, uint64_t>>* out) {
  out->clear();
  if (!owner || !(c->ext.enabled & GS_EXT_RESERVATION)) return;
  auto it = c->rsv_owner.find(owner);
  if (it == c->rsv_owner.end()) return;
  for (uint64_t uid : it->second) {
    const gs_reservation& r = c->rsv.at(uid);
    if (rsv_matches(r, owner)) out->push_back({r.node, uid});
  }
  std::sort(out->begin(), out->end());
}

bool is_ext_pod(const gs_ctx* c, const gs_pod_ext& e) {
  if (e.xres_request_mask & ((1u << GS_MAX_XRES) - 1u)) return true;   // Fit over a registered extended resource
  if ((c->ext.enabled & GS_EXT_DEVICESHARE) && (e.gpu_request_mask & 0x1Fu)) return true;
  if (!(c->ext.enabled & GS_EXT_RESERVATION)) return false;
  if (e.reservation_required) return true;
  std::vector<std::pair<uint32_t, uint64_t>> m;
  matched_of(c, e.reservation_owner, &m);
  return !m.empty();
}

// DeviceShare Reserve (deviceshare/plugin.go:377-430) on the host mirror: defaultAllocateDevices with the scorer
// (device_allocator.go:397-467; minors by device score descending, then minor), within the node's NUMA affinity
// (aff: 0x10 | zone-slot mask, 0 = none; device_allocator.go:148-152)
int ext_device_reserve(gs_ctx* c, uint32_t node, const int64_t preq[3], uint32_t pmask, gs_ext_placement* eo,
                       uint32_t aff) {
  gs_node_devices& d = c->devs[node];
  if (!d.has_device) return GS_OK;
  const DevNode img = dev_image(c, node);
  int64_t total_mem = -1;
  for (int g = 0; g < img.num_gpus; ++g)
    if (img.g[g].total[0] | img.g[g].total[1] | img.g[g].total[2]) { total_mem = img.g[g].total[2]; break; }
  if (img.num_gpus <= 0 || total_mem < 0) return fail(c, GS_ESTATE, "DeviceShare Reserve: no GPU on node %u", node);
  int64_t core = preq[0], ratio = preq[1], mem = preq[2];
  if (pmask & 4u) ratio = (int64_t)((double)mem / (double)total_mem * 100.0);
  else mem = ratio * total_mem / 100;
  uint32_t m = pmask | 6u;
  int64_t count = 1;
  if (ratio > 100 && ratio % 100 == 0) { count = ratio / 100; core /= count; mem /= count; ratio /= count; m = 7u; }
  const int64_t inst[3] = {core, ratio, mem};
  struct Cand { int g; int64_t score; };
  std::vector<Cand> cs;
  for (int g = 0; g < img.num_gpus; ++g) {
    if (!img.g[g].has_info) continue;
    if ((aff & 0x10u) && (img.g[g].zone < 0 || !(aff >> img.g[g].zone & 1u))) continue;
    int64_t ns = 0, ws = 0;   // scoreDevice (deviceshare/scoring.go:186-211)
    for (int r = 0; r < 3; ++r) {
      const int64_t w = c->ext.device_weights[r], t = img.g[g].total[r], f = img.g[g].free[r];
      if (!w || t == 0) continue;
      int64_t rq = t;
      if (t >= f) rq = t - f + ((m >> r & 1u) ? inst[r] : 0);
      int64_t sc;
      if (c->ext.device_scoring_type == GS_SCORING_MOST_ALLOCATED) sc = (std::min(rq, t) * 100) / t;
      else sc = rq > t ? 0 : ((t - rq) * 100) / t;
      ns += sc * w;
      ws += w;
    }
    cs.push_back({g, ws ? ns / ws : 0});
  }
  std::stable_sort(cs.begin(), cs.end(), [&](const Cand& a, const Cand& b) {
    if (a.score != b.score) return a.score > b.score;
    return img.g[a.g].minor < img.g[b.g].minor;
  });
  std::vector<int> take;
  for (const Cand& x : cs) {
    const DevGpu& g = img.g[x.g];
    if (!(g.free[0] | g.free[1] | g.free[2])) continue;
    bool ok = true;
    for (int r = 0; r < 3; ++r) ok &= !(m >> r & 1u) || inst[r] <= g.free[r];
    if (!ok) continue;
    take.push_back(x.g);
    if ((int64_t)take.size() == count) break;
  }
  if ((int64_t)take.size() < count)
    return fail(c, GS_ESTATE, "DeviceShare Reserve: allocation failed on node %u after a feasible Filter", node);
  for (int g : take) {
    for (int r = 0; r < 3; ++r)
      if (m >> r & 1u) d.gpus[g].used[r] += inst[r];
    eo->gpu_minor_mask |= 1u << (d.gpus[g].minor & 31);
  }
  eo->gpu_count = (int32_t)count;
  for (int r = 0; r < 3; ++r) eo->gpu_per_instance[r] = (m >> r & 1u) ? inst[r] : 0;
  dev_mark(c, node);
  return GS_OK;
}

// scheduleOne of one extension pod: eval pass (B = 1) -> ext_nodes -> ext_matched -> ext_select, then the Reserve
// of NodeNUMAResource (no-op on the supported nodes), DeviceShare and Reservation, and assume.
int ext_schedule_one(gs_ctx* c, const gs_pod& pod, const gs_pod_ext& e, uint64_t seq, gs_placement* out,
                     gs_ext_placement* eo) {
  *out = gs_placement{-1, 0, 0, 0, 0};
  *eo = gs_ext_placement{};
  // several ranks: with the score-row exchange every rank holds every node's state and runs the one-GPU pipeline, so an
  // extension pod runs whole on every rank (no exchange: the same inputs give the same placement everywhere); the
  // level exchange's ranks hold their shard's rows only
  if ((c->nranks > 1 && !c->sgather) || c->window_k)
    return fail(c, GS_EUNSUPPORTED, "Reservation / DeviceShare pods need one rank (or the score-row exchange) and no "
                "node sampling");
  const bool ds_on = c->ext.enabled & GS_EXT_DEVICESHARE, rs_on = c->ext.enabled & GS_EXT_RESERVATION;
  int64_t greq[3];
  uint32_t gmask = 0;
  if (ds_on && gpu_request_of(e, greq, &gmask) < 0) {   // DeviceShare PreFilter: UnschedulableAndUnresolvable
    eo->fail_code = GS_EXT_FAIL_POD;
    c->stats.pods += 1;
    return GS_OK;
  }
  if (!ds_on) { greq[0] = greq[1] = greq[2] = 0; gmask = 0; }
  std::vector<std::pair<uint32_t, uint64_t>> matched;
  if (rs_on) matched_of(c, e.reservation_owner, &matched);
  for (int x = 0; x < GS_MAX_XRES; ++x)
    if (e.xres_requests[x] < 0 || !in_range(e.xres_requests[x]))
      return fail(c, GS_EUNSUPPORTED, "extended resource request outside [0, 2^53)");
  PodVec v = prep_pod(c, pod);
  if (rs_on && e.reservation_required && matched.empty()) {   // PreFilter: ErrReasonReservationAffinity
    c->stats.pods += 1;
    return GS_OK;
  }
  int rc;
  using hx_clk = std::chrono::steady_clock;
  const auto hx0 = hx_clk::now();
  if ((rc = ext_alloc(c))) return rc;
  if ((rc = ext_flush_devices(c))) return rc;
  if ((rc = flush_rows(c))) return rc;
  if (c->prep_stale && (rc = node_prep(c))) return rc;
  const auto hx1 = hx_clk::now();
  // ---- BeforePreFilter: per-node restore records (reservation/transformer.go:50-235)
  c->xrec.clear();
  c->xres.clear();
  c->xres_uid.clear();
  for (size_t a = 0; a < matched.size();) {
    const uint32_t node = matched[a].first;
    size_t b = a;
    while (b < matched.size() && matched[b].first == node) ++b;
    if (b - a > (size_t)EXT_MAX_RES_PER_NODE)
      return fail(c, GS_EUNSUPPORTED, "more than %d matched reservations on node %u", EXT_MAX_RES_PER_NODE, node);
    ExtRec rec{};
    rec.node = node;
    rec.nres = (int32_t)(b - a);
    rec.first = (int32_t)c->xres.size();
    rec.dpods = rec.nres;
    rec.order_min = INT64_MAX;
    const gs_node mirror = reservation_view(c, node, 0);
    const gs_node podreq = reservation_view(c, node, e.reservation_owner);
    for (int s = 0; s < 7; ++s) {
      rec.pod_requested[s] = podreq.requested[s];
      rec.allocatable[s] = podreq.allocatable[s];
    }
    gs_node restored = podreq;
    for (size_t k = a; k < b; ++k) {
      const gs_reservation& r = c->rsv.at(matched[k].second);
      if (c->numa_on && (v.numa & PN_BIND)) {
        // NodeNUMAResource's reservation restore (nodenumaresource/reservation.go:76-113, plugin.go:488-549) hands a
        // cpuset pod the reservation's remaining CPUs (preferredCPUs, reusableResources): not restated. It applies only
        // when the reservation itself holds a cpuset allocation; without one the restore is empty
        auto it = c->numa[node].pods.find(r.uid);
        if (it != c->numa[node].pods.end() && !it->second.cpus.empty())
          return fail(c, GS_EUNSUPPORTED, "a cpuset pod matching reservation %llu, which holds a cpuset on node %u, is "
                      "not on the device path", (unsigned long long)r.uid, node);
      }
      rsv_request_delta(r.allocatable, r.allocatable_mask, -1, restored.requested, restored.nonzero_requested);
      ExtRes x{};
      int64_t rem[GS_NUM_RES];
      (void)rsv_remained(r, rem);
      for (int s = 0; s < 7; ++s) {
        x.alloc[s] = (r.allocatable_mask >> s & 1u) ? r.allocatable[s] : 0;
        x.allocated[s] = (r.allocated_mask >> s & 1u) ? r.allocated[s] : 0;
        rec.r_allocated[s] += x.allocated[s];
        // SubtractWithNonNegativeResult(Allocatable, Mask(Allocated, ResourceNames)) (Restricted policy)
        const int64_t am = (r.resource_names_mask >> s & 1u) ? x.allocated[s] : 0;
        x.remained_nn[s] = std::max<int64_t>(0, x.alloc[s] - am);
      }
      x.order = r.order;
      x.alloc_mask = r.allocatable_mask;
      x.allocated_mask = r.allocated_mask;
      x.names = r.resource_names_mask;
      x.policy = r.allocate_policy;
      x.skip = (r.allocate_once && r.assigned_pods > 0) ? 1 : 0;
      if (r.order != 0 && rec.order_min > r.order) rec.order_min = r.order;
      c->xres.push_back(x);
      c->xres_uid.push_back(r.uid);
    }
    for (int s = 0; s < 7; ++s) rec.dfree[s] = mirror.requested[s] - restored.requested[s];
    rec.dnz[0] = mirror.nonzero_requested[0] - restored.nonzero_requested[0];
    rec.dnz[1] = mirror.nonzero_requested[1] - restored.nonzero_requested[1];
    rec.restored_pods = podreq.pod_count - rec.nres;
    rec.allowed_pods = podreq.allowed_pod_number;
    c->xrec.push_back(rec);
    a = b;
  }
  const int nrec = (int)c->xrec.size();
  if ((rc = ext_stage_reserve(c, (uint32_t)nrec, (uint32_t)c->xres.size()))) return rc;
  ExtPod& xp = *c->h_xpod;
  xp = ExtPod{};
  for (int r = 0; r < 3; ++r) { xp.gpu_req[r] = greq[r]; xp.dev_w[r] = c->ext.device_weights[r]; }
  xp.gpu_mask = gmask;
  const uint32_t gpu_names_all = gmask ? (e.gpu_request_mask & 0x1Fu) : 0u;   // NodeInfo.AddPod adds them all
  xp.gpu_names = gpu_names_all & ~c->ext.fit_ignored_gpu_names;               // Fit checks the non-ignored ones
  for (int n = 0; n < GS_NUM_GPU_NAMES; ++n) xp.gpu_name_req[n] = (xp.gpu_names >> n & 1u) ? e.gpu_requests[n] : 0;
  const uint32_t xres_all = e.xres_request_mask & ((1u << GS_MAX_XRES) - 1u);
  const uint32_t xres_fit = xres_all & ~c->ext.fit_ignored_xres;
  xp.gpu_names |= xres_fit << GS_NUM_GPU_NAMES;
  for (int x = 0; x < GS_MAX_XRES; ++x)
    xp.gpu_name_req[GS_NUM_GPU_NAMES + x] = (xres_fit >> x & 1u) ? e.xres_requests[x] : 0;
  xp.w_ds = c->ext.weight_deviceshare;
  xp.w_rs = c->ext.weight_reservation;
  for (int s = 0; s < 7; ++s) xp.pod_req[s] = pod.requests[s];
  xp.pod_mask = pod.request_mask & 0x7Fu;
  xp.required = rs_on && e.reservation_required;
  xp.nrec = nrec;
  xp.ds_on = ds_on;
  xp.rs_on = rs_on;
  xp.dev_most = c->ext.device_scoring_type == GS_SCORING_MOST_ALLOCATED;
  xp.seq = seq;
  // GPU names are scalar requests: the Fit filter's all-zero short cut no longer applies
  if (gpu_names_all || xres_all) v.flags &= ~PF_ALL_ZERO;
  *reinterpret_cast<PodVec*>(c->h_xin + ((sizeof(ExtPod) + 15) & ~(size_t)15)) = v;
  // the NUMA-policy work list over [n0, n1) for the eval pass and ext_numa_kernel (launch_batch's list is the shard's)
  if (c->numa_on && c->xnuma_stale) {
    std::vector<uint32_t> idx;
    for (uint32_t n = c->n0; n < c->n1; ++n)
      if (c->numa[n].cfg.numa_topology_policy != GS_NUMA_POLICY_NONE) idx.push_back(n);
    HIP_TRY(c, host_wait_stream(c->st));
    if (c->d_xnuma_idx) { (void)hipFree(c->d_xnuma_idx); c->d_xnuma_idx = nullptr; }
    c->xnuma_n = (uint32_t)idx.size();
    if (c->xnuma_n) {
      HIP_TRY(c, hipMalloc(&c->d_xnuma_idx, 4 * idx.size()));
      HIP_TRY(c, hipMemcpy(c->d_xnuma_idx, idx.data(), 4 * idx.size(), hipMemcpyHostToDevice));
    }
    c->xnuma_stale = false;
  }
  const int prod_cols = (v.flags & PF_PROD_SCORE) ? 1 : 0;
  // inputs: one copy of the staged block (ExtPod, PodVec, the matched records and reservations)
  if (nrec) {
    std::memcpy(c->h_xin + c->xin_off_rec, c->xrec.data(), sizeof(ExtRec) * nrec);
    std::memcpy(c->h_xin + c->xin_off_res, c->xres.data(), sizeof(ExtRes) * c->xres.size());
  }
  const size_t in_bytes = nrec ? c->xin_off_res + sizeof(ExtRes) * c->xres.size() : c->xin_off_rec;
  // no event markers inside the chain (each one holds the next dispatch for microseconds): the pass is timed on the
  // host, from the input copy's enqueue to the end of the stream synchronisation (GS_EXT_EVENTS=1: per-kernel events)
  static const bool ext_ev = getenv("GS_EXT_EVENTS") && getenv("GS_EXT_EVENTS")[0] == '1';
  const auto ext_t0 = std::chrono::steady_clock::now();
  HIP_TRY(c, hipMemcpyAsync(c->d_xin, c->h_xin, in_bytes, hipMemcpyHostToDevice, c->st));
  if (ext_ev) HIP_TRY(c, hipEventRecord(c->ev[0], c->st));
  HIP_TRY(c, launch_eval(c->mv, c->d_xpv, 1, c->pf, c->n0, c->n1, c->d_S, c->ld, prod_cols, c->d_xnuma_idx, c->xnuma_n,
                         c->d_aff, c->st));
  if (ext_ev) HIP_TRY(c, hipEventRecord(c->ev[1], c->st));
  // (ext_nodes_kernel also resets the select accumulators; ext_matched runs for pods with matched reservations only)
  HIP_TRY(c, launch_ext_nodes(c->d_dev, c->d_S, c->n0, c->n1, c->d_xpod, c->d_xtot, c->d_xds, c->d_xrs, c->d_xT,
                              c->st));
  // GPU pods on NUMA-policy nodes: DeviceShare is the topology manager's second hint provider
  if (gmask && c->numa_on && c->xnuma_n)
    HIP_TRY(c, launch_ext_numa(c->mv, c->d_xpv, c->pf, prod_cols, c->d_dev, c->d_xpod, c->d_xnuma_idx, c->xnuma_n, c->n0,
                               c->d_xtot, c->d_xds, c->d_aff, c->d_xT, c->n1 - c->n0, c->st));
  // the matched nodes last: their restored rows over the whole Filter chain (incl. the policy nodes' affinity)
  if (nrec)
    HIP_TRY(c, launch_ext_matched(c->mv, c->d_xpv, c->pf, prod_cols, c->d_dev, c->d_xpod, c->d_xrec, c->d_xres, nrec,
                                  c->d_xtot, c->d_xds, c->d_xrs, c->d_xnom, c->d_aff, c->n0, c->d_xT, c->n1 - c->n0,
                                  c->st));
  HIP_TRY(c, launch_ext_select(c->d_xtot, c->d_xds, c->d_xrs, c->d_xrec, c->n0, c->n1, c->d_xpod, c->cfg.seed, c->d_xT,
                               c->d_xout, c->st));
  // outputs: the NodeNUMAResource Reserve of the selected node along its affinity, and the result and nominations
  // written straight into pinned host memory (no copy)
  HIP_TRY(c, launch_ext_finish(c->mv, c->d_xpv, c->pf, prod_cols, c->d_aff, c->n0, c->numa_on ? 1 : 0, c->d_xout,
                               c->d_xnom, nrec, c->h_xout, c->h_xnom, c->st));
  if (ext_ev) HIP_TRY(c, hipEventRecord(c->ev[4], c->st));
  HIP_TRY(c, host_wait_stream(c->st));
  const auto hx3 = hx_clk::now();
  if (c->host_timing) {
    const auto us = [](hx_clk::duration d) { return std::chrono::duration<double, std::micro>(d).count(); };
    c->hx_flush += us(hx1 - hx0);
    c->hx_prep += us(ext_t0 - hx1);
    c->hx_gpu += us(hx3 - ext_t0);
    c->hx_pods += 1;
  }
  if (ext_ev) {
    c->stats.eval_ms += ev_ms(c->ev[0], c->ev[1]);
    c->stats.commit_ms += ev_ms(c->ev[1], c->ev[4]);
  } else {
    c->stats.commit_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ext_t0).count();
  }
  c->stats.eval_launches += 1;
  c->stats.eval_pairs += c->n1 - c->n0;
  c->stats.batches += 1;
  c->stats.pods += 1;
  const ExtOut xo = *c->h_xout;
  if (xo.err & 1u)
    return fail(c, GS_EUNSUPPORTED, "a GPU's NUMA node is not one of its node's NUMA zones (DeviceShare hints)");
  if (xo.err & 2u)
    return fail(c, GS_EUNSUPPORTED, "the topology-manager merge of a GPU pod exceeds its permutation bound");
  out->feasible = xo.feasible;
  if (xo.node < 0) return GS_OK;
  out->node = xo.node;
  out->score = xo.score;
  out->ties = xo.ties;
  eo->deviceshare_score = xo.ds_norm;
  eo->reservation_score = xo.rs_norm;
  const uint32_t node = (uint32_t)xo.node;
  // ---- Reserve: NodeNUMAResource (the zones the device allocated along the affinity), DeviceShare, Reservation
  if (c->numa_on) {
    PlacementDev pd{};
    pd.node = xo.node;
    pd.flags = xo.nflags;
    pd.zkeys = xo.zkeys;
    for (int z = 0; z < 4; ++z) { pd.zcpu[z] = xo.zcpu[z]; pd.zmem[z] = xo.zmem[z]; }
    if ((rc = numa_reserve(c, pod, v, pd))) return rc;
    out->flags = xo.nflags & ~PL_INTERNAL_FLAGS;
  }
  if (gmask && (rc = ext_device_reserve(c, node, greq, gmask, eo, xo.aff))) {
    // the reference runs every plugin's Unreserve on a Reserve failure: NodeNUMAResource's allocation goes again
    if (c->numa_on && c->numa_uid_node.count(pod.uid)) {
      numa_release(c->numa[node], pod.uid);
      c->numa_uid_node.erase(pod.uid);
      mark_dirty(c, node);
    }
    return rc;
  }
  int rec_i = -1;   // the chosen node's matched record (records are in node order)
  {
    auto it = std::lower_bound(c->xrec.begin(), c->xrec.end(), node,
                               [](const ExtRec& r, uint32_t n) { return r.node < n; });
    if (it != c->xrec.end() && it->node == node) rec_i = (int)(it - c->xrec.begin());
  }
  if (rs_on && rec_i >= 0) {   // Reservation.Reserve -> reservationCache.assumePod (AddAssignedPod, reservation_info.go:379-388)
    const int nom = c->h_xnom[rec_i];
    if (nom >= 0) {
      gs_reservation& r = c->rsv.at(c->xres_uid[c->xrec[rec_i].first + nom]);
      for (int s = 0; s < 7; ++s)
        if ((r.resource_names_mask >> s & 1u) && (pod.request_mask >> s & 1u)) {
          r.allocated[s] = ((r.allocated_mask >> s & 1u) ? r.allocated[s] : 0) + pod.requests[s];
          r.allocated_mask |= 1u << s;
        }
      r.assigned_pods += 1;
      eo->reservation_uid = r.uid;
    }
  }
  for (int n = 0; n < GS_NUM_GPU_NAMES; ++n)   // NodeInfo.AddPod of the GPU-name scalars
    if (gpu_names_all >> n & 1u) { c->devs[node].requested[n] += e.gpu_requests[n]; dev_mark(c, node); }
  for (int x = 0; x < GS_MAX_XRES; ++x)         // ... and of the registered extended resources
    if (xres_all >> x & 1u) { c->devs[node].xres_requested[x] += e.xres_requests[x]; dev_mark(c, node); }
  if (gmask || (rs_on && rec_i >= 0 && c->h_xnom[rec_i] >= 0) || gpu_names_all || xres_all)
    c->ext_reserved.insert(pod.uid);   // gs_pods_forget cannot undo these Reserves
  apply_placement(c, pod, xo.node, true);
  if (c->host_timing)
    c->hx_reserve += std::chrono::duration<double, std::micro>(hx_clk::now() - hx3).count();
  return GS_OK;
}

}  // namespace

// ================================================================================================
extern "C" {

uint32_t gs_num_feasible_nodes_to_find(uint32_t num_all_nodes, int32_t pct) {
  // [upstream] schedule_one.go numFeasibleNodesToFind: minFeasibleNodesToFind = 100,
  // minFeasibleNodesPercentageToFind = 5, adaptive 50 - N/125 % (int32 arithmetic)
  const int32_t n = (int32_t)num_all_nodes;
  if (n < 100 || pct >= 100) return num_all_nodes;
  int32_t p = pct > 0 ? pct : std::max<int32_t>(5, 50 - n / 125);
  const int32_t k = n * p / 100;
  return k < 100 ? 100u : (uint32_t)k;
}

const char* gs_version(void) { return "libgpuscore 0.1 (gfx950, ABI 1)"; }

void gs_abi_sizes(uint64_t* out, uint32_t n) {
  const uint64_t s[] = {sizeof(gs_pod), sizeof(gs_node), sizeof(gs_node_metric), sizeof(gs_pod_metric),
                        sizeof(gs_config), sizeof(gs_placement), sizeof(gs_stats), sizeof(gs_loadaware_args),
                        sizeof(gs_cpu_topology), sizeof(gs_node_numa), sizeof(gs_pod_allocation), sizeof(gs_numa_args),
                        sizeof(gs_quota_group), sizeof(gs_quota_status), sizeof(gs_node_devices),
                        sizeof(gs_reservation), sizeof(gs_pod_ext), sizeof(gs_ext_args), sizeof(gs_ext_placement)};
  for (uint32_t i = 0; i < n && i < sizeof(s) / sizeof(s[0]); ++i) out[i] = s[i];
}

void gs_loadaware_args_default(gs_loadaware_args* a) {
  if (!a) return;
  std::memset(a, 0, sizeof(*a));
  a->filter_expired_node_metrics = 1;
  a->has_node_metric_expiration = 1;
  a->node_metric_expiration_seconds = 180;
  a->resource_weights[0] = a->resource_weights[1] = 1;
  a->resource_weights_mask = GS_USAGE_CPU | GS_USAGE_MEMORY;
  a->usage_thresholds[0] = 65;
  a->usage_thresholds[1] = 95;
  a->usage_thresholds_mask = GS_USAGE_CPU | GS_USAGE_MEMORY;
  a->estimated_scaling_factors[0] = 85;
  a->estimated_scaling_factors[1] = 70;
  a->estimated_scaling_factors_mask = GS_USAGE_CPU | GS_USAGE_MEMORY;
  a->agg_usage_type = GS_AGG_NONE;
  a->agg_score_type = GS_AGG_NONE;
}

void gs_fit_args_default(gs_fit_args* a) {
  if (!a) return;
  std::memset(a, 0, sizeof(*a));
  a->resource_weights[GS_RES_CPU] = 1;
  a->resource_weights[GS_RES_MEMORY] = 1;
}

int gs_loadaware_args_validate(const gs_loadaware_args* a, char* msg, size_t len) {
  auto bad = [&](const char* s) {
    if (msg && len) snprintf(msg, len, "%s", s);
    return GS_EINVAL;
  };
  if (!a) return bad("nil args");
  if (a->has_node_metric_expiration && a->node_metric_expiration_seconds <= 0)
    return bad("nodeMetricExpiredSeconds should be a positive value");
  for (int r = 0; r < 2; ++r) {
    if (a->resource_weights_mask & (1u << r)) {
      if (a->resource_weights[r] <= 0) return bad("resource Weight should be a positive value");
      if (a->resource_weights[r] > 100) return bad("resource Weight should be less than 100");
    }
    if (a->usage_thresholds_mask & (1u << r)) {
      if (a->usage_thresholds[r] < 0) return bad("resource Threshold should be a positive value");
      if (a->usage_thresholds[r] > 100) return bad("resource Threshold should be less than 100");
    }
    if (a->estimated_scaling_factors_mask & (1u << r)) {
      if (a->estimated_scaling_factors[r] <= 0) return bad("estimated resource Threshold should be a positive value");
      if (a->estimated_scaling_factors[r] > 100) return bad("estimated  resource Threshold should be less than 100");
    }
    if ((a->resource_weights_mask & (1u << r)) && !(a->estimated_scaling_factors_mask & (1u << r)))
      return bad("estimatedScalingFactors: Not found");
  }
  if ((a->resource_weights_mask | a->usage_thresholds_mask | a->prod_usage_thresholds_mask |
       a->estimated_scaling_factors_mask | a->agg_usage_thresholds_mask) & GS_USAGE_OTHER)
    return bad("resources other than cpu/memory are not supported on this path");
  if (msg && len) msg[0] = 0;
  return GS_OK;
}

int gs_create(const gs_config* cfg, gs_ctx** out) {
  if (!cfg || !out) return GS_EINVAL;
  *out = nullptr;
  if (cfg->abi_version != GS_ABI_VERSION) return GS_EINVAL;
  gs_ctx* c = new gs_ctx();
  c->cfg = *cfg;
  char msg[256];
  if (gs_loadaware_args_validate(&cfg->loadaware, msg, sizeof msg) != GS_OK) {
    fprintf(stderr, "gpuscore: invalid LoadAwareSchedulingArgs: %s\n", msg);
    delete c;
    return GS_EINVAL;
  }
  if (cfg->num_nodes == 0) { delete c; return GS_EINVAL; }
  if (compute_profile(c) != GS_OK) {
    fprintf(stderr, "gpuscore: %s\n", c->err.c_str());
    delete c;
    return GS_EINVAL;
  }
  if (cfg->sample_nodes != 0 && cfg->sample_nodes != 1) { delete c; return GS_EINVAL; }
  c->window_k = cfg->sample_nodes ? gs_num_feasible_nodes_to_find(cfg->num_nodes, cfg->percentage_of_nodes_to_score) : 0;
  c->B = cfg->batch_size ? (int)cfg->batch_size : MAX_BATCH;
  if (c->B < 1 || c->B > MAX_BATCH || (cfg->cand_cap && cfg->cand_cap != (uint32_t)LCAP)) {
    fprintf(stderr, "gpuscore: batch_size must be in [1,%d] and cand_cap %d\n", MAX_BATCH, LCAP);
    delete c;
    return GS_EUNSUPPORTED;
  }
  c->N = cfg->num_nodes;
  c->npad = (c->N + 1023) & ~1023u;
  c->nodes.resize(c->N);
  c->numa.resize(c->N);
  // pod uid -> node maps grow by one entry per placement: buckets for a few pods per node up front, so the scheduling
  // loop does not stop for a rehash of tens of thousands of entries (a multi-ms stall of the batch pipeline)
  c->uid_node.reserve(std::max<size_t>(size_t(1) << 17, 4 * (size_t)c->N));
  c->numa_uid_node.reserve(std::max<size_t>(size_t(1) << 16, (size_t)c->N));
  c->row_dirty.assign(c->N, 0);
  c->devs.assign(c->N, gs_node_devices{});
  c->dev_dirty.assign(c->N, 0);
  c->rsv_node.assign(c->N, {});
  gs_ext_args_default(&c->ext);
  c->ext.enabled = 0;   // the extension plugins are off until gs_ext_configure
  set_shard(c);
  auto bail = [&](const char* what, hipError_t e) {
    fprintf(stderr, "gpuscore: %s: %s\n", what, hipGetErrorString(e));
    gs_destroy(c);
    return GS_EDEVICE;
  };
  hipError_t e;
  if ((e = hipSetDevice(cfg->device)) != hipSuccess) return bail("hipSetDevice", e);
  if ((e = set_kernel_attributes()) != hipSuccess) return bail("hipFuncSetAttribute", e);
  // priorities: the commit chain (patch, cand, commit on st) before the next batch's eval pass (st_ev, st2), which
  // otherwise fills every CU while patch / cand wait for slots
  int prio_lo = 0, prio_hi = 0;
  if ((e = hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi)) != hipSuccess) return bail("hipDeviceGetStreamPriorityRange", e);
  static const bool same_prio = getenv("GS_STREAM_PRIO") && getenv("GS_STREAM_PRIO")[0] == '0';
  if (same_prio) prio_hi = prio_lo;
  // (Round 3 tried a CU partition here: the commit chain on CU-masked streams, the eval pass on the other CUs, with the
  // host applying a batch's placements one batch late. CU-masked streams are blocking streams — they synchronise with
  // the null stream, which hipMemset / hipMemcpy / hipFree use — and a one-pod-batch test hung in gs_destroy's hipFree
  // with it; the commit measured no faster on a CU of its own (GS_COMMIT_EXCL). Removed)
  if ((e = hipStreamCreateWithPriority(&c->st, hipStreamNonBlocking, prio_hi)) != hipSuccess) return bail("hipStreamCreate", e);
  if ((e = hipStreamCreateWithPriority(&c->st2, hipStreamNonBlocking, prio_lo)) != hipSuccess) return bail("hipStreamCreate", e);
  if ((e = hipStreamCreateWithPriority(&c->st_ev, hipStreamNonBlocking, prio_lo)) != hipSuccess) return bail("hipStreamCreate", e);
  if ((e = hipStreamCreateWithFlags(&c->st_rb, hipStreamNonBlocking)) != hipSuccess) return bail("hipStreamCreate", e);
  if ((e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming)) != hipSuccess) return bail("hipEventCreate", e);
  if ((e = hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming)) != hipSuccess) return bail("hipEventCreate", e);
  // GS_EV_FENCE (experiments): the device-side timing events 0, 1, 4 (and with "dev2" the eval-done events the commit
  // stream waits on) recorded with a device-scope release ("dev") or no system-scope fence ("none") instead of the
  // default system-scope release (an L2 write-back between the commit and the next kernel on its stream)
  static const char* evf = getenv("GS_EV_FENCE");
  const unsigned ev_fence = !evf ? 0u : !strncmp(evf, "dev", 3) ? (unsigned)hipEventReleaseToDevice
                          : !strcmp(evf, "none") ? (unsigned)hipEventDisableSystemFence : 0u;
  const bool evdone_fence = evf && !strcmp(evf, "dev2");
  for (int i = 0; i < 6; ++i)
    if ((e = hipEventCreateWithFlags(&c->ev[i], (i == 0 || i == 1 || i == 4) ? ev_fence : 0u)) != hipSuccess)
      return bail("hipEventCreate", e);
  // GS_EV4_NT=1 (experiments): the commit-end event without timing (the levels interval then reads 0)
  static const bool ev4_nt = getenv("GS_EV4_NT") && getenv("GS_EV4_NT")[0] == '1';
  if (ev4_nt) {
    (void)hipEventDestroy(c->ev[4]);
    if ((e = hipEventCreateWithFlags(&c->ev[4], hipEventDisableTiming)) != hipSuccess) return bail("hipEventCreate", e);
  }
  size_t np = c->npad;
  if ((e = hipMalloc(&c->d_i64, np * NUM_I64_COLS * 8)) != hipSuccess) return bail("hipMalloc mirror", e);
  if ((e = hipMalloc(&c->d_i32, np * NUM_I32_COLS * 4)) != hipSuccess) return bail("hipMalloc mirror", e);
  (void)hipMemset(c->d_i64, 0, np * NUM_I64_COLS * 8);
  (void)hipMemset(c->d_i32, 0, np * NUM_I32_COLS * 4);
  c->mv.i64 = c->d_i64;
  c->mv.i32 = c->d_i32;
  c->mv.npad = (uint32_t)np;
  c->ld = c->npad;
  // pods | seq and committed | out share one allocation each: one copy per batch each way
  static_assert(sizeof(PodVec) % 8 == 0 && sizeof(PlacementDev) % 8 == 0, "staging layout");
  if ((e = hipMalloc(&c->d_pods, (sizeof(PodVec) + 8) * c->B)) != hipSuccess) return bail("hipMalloc", e);
  c->d_seq = reinterpret_cast<uint64_t*>(c->d_pods + c->B);
  if ((e = hipMalloc(&c->d_S, (size_t)c->B * c->ld * 2)) != hipSuccess) return bail("hipMalloc S", e);
  if ((e = hipMalloc(&c->d_aff, (size_t)c->B * c->ld)) != hipSuccess) return bail("hipMalloc aff", e);
  size_t xb = xchg_block_bytes(c->B, LCAP);
  if ((e = hipMalloc(&c->d_xchg_send, xb)) != hipSuccess) return bail("hipMalloc", e);
  c->xchg_bytes = xb;
  if ((e = hipMalloc(&c->d_committed, COMMITTED_BYTES + sizeof(PlacementDev) * c->B)) != hipSuccess) return bail("hipMalloc", e);
  c->d_out = reinterpret_cast<PlacementDev*>(c->d_committed + COMMITTED_BYTES / 4);
  if ((e = hipMalloc(&c->d_tb, sizeof(int32_t) * TB_N * c->B)) != hipSuccess) return bail("hipMalloc", e);
  if ((e = hipMalloc(&c->d_rowstat, sizeof(RowStat) * (1 + MAX_RANKS))) != hipSuccess) return bail("hipMalloc", e);
  if ((e = hipMalloc(&c->d_sel, 4 * (1 + MAX_RANKS))) != hipSuccess) return bail("hipMalloc", e);
  c->stage_cap = std::min<uint32_t>(c->N, 65536);
  // staged rows then their node indices (flush_rows)
  if ((e = hipMalloc(&c->d_stage_rows, (size_t)(8 * ROW_WORDS + 4) * c->stage_cap)) != hipSuccess) return bail("hipMalloc", e);
  if ((e = hipHostMalloc(&c->h_stage_rows, (size_t)(8 * ROW_WORDS + 4) * c->stage_cap, hipHostMallocDefault)) != hipSuccess)
    return bail("hipHostMalloc", e);
  if ((e = hipHostMalloc(&c->h_pods, (sizeof(PodVec) + 8) * c->B, hipHostMallocDefault)) != hipSuccess)
    return bail("hipHostMalloc", e);
  c->h_seq = reinterpret_cast<uint64_t*>(c->h_pods + c->B);
  if ((e = hipHostMalloc(&c->h_committed, COMMITTED_BYTES + sizeof(PlacementDev) * c->B, hipHostMallocDefault)) != hipSuccess)
    return bail("hipHostMalloc", e);
  c->h_out = reinterpret_cast<PlacementDev*>(c->h_committed + COMMITTED_BYTES / 4);
  if ((e = hipHostMalloc(&c->h_xchg_send, xb, hipHostMallocDefault)) != hipSuccess) return bail("hipHostMalloc", e);
  (void)hipMemset(c->d_S, 0xff, (size_t)c->B * c->ld * 2);
  {
    for (auto& sl : c->slot) {
      if ((e = hipEventCreateWithFlags(&sl.ev_go, hipEventDisableTiming)) != hipSuccess) return bail("hipEventCreate", e);
      if ((e = hipEventCreateWithFlags(&sl.ev_evdone, hipEventDisableTiming |
                                                         (evdone_fence ? (unsigned)hipEventReleaseToDevice : 0u))) != hipSuccess)
        return bail("hipEventCreate", e);
    }
    gs_ctx::Slot& s0 = c->slot[0];
    s0.d_S = c->d_S; s0.d_aff = c->d_aff;
    s0.d_pods = c->d_pods; s0.d_seq = c->d_seq; s0.d_out = c->d_out; s0.d_committed = c->d_committed;
    s0.h_pods = c->h_pods; s0.h_seq = c->h_seq; s0.h_out = c->h_out; s0.h_committed = c->h_committed;
    for (int i = 0; i < 6; ++i) s0.ev[i] = c->ev[i];
    gs_ctx::Slot& s1 = c->slot[1];
    if ((e = hipMalloc(&s1.d_S, (size_t)c->B * c->ld * 2)) != hipSuccess) return bail("hipMalloc S", e);
    if ((e = hipMalloc(&s1.d_aff, (size_t)c->B * c->ld)) != hipSuccess) return bail("hipMalloc aff", e);
    (void)hipMemset(s1.d_S, 0xff, (size_t)c->B * c->ld * 2);
    if ((e = hipMalloc(&s1.d_pods, (sizeof(PodVec) + 8) * c->B)) != hipSuccess) return bail("hipMalloc", e);
    s1.d_seq = reinterpret_cast<uint64_t*>(s1.d_pods + c->B);
    if ((e = hipMalloc(&s1.d_committed, COMMITTED_BYTES + sizeof(PlacementDev) * c->B)) != hipSuccess) return bail("hipMalloc", e);
    s1.d_out = reinterpret_cast<PlacementDev*>(s1.d_committed + COMMITTED_BYTES / 4);
    if ((e = hipHostMalloc(&s1.h_pods, (sizeof(PodVec) + 8) * c->B, hipHostMallocDefault)) != hipSuccess)
      return bail("hipHostMalloc", e);
    s1.h_seq = reinterpret_cast<uint64_t*>(s1.h_pods + c->B);
    if ((e = hipHostMalloc(&s1.h_committed, COMMITTED_BYTES + sizeof(PlacementDev) * c->B, hipHostMallocDefault)) != hipSuccess)
      return bail("hipHostMalloc", e);
    s1.h_out = reinterpret_cast<PlacementDev*>(s1.h_committed + COMMITTED_BYTES / 4);
    for (int i = 0; i < 6; ++i)
      if ((e = hipEventCreateWithFlags(&s1.ev[i], i == 4 && ev4_nt ? hipEventDisableTiming
                                                   : (i == 0 || i == 1 || i == 4) ? ev_fence : 0u)) != hipSuccess)
        return bail("hipEventCreate", e);
    c->cand_overlap = !(getenv("GS_CAND_OVERLAP") && getenv("GS_CAND_OVERLAP")[0] == '0');
    if (c->cand_overlap)
      for (auto& sl : c->slot) {
        if ((e = hipMalloc(&sl.d_lst, xb)) != hipSuccess) return bail("hipMalloc", e);
        if ((e = hipMalloc(&sl.d_hist, (size_t)4 * c->B * (MAX_SCORE_LIMIT + 1))) != hipSuccess) return bail("hipMalloc", e);
      }
    c->d_lst = s0.d_lst;
    c->d_hist = s0.d_hist;
  }
  if ((e = hipMalloc(&c->d_cscratch, cand_split_scratch_bytes())) != hipSuccess) return bail("hipMalloc", e);
  c->host_timing = getenv("GS_HOST_TIMING") && getenv("GS_HOST_TIMING")[0] == '1';
  if (getenv("GS_COMMIT_STAMPS") && getenv("GS_COMMIT_STAMPS")[0] == '1') {
    // 8 waves x 64 entries (commit_spec_kernel: one region per wave; the other commit kernels: region 0), then the
    // cand kernel's 8 at entry 512
    if ((e = hipMalloc(&c->d_stamps, 8 * 524)) != hipSuccess) return bail("hipMalloc", e);
    (void)hipMemset(c->d_stamps, 0, 8 * 524);
    set_cand_stamps(c->d_stamps + 512);
  }
  if ((e = hipDeviceSynchronize()) != hipSuccess) return bail("hipDeviceSynchronize", e);
  // 96 B (LoadAware + Fit row), + 192 B NodeNUMAResource columns when enabled
  c->stats.node_row_bytes = 3 * 8 + 4 + 2 * 8 + 2 * 8 + 2 * 8 + 2 * 8 + 4 + (c->numa_on ? 18 * 8 + 12 * 4 : 0);
  if (const char* wd = getenv("GS_WATCHDOG_S")) {
    const double lim = atof(wd);
    if (lim > 0) c->watchdog = std::thread(watchdog_loop, c, lim);
  }
  *out = c;
  return GS_OK;
}

int gs_destroy(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  async_stop(c);
  if (c->watchdog.joinable()) {
    c->wd_stop.store(true);
    c->watchdog.join();
  }
  if (c->host_timing && c->ht_batches) {
    const double n = (double)c->ht_batches;
    fprintf(stderr, "gpuscore host per batch (us, %llu batches): waiting for the batch %.0f | applying placements %.0f | "
            "staging the next %.0f | enqueueing it %.0f | busy max %.0f; busy histogram (100-us bins):",
            (unsigned long long)c->ht_batches, c->ht_wait / n, c->ht_apply / n, c->ht_stage / n, c->ht_launch / n,
            c->ht_max_busy);
    for (int k = 0; k < 8; ++k) fprintf(stderr, " %llu", (unsigned long long)c->ht_busy_hist[k]);
    fprintf(stderr, "\n");
  }
  if (c->host_timing && c->hx_pods) {
    const double n = (double)c->hx_pods;
    fprintf(stderr, "gpuscore extension path (us): per extension pod (%llu): records %.1f | flushes %.1f | device chain "
            "to wake-up %.1f | Reserves %.1f; per plain run (%llu): gs_schedule %.1f\n", (unsigned long long)c->hx_pods,
            c->hx_prep / n, c->hx_flush / n, c->hx_gpu / n, c->hx_reserve / n, (unsigned long long)c->hx_runs,
            c->hx_runs ? c->hx_plain / (double)c->hx_runs : 0.0);
  }
  if (c->d_dev_stage) (void)hipFree(c->d_dev_stage);
  if (c->h_dev_stage) (void)hipHostFree(c->h_dev_stage);
  for (void* p : {(void*)c->d_dev, (void*)c->d_xin, (void*)c->d_xtot,
                  (void*)c->d_xds, (void*)c->d_xrs, (void*)c->d_xnom, (void*)c->d_xT, (void*)c->d_xout})
    if (p) (void)hipFree(p);
  for (void* p : {(void*)c->h_xin, (void*)c->h_xout, (void*)c->h_xnom})
    if (p) (void)hipHostFree(p);
  if (c->d_stamps) {
    std::vector<uint64_t> sa(524);
    if (hipMemcpy(sa.data(), c->d_stamps, 8 * 524, hipMemcpyDeviceToHost) == hipSuccess) {
      if (!c->window_k) {   // speculative commit kernel: one stamp region per wave
        const double np = c->stats_all_pods ? (double)c->stats_all_pods : 1.0;
        auto W = [&](int w, int i) { return (double)sa[w * 64 + i] / np; };
        fprintf(stderr, "gpuscore spec commit, cycles per committed pod (%llu pods, %llu decisions, %llu rollbacks, %.0f "
                "rollback cycles, full-row %llu):\n", (unsigned long long)c->stats_all_pods, (unsigned long long)sa[9],
                (unsigned long long)sa[3], W(0, 4) + W(0, 37) + W(0, 38) + W(0, 39),
                (unsigned long long)sa[10]);
        fprintf(stderr, "  wave 0 total %.0f: checks %.0f | dirty state %.0f | hdr+fresh store+dirty loads %.0f | level scan "
                "%.0f | winner %.0f | fresh slot %.0f | record %.0f | waiting %.0f (at batch end %.0f) | full-row %.0f\n",
                W(0, 12), W(0, 27), W(0, 28), W(0, 29), W(0, 18), W(0, 19), W(0, 20), W(0, 0), W(0, 2), W(0, 23), W(0, 11));
        if (sa[64 + 9] > 0)   // the split selector: wave 0 finishes the prep wave's decisions and verifies
          fprintf(stderr, "  wave 0 (split): verification loop %.0f | fresh slot's scores + snapshot %.0f | record read + late "
                  "decisions %.0f | exclusions %.0f | rows settled early %.0f | window %.0f | record %.0f (fresh slot %.0f) | "
                  "waiting %.0f (the loop's passes while waiting count in the first two)\n", W(0, 55), W(0, 27), W(0, 52),
                  W(0, 53), W(0, 54), W(0, 19), W(0, 0), W(0, 20), W(0, 2));
        if (sa[64 + 9] > 0)
          fprintf(stderr, "  wave 0 (split) waiting passes per pod: batch end %.2f | speculation depth %.2f | host cut %.2f | "
                  "exact record asked %.2f | prep record not ready %.2f\n", W(0, 56), W(0, 57), W(0, 58), W(0, 59), W(0, 60));
        fprintf(stderr, "  winner split: ties + tie-break position %.0f | old-nodes path: level segment + list window %.0f\n",
                W(0, 30), W(0, 46));
        if (sa[64 + 9] == 0)   // (single selector wave; the split selector reuses these entries, printed below)
          fprintf(stderr, "  late-landing estimate: %llu decisions, previous pod's row as it stood > M %llu, == M %llu (tie-break "
                "position moves %llu)\n", (unsigned long long)sa[47], (unsigned long long)sa[48], (unsigned long long)sa[49],
                (unsigned long long)sa[50]);
        fprintf(stderr, "  wave 0 raw (cycles per pod by stamp index):");
        for (int i = 0; i < 60; ++i)
          if (sa[i] && (i < 47 || i > 50)) fprintf(stderr, " %d=%.0f", i, W(0, i));
        fprintf(stderr, "\n  wave 1 raw (the split selector's prep wave):");
        for (int i = 0; i < 52; ++i)
          if (sa[64 + i]) fprintf(stderr, " %d=%.0f", i, W(1, i));
        fprintf(stderr, "\n  split: late landings %llu, full decisions %llu, excluded ties %llu, rows settled early %llu\n",
                (unsigned long long)sa[47], (unsigned long long)sa[48], (unsigned long long)sa[49], (unsigned long long)sa[50]);
        const double ng = sa[31] ? (double)sa[31] : 1.0;
        fprintf(stderr, "  winner: old-nodes-only path %llu decisions (%.1f%%), general path %llu (%.1f%%): avg old %.1f new "
                "%.1f window %.1f; avg dirty slots %.1f; list window beyond 32: %llu, beyond 64: %llu\n",
                (unsigned long long)sa[36], 100.0 * sa[36] / np, (unsigned long long)sa[31], 100.0 * sa[31] / np,
                sa[32] / (ng + sa[36]), sa[33] / ng, sa[34] / ng, sa[35] / np, (unsigned long long)sa[24],
                (unsigned long long)sa[25]);
        const double nr = sa[3] ? (double)sa[3] : 1.0;
        auto R = [&](int i) { return (double)sa[i] / nr; };
        fprintf(stderr, "  rollback (cycles per rollback): parking %.0f | undo+hash %.0f | restored-row re-scoring %.0f | "
                "rest %.0f; restored rows %.2f, depth %.2f decisions\n", R(37), R(38), R(39), R(4), R(40), R(41));
        fprintf(stderr, "  pending row's pre-landing score >= M: %llu decisions, %llu of the rollbacks; > M: %llu decisions, %llu "
                "of the rollbacks\n", (unsigned long long)sa[42], (unsigned long long)sa[43], (unsigned long long)sa[44],
                (unsigned long long)sa[45]);
        const bool split = sa[64 + 9] > 0;   // the prep wave counted its records: the split selector ran
        if (split)
          fprintf(stderr, "  wave 1 (prep): busy %.0f (dirty state %.0f, loads %.0f, level scan %.0f, winner %.0f, record "
                  "%.0f) waiting %.0f\n", W(1, 28) + W(1, 29) + W(1, 18) + W(1, 30) + W(1, 46) + W(1, 19) + W(1, 0),
                  W(1, 28), W(1, 29), W(1, 18), W(1, 30) + W(1, 46) + W(1, 19), W(1, 0), W(1, 2));
        else
          fprintf(stderr, "  wave 4 (verify): busy %.0f waiting %.0f\n", W(4, 1), W(4, 2));
        for (int w = 2; w < 4; ++w)
          fprintf(stderr, "  wave %d (Reserve): fetch+undo %.0f numa_eval %.0f lane0 %.0f rest %.0f (fresh fetch %.0f, landed-"
                  "again wait %.0f) waiting %.0f (first decision %.0f)\n", w, W(w, 15), W(w, 16), W(w, 17), W(w, 5), W(w, 21),
                  W(w, 22), W(w, 6), W(w, 26));
        for (int w : {split ? 4 : 1, 5, 6, 7})
          fprintf(stderr, "  wave %d (re-scoring): busy %.0f (row copy + hint table %.0f, scores %.0f) waiting %.0f, jobs %.2f "
                  "per pod\n", w, W(w, 7) + W(w, 9), W(w, 9), W(w, 7), W(w, 8), W(w, 10));
        for (int base : {30, 40}) {   // re-scoring jobs by what their lanes needed (gs_commit_spec.hip, ST)
          uint64_t v[8] = {};
          for (int w : {split ? 4 : 1, 5, 6, 7})
            for (int i = 0; i < 8; ++i) v[i] += sa[w * 64 + base + i];
          fprintf(stderr, "  re-scoring jobs on %s rows: %llu jobs, %llu lanes: infeasible at batch start %llu, below the "
                  "lowest listed level %llu, needed %llu, lists too short %llu; jobs with every lane infeasible %llu, with "
                  "no lane needed %llu\n", base == 30 ? "no-policy" : "NUMA-policy", (unsigned long long)v[0],
                  (unsigned long long)v[1], (unsigned long long)v[2], (unsigned long long)v[3], (unsigned long long)v[4],
                  (unsigned long long)v[5], (unsigned long long)v[6], (unsigned long long)v[7]);
        }
        const double nb = c->stats.batches ? (double)c->stats.batches * c->B : 1.0;
        fprintf(stderr, "gpuscore cand_kernel, wave-0 cycles per pod row: pass 1 %.0f, level sums %.0f, level pick %.0f, "
                "offsets %.0f, pass 2 %.0f\n", sa[512] / nb, sa[513] / nb, sa[514] / nb, sa[515] / nb, sa[516] / nb);
        fprintf(stderr, "gpuscore fix_levels_kernel, thread-0 cycles per pod row: loads+dedupe %.0f, landed rows + level pick "
                "%.0f, lists %.0f; the block's slowest landed-row lane: row loads %.0f, loads + evaluation %.0f; thread 0: "
                "start -> its evaluation %.0f, start -> every lane evaluated %.0f\n",
                sa[517] / nb, sa[518] / nb, sa[519] / nb, sa[520] / nb, sa[521] / nb, sa[522] / nb, sa[523] / nb);
        (void)hipFree(c->d_stamps);
        c->d_stamps = nullptr;
      }
    }
  }
  if (c->d_stamps) {
    uint64_t st[32] = {};
    if (hipMemcpy(st, c->d_stamps, 256, hipMemcpyDeviceToHost) == hipSuccess) {
      uint64_t tot = 0;
      for (int i = 0; i < 12; ++i) tot += st[i];
      fprintf(stderr, "gpuscore commit phases (s_memtime ticks, %% of %llu):", (unsigned long long)tot);
      for (int i = 0; i < 12; ++i) fprintf(stderr, " p%d=%.1f%%", i, tot ? 100.0 * st[i] / tot : 0.0);
      fprintf(stderr, "\n  raw ticks per committed pod (%llu pods):", (unsigned long long)c->stats_all_pods);
      for (int i = 0; i < 22; ++i)
        fprintf(stderr, " s%d=%.0f", i, c->stats_all_pods ? (double)st[i] / (double)c->stats_all_pods : 0.0);
      fprintf(stderr, "\n  pods through full-row resolution %llu, FitError %llu, slow path %llu",
              (unsigned long long)st[18], (unsigned long long)st[19], (unsigned long long)st[20]);
      fprintf(stderr, ", winners on NUMA-policy rows %llu, fresh winners %llu, cpuset pods %llu | s24 (Reserve pair "
              "evaluation) %.0f", (unsigned long long)st[22], (unsigned long long)st[23], (unsigned long long)st[25],
              c->stats_all_pods ? (double)st[24] / (double)c->stats_all_pods : 0.0);
      fprintf(stderr, " | s26 (full-row resolution, per such pod) %.0f", st[18] ? (double)st[26] / (double)st[18] : 0.0);
      fprintf(stderr, " | policy-row rescoring: %llu pods, %.0f ticks per pair (thread 128)\n",
              (unsigned long long)st[12], st[12] ? (double)st[13] / st[12] : 0.0);
    }
    (void)hipFree(c->d_stamps);
  }
  if (c->comm) ncclCommDestroy(c->comm);
  if (c->lg_ready) (void)hipEventDestroy(c->lg_ready);
  if (c->lg_done) (void)hipEventDestroy(c->lg_done);
  for (hipEvent_t ev : c->x_ev) (void)hipEventDestroy(ev);
  if (c->st) (void)host_wait_stream(c->st);
  if (c->st_ev) (void)host_wait_stream(c->st_ev);
  if (c->st_rb) (void)host_wait_stream(c->st_rb);   // readbacks into the pinned buffers freed below
  if (c->slot[0].d_pods) bind_slot(c, 0);
  {
    gs_ctx::Slot& s1 = c->slot[1];
    for (auto& sl : c->slot) {
      if (sl.ev_go) (void)hipEventDestroy(sl.ev_go);
      if (sl.ev_evdone) (void)hipEventDestroy(sl.ev_evdone);
    }
      for (auto& sl : c->slot) {
      if (sl.d_lst) (void)hipFree(sl.d_lst);
      if (sl.d_hist) (void)hipFree(sl.d_hist);
      sl.d_lst = nullptr;
      sl.d_hist = nullptr;
    }
    c->d_lst = nullptr;
    c->d_hist = nullptr;
    if (c->d_cscratch) (void)hipFree(c->d_cscratch);
    c->d_cscratch = nullptr;
    void* d1[] = {s1.d_pods, s1.d_committed, s1.d_S, s1.d_aff};   // (seq / out live inside pods / committed)
    for (void* p : d1)
      if (p) (void)hipFree(p);
    void* h1[] = {s1.h_pods, s1.h_committed};
    for (void* p : h1)
      if (p) (void)hipHostFree(p);
    for (auto& ev : s1.ev)
      if (ev) (void)hipEventDestroy(ev);
  }
  void* dev[] = {c->d_xerr, c->d_xsmall,
                 c->d_i64, c->d_i32, c->d_pods, c->d_S, c->d_xchg_send, c->d_xchg_recv, c->d_xmerged,
                 c->d_committed, c->d_rowstat, c->d_sel, c->d_stage_idx, c->d_stage_rows, c->d_numa_idx, c->d_xnuma_idx,
                 c->d_topos, c->d_aff, c->d_tb, c->d_sx_send, c->d_sx_recv};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  void* host[] = {c->h_sx_send, c->h_sx_recv, c->h_xsmall, c->h_pods, c->h_committed, c->h_stage_idx, c->h_stage_rows, c->h_xchg_send,
                  c->h_xchg_recv};
  for (void* p : host)
    if (p) (void)hipHostFree(p);
  for (auto& ev : c->ev)
    if (ev) (void)hipEventDestroy(ev);
  if (c->st_ev) (void)hipStreamDestroy(c->st_ev);
  if (c->st_rb) (void)hipStreamDestroy(c->st_rb);
  if (c->slab_mv.i64) (void)hipFree(c->slab_mv.i64);
  if (c->slab_mv.i32) (void)hipFree(c->slab_mv.i32);
  if (c->st2) (void)host_wait_stream(c->st2);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->st2) (void)hipStreamDestroy(c->st2);
  if (c->st) (void)hipStreamDestroy(c->st);
  delete c;
  return GS_OK;
}

const char* gs_last_error(gs_ctx* c) {
  if (!c) return "nil context";
  quiesce(c);
  return c->err.c_str();
}

int gs_set_now(gs_ctx* c, int64_t now) {
  if (!c) return GS_EINVAL;
  quiesce(c);
  if (now != c->now) c->prep_stale = true;
  c->now = now;
  return GS_OK;
}

int gs_nodes_upsert(gs_ctx* c, const uint32_t* idx, const gs_node* nodes, uint32_t n) {
  if (!c || (!nodes && n)) return GS_EINVAL;
  quiesce(c);
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t i = idx ? idx[j] : j;
    if (i >= c->N) return fail(c, GS_EINVAL, "node index %u >= %u", i, c->N);
    int rc = validate_node(c, nodes[j]);
    if (rc) return rc;
    c->nodes[i].node = nodes[j];
    if (!c->nodes[i].valid) ++c->n_valid;
    c->nodes[i].valid = true;
    mark_dirty(c, i);
  }
  return flush_rows(c);
}

int gs_node_metrics_upsert(gs_ctx* c, const uint32_t* idx, const gs_node_metric* m, uint32_t n,
                           const gs_pod_metric* pm, const uint32_t* off) {
  if (!c || (!m && n)) return GS_EINVAL;
  quiesce(c);
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t i = idx ? idx[j] : j;
    if (i >= c->N) return fail(c, GS_EINVAL, "node index %u >= %u", i, c->N);
    if (m[j].n_aggregated < 0 || m[j].n_aggregated > GS_MAX_AGG_USAGES)
      return fail(c, GS_EINVAL, "n_aggregated %d outside [0,%d]", m[j].n_aggregated, GS_MAX_AGG_USAGES);
    HostNode& hn = c->nodes[i];
    index_metric_names(c, hn, -1);
    hn.metric = m[j];
    hn.pms.clear();
    if (pm && off) hn.pms.assign(pm + off[j], pm + off[j + 1]);
    index_metric_names(c, hn, +1);
    mark_dirty(c, i);
  }
  return flush_rows(c);
}

int gs_pods_assign(gs_ctx* c, const uint32_t* node_idx, const gs_pod* pods, const int64_t* ts, uint32_t n) {
  if (!c || (n && (!node_idx || !pods))) return GS_EINVAL;
  quiesce(c);
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t i = node_idx[j];
    if (i >= c->N) return fail(c, GS_EINVAL, "node index %u >= %u", i, c->N);
    if (pods[j].flags & GS_POD_TERMINATED) continue;       // pod_assign_cache.go:54
    c->nodes[i].assigned[pods[j].uid] = Assigned{ts ? ts[j] : c->now, pods[j]};
    c->uid_node[pods[j].uid] = i;
    mark_dirty(c, i);
  }
  return flush_rows(c);
}

int gs_pods_unassign(gs_ctx* c, const uint32_t* node_idx, const gs_pod* pods, uint32_t n) {
  if (!c || (n && (!node_idx || !pods))) return GS_EINVAL;
  quiesce(c);
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t i = node_idx[j];
    if (i >= c->N) return fail(c, GS_EINVAL, "node index %u >= %u", i, c->N);
    c->nodes[i].assigned.erase(pods[j].uid);
    auto it = c->uid_node.find(pods[j].uid);
    if (it != c->uid_node.end() && it->second == i) c->uid_node.erase(it);
    c->ext_reserved.erase(pods[j].uid);   // the pod left: its extension-path Reserve record goes with it
    mark_dirty(c, i);
  }
  return flush_rows(c);
}

// The scheduler cache's ForgetPod of an assumed pod after the Unreserve plugins ([upstream] scheduleOne's binding-cycle
// failure path): NodeInfo.RemovePod, LoadAware Unreserve (podAssignCache.unAssign, load_aware.go:265-267) and
// NodeNUMAResource Unreserve (resourceManager.Release, plugin.go:467-476).
int gs_pods_forget(gs_ctx* c, const uint32_t* node_idx, const gs_pod* pods, uint32_t n) {
  if (!c || (n && (!node_idx || !pods))) return GS_EINVAL;
  quiesce(c);
  for (uint32_t j = 0; j < n; ++j) {
    if (node_idx[j] >= c->N) return fail(c, GS_EINVAL, "node index %u >= %u", node_idx[j], c->N);
    // the extension path's Reserves (DeviceShare minors and GPU-name / extended-resource requests, Reservation
    // AddAssignedPod) have no Unreserve here: refused before anything changes
    if (c->ext_reserved.count(pods[j].uid))
      return fail(c, GS_EUNSUPPORTED, "gs_pods_forget: pod %llu was placed with a DeviceShare / Reservation Reserve "
                  "(gs_schedule_ext), whose Unreserve this library does not restate", (unsigned long long)pods[j].uid);
  }
  for (uint32_t j = 0; j < n; ++j) {
    const uint32_t i = node_idx[j];
    const gs_pod& p = pods[j];
    HostNode& hn = c->nodes[i];
    for (int s = 0; s < GS_NUM_RES; ++s) hn.node.requested[s] -= p.requests[s];
    hn.node.nonzero_requested[0] -= p.nonzero_requests[0];
    hn.node.nonzero_requested[1] -= p.nonzero_requests[1];
    hn.node.pod_count -= 1;
    hn.assigned.erase(p.uid);
    auto it = c->uid_node.find(p.uid);
    if (it != c->uid_node.end() && it->second == i) c->uid_node.erase(it);
    if (c->numa_on) {
      numa_release(c->numa[i], p.uid);
      auto nt = c->numa_uid_node.find(p.uid);
      if (nt != c->numa_uid_node.end() && nt->second == i) c->numa_uid_node.erase(nt);
    }
    mark_dirty(c, i);
  }
  return flush_rows(c);
}

int gs_pods_on_event(gs_ctx* c, int event, const int32_t* node_idx, const gs_pod* pods, uint32_t n) {
  if (!c || (n && (!node_idx || !pods))) return GS_EINVAL;
  quiesce(c);
  if (event < GS_POD_EVENT_ADD || event > GS_POD_EVENT_DELETE) return fail(c, GS_EINVAL, "unknown pod event %d", event);
  for (uint32_t j = 0; j < n; ++j) {
    const int32_t i = node_idx[j];
    if (i >= (int32_t)c->N) return fail(c, GS_EINVAL, "node index %d >= %u", i, c->N);
    if (i < 0) continue;                                      // nodeName == "": assign / unAssign return early
    const bool terminated = pods[j].flags & GS_POD_TERMINATED;
    const bool assign = event == GS_POD_EVENT_ADD || (event == GS_POD_EVENT_UPDATE && !terminated);
    int rc = assign ? gs_pods_assign(c, (const uint32_t*)&node_idx[j], &pods[j], nullptr, 1)
                    : gs_pods_unassign(c, (const uint32_t*)&node_idx[j], &pods[j], 1);
    if (rc) return rc;
  }
  return GS_OK;
}

int gs_assign_cache_get(gs_ctx* c, uint32_t node, uint64_t* uids, int64_t* ts, uint32_t cap) {
  if (!c || node >= c->N) return GS_EINVAL;
  quiesce(c);
  std::vector<std::pair<uint64_t, int64_t>> v;
  for (const auto& kv : c->nodes[node].assigned) v.push_back({kv.first, kv.second.ts});
  std::sort(v.begin(), v.end());
  for (uint32_t k = 0; k < v.size() && k < cap; ++k) {
    if (uids) uids[k] = v[k].first;
    if (ts) ts[k] = v[k].second;
  }
  return (int)v.size();
}

int gs_evaluate(gs_ctx* c, const gs_pod* pods, uint32_t npods, int16_t* scores, uint16_t* codes,
                int16_t* plugin_scores) {
  if (!c || (npods && !pods)) return GS_EINVAL;
  quiesce(c);
  int rc = ready(c);
  if (rc) return rc;
  if ((rc = flush_rows(c))) return rc;
  if ((rc = node_prep(c))) return rc;
  const uint32_t N = c->N;
  const int chunk = c->B;
  int16_t *d_sc = nullptr, *d_pl = nullptr;
  uint16_t* d_cd = nullptr;
  HIP_TRY(c, hipMalloc(&d_sc, (size_t)chunk * N * 2));
  HIP_TRY(c, hipMalloc(&d_cd, (size_t)chunk * N * 2));
  HIP_TRY(c, hipMalloc(&d_pl, (size_t)chunk * N * 2 * GS_NUM_PLUGINS));
  for (uint32_t p0 = 0; p0 < npods; p0 += chunk) {
    int b = (int)std::min<uint32_t>(chunk, npods - p0);
    int prod_cols = 0;
    for (int i = 0; i < b; ++i) {
      if ((rc = validate_pod(c, pods[p0 + i]))) break;
      c->h_pods[i] = prep_pod(c, pods[p0 + i]);
      prod_cols |= (c->h_pods[i].flags & PF_PROD_SCORE) ? 1 : 0;
    }
    if (rc) break;
    HIP_TRY(c, hipMemcpyAsync(c->d_pods, c->h_pods, sizeof(PodVec) * b, hipMemcpyHostToDevice, c->st));
    HIP_TRY(c, launch_eval_full(c->mv, c->d_pods, b, c->pf, N, d_sc, d_cd, d_pl, prod_cols, c->st));
    if (scores) HIP_TRY(c, hipMemcpyAsync(scores + (size_t)p0 * N, d_sc, (size_t)b * N * 2, hipMemcpyDeviceToHost, c->st));
    if (codes) HIP_TRY(c, hipMemcpyAsync(codes + (size_t)p0 * N, d_cd, (size_t)b * N * 2, hipMemcpyDeviceToHost, c->st));
    if (plugin_scores)
      HIP_TRY(c, hipMemcpyAsync(plugin_scores + (size_t)p0 * N * GS_NUM_PLUGINS, d_pl, (size_t)b * N * 2 * GS_NUM_PLUGINS,
                                hipMemcpyDeviceToHost, c->st));
    HIP_TRY(c, host_wait_stream(c->st));
  }
  (void)hipFree(d_sc);
  (void)hipFree(d_cd);
  (void)hipFree(d_pl);
  return rc;
}

namespace {
// batch [i, i+b): a special pod always runs alone (its row is re-derived on the host afterwards)
int batch_len(const gs_ctx* c, const gs_pod* pods, uint32_t i, uint32_t npods, bool* special_first) {
  int b = (int)std::min<uint32_t>(c->B, npods - i);
  *special_first = special_pod(c, pods[i]);
  if (*special_first) return 1;
  for (int j = 1; j < b; ++j)
    if (special_pod(c, pods[i + j])) return j;
  return b;
}

// PreFilter of pods [i, i+b) into the bound slot, and their upload
// (uploads on st_ev, where the batch's eval pass runs; a non-speculative batch's eval first waits for everything
// enqueued on st — row deltas, node prep, the previous commit — a speculative one only for the eval pass before it)
int stage_batch(gs_ctx* c, const gs_pod* pods, const uint64_t* seq, uint32_t i, int b, bool speculative) {
  for (int j = 0; j < b; ++j) {
    c->h_pods[j] = prep_pod(c, pods[i + j]);
    c->h_seq[j] = seq ? seq[i + j] : (uint64_t)(i + j);
  }
  if (!speculative) {
    const gs_ctx::Slot& sl = c->slot[c->cur_slot];
    HIP_TRY(c, hipEventRecord(sl.ev_go, c->st));
    HIP_TRY(c, hipStreamWaitEvent(c->st_ev, sl.ev_go, 0));
  }
  // one copy: the B pod vectors' block (b of them staged) and the b sequence numbers after it (GS_MERGE_UP=0,
  // experiments: two copies)
  static const bool merge_up = !(getenv("GS_MERGE_UP") && getenv("GS_MERGE_UP")[0] == '0');
  hipStream_t up = direct_batch(c, b, speculative) ? c->st : c->st_ev;
  // (the merged copy spans all B pod vectors, d_seq following the block: a short batch copies its b vectors and seq)
  if (merge_up && 4 * b >= c->B) {
    HIP_TRY(c, hipMemcpyAsync(c->d_pods, c->h_pods, sizeof(PodVec) * c->B + 8 * b, hipMemcpyHostToDevice, up));
  } else {
    HIP_TRY(c, hipMemcpyAsync(c->d_pods, c->h_pods, sizeof(PodVec) * b, hipMemcpyHostToDevice, up));
    HIP_TRY(c, hipMemcpyAsync(c->d_seq, c->h_seq, 8 * b, hipMemcpyHostToDevice, up));
  }
  return GS_OK;
}

bool uid_overlap(const gs_pod* a, int na, const gs_pod* b, int nb) {
  std::unordered_set<uint64_t> u;
  u.reserve(2 * na);
  for (int i = 0; i < na; ++i) u.insert(a[i].uid);
  for (int i = 0; i < nb; ++i)
    if (u.count(b[i].uid)) return true;
  return false;
}
}  // namespace

extern "C++" {
namespace {
// A contiguous run of the pod stream: one gs_schedule call or one gs_schedule_submit.
struct PodRun {
  const gs_pod* pods = nullptr;
  const uint64_t* seq = nullptr;
  gs_placement* out = nullptr;
  uint32_t n = 0;
  void* tag = nullptr;
};

// Several ranks: whether the next run is already known (gs_schedule_submit) is a matter of each rank's timing. The
// ranks agree on it at every batch that ends a run (all of them must hold it), so that they speculate across the run
// boundary together and their exchanges pair up; a rank that holds the next run when the others do not starts it
// after the current one without speculation, as they do. Behind the current batch's all-gather on its stream, so that
// every collective of the context is ordered by its streams (an RCCL communicator's collectives must run in issue
// order): score rows on st_ev (the commit in flight on st keeps running while the host waits), levels on st.
int agree_next_run(gs_ctx* c, bool* use) {
  const uint32_t mine = *use ? 1u : 0u;
  std::vector<uint32_t> all(c->nranks);
  if (int rc = exchange_small(c, XSITE_RUNS, nullptr, 4, all.data(), c->sgather ? c->st_ev : c->st, &mine)) return rc;
  for (uint32_t v : all) *use = *use && v;
  return GS_OK;
}

// The scheduleOne loop over the pod stream, batch by batch. Pipelining: while batch [i, i+b) runs, the next batch is
// staged and enqueued behind it on the stream (other slot). Its commit kernel checks on the device that the batch
// before committed all its pods with no host-side Reserve pending, else it is a no-op; the host only keeps it when the
// same holds on its side. The next batch may be the first of the next run (next_run: the run after the current one
// if it is already known), so the pipeline continues across runs. Every rank takes the same decisions (replicated
// host state), so speculative exchanges pair up; with the host-callback transport the speculative pass's exchange
// waits for the current batch (no overlap, same result). run_done(run, rc): the run's placements are all written
// (rc 0), or it failed; on an error the current run gets the error and a run already taken from next_run GS_ESTATE.
template <class Next, class Done>
int schedule_stream(gs_ctx* c, PodRun run, Next&& next_run, Done&& run_done) {
  static const bool no_spec = getenv("GS_NO_PIPELINE") && getenv("GS_NO_PIPELINE")[0] == '1';
  const bool can_spec = !no_spec;
  PodRun nxt{};
  bool have_nxt = false;
  auto drain = [&]() {
    Where w_(c, "schedule_stream: drain");
    (void)host_wait_stream(c->st);
    (void)host_wait_stream(c->st_ev);
    (void)host_wait_stream(c->st_rb);   // a voided or in-flight batch's readback into the pinned buffers
  };
  auto apply_batch = [&](const gs_pod* pods, gs_placement* outp, int n, const PlacementDev* hout, const PodVec* hpods,
                         bool special) -> int {
    for (int k = 0; k < n; ++k) {
      const PlacementDev& pd = hout[k];
      gs_placement& o = outp[k];
      o.node = pd.node;
      o.feasible = pd.feasible;
      o.score = pd.node >= 0 ? pd.score : 0;
      o.ties = pd.node >= 0 ? pd.ties : 0;
      o.flags = pd.flags & ~PL_INTERNAL_FLAGS;
      if (pd.flags & GS_PLACED_SLOWPATH) c->stats.slowpath_pods += 1;   // resolved from its whole score row
      if (int rc = numa_reserve(c, pods[k], hpods[k], pd)) return rc;
      apply_placement(c, pods[k], pd.node, special);
    }
    return GS_OK;
  };
  // Deferred application: a batch that committed every pod with no host work and no special pod changes no row on
  // the host side (apply_placement / numa_reserve only mirror what the commit wrote to HBM), so its placements are
  // applied to the host state after the batch two ahead is launched — the eval pass then starts right as the previous
  // commit ends instead of after the host's ~0.2 ms of bookkeeping, and runs beside the next commit (GS_DEFER_APPLY=0:
  // apply first).
  static const bool defer_ok = !(getenv("GS_DEFER_APPLY") && getenv("GS_DEFER_APPLY")[0] == '0');
  struct Pend {
    const gs_pod* pods = nullptr;
    gs_placement* out = nullptr;
    int n = 0;
    bool active = false;
  } pend;
  std::vector<PlacementDev> pend_out;
  std::vector<PodVec> pend_pods;
  auto apply_pending = [&]() -> int {
    if (!pend.active) return GS_OK;
    pend.active = false;
    return apply_batch(pend.pods, pend.out, pend.n, pend_out.data(), pend_pods.data(), false);
  };
  auto body = [&]() -> int {
    int rc = GS_OK;
    uint32_t i = 0;
    bool inflight = false, cur_special = false, spec_ok = true;
    int cur_b = 0;
    for (;;) {
      if (i == run.n) {   // the run is complete; the next one (its first batch may be in flight already)
        if ((rc = apply_pending())) { drain(); return rc; }
        run_done(run, GS_OK);
        if (!have_nxt) have_nxt = next_run(&nxt);
        if (!have_nxt) break;
        run = nxt;
        have_nxt = false;
        i = 0;
        continue;
      }
      const gs_pod* pods = run.pods;
      if (!inflight) {
        if ((rc = apply_pending())) { drain(); return rc; }
        if ((rc = flush_rows(c))) return rc;
        if (c->prep_stale && (rc = node_prep(c))) return rc;
        cur_b = batch_len(c, pods, i, run.n, &cur_special);
        // (a cpuset pod whose node is outside the device cpuset scope ends the batch inside the commit kernel)
        if ((rc = stage_batch(c, pods, run.seq, i, cur_b, false))) return rc;
        if ((rc = launch_batch(c, cur_b, nullptr))) return rc;
      }
      // the batch after this one: in this run, or the first of the next run
      const gs_pod* np = nullptr;
      const uint64_t* ns = nullptr;
      uint32_t nj = 0, nn = 0;
      const uint32_t j = i + cur_b;
      if (j < run.n) {
        np = pods; ns = run.seq; nj = j; nn = run.n;
      } else {
        if (!have_nxt) have_nxt = next_run(&nxt);
        bool use = have_nxt && nxt.n;
        if (c->nranks > 1 && (rc = agree_next_run(c, &use))) { drain(); return rc; }
        if (use) { np = nxt.pods; ns = nxt.seq; nn = nxt.n; }
      }
      bool spec = false;
      int nb = 0;
      using hclk = std::chrono::steady_clock;
      const auto t_a = hclk::now();
      double busy = 0;
      if (pend.active && np) {   // the next batch shares a pod uid with the deferred one: its host state first
        const int nb0 = std::min<int>(c->B, (int)(nn - nj));
        if (uid_overlap(pend.pods, pend.n, np + nj, nb0) && (rc = apply_pending())) { drain(); return rc; }
      }
      if (can_spec && spec_ok && !cur_special && np && c->dirty_list.empty() && !c->prep_stale) {
        bool sf = false;
        nb = batch_len(c, np, nj, nn, &sf);
        if (!sf && !uid_overlap(pods + i, cur_b, np + nj, nb)) {
          const int32_t* prev = c->d_committed;
          const PlacementDev* prev_out = c->d_out;
          const int here = c->cur_slot;
          bind_slot(c, 1 - here);
          rc = stage_batch(c, np, ns, nj, nb, true);
          const auto t_b = hclk::now();
          if (!rc) rc = launch_batch(c, nb, prev, prev_out, cur_b);
          if (c->host_timing) {
            const double st = std::chrono::duration<double, std::micro>(t_b - t_a).count();
            const double la = std::chrono::duration<double, std::micro>(hclk::now() - t_b).count();
            c->ht_stage += st;
            c->ht_launch += la;
            busy += st + la;
          }
          bind_slot(c, here);
          if (rc) { drain(); return rc; }
          spec = true;
        }
      }
      // the previous batch's deferred placements, while this batch and the one after it run
      if ((rc = apply_pending())) { drain(); return rc; }
      spec_ok = true;
      int committed = 0;
      const auto t_w = hclk::now();
      rc = finish_batch(c, cur_b, spec, &committed);
      const auto t_f = hclk::now();
      if (rc == GS_REDO) {   // pod 0 needs the full-row path, the speculative pass (void) overwrote its lists: re-run
        drain();
        if ((rc = apply_pending())) return rc;
        if ((rc = stage_batch(c, pods, run.seq, i, cur_b, false))) return rc;
        if ((rc = launch_batch(c, cur_b, nullptr))) return rc;
        inflight = true;
        spec_ok = false;
        continue;
      }
      if (rc) { if (spec) drain(); return rc; }
      const bool host_work = c->h_committed[1] != 1;   // the device-side continuation flag the speculative pass read
      if (defer_ok && spec && !host_work && !cur_special && committed == cur_b) {
        // no host row changes: keep the results (this slot's buffers are reused by the batch two ahead) and apply them
        // after that batch is launched
        pend_out.assign(c->h_out, c->h_out + committed);
        pend_pods.assign(c->h_pods, c->h_pods + committed);
        pend.pods = pods + i;
        pend.out = run.out + i;
        pend.n = committed;
        pend.active = true;
      } else if ((rc = apply_batch(pods + i, run.out + i, committed, c->h_out, c->h_pods, cur_special))) {
        if (spec) drain();
        return rc;
      }
      if (c->host_timing) {
        const double wt = std::chrono::duration<double, std::micro>(t_f - t_w).count();
        const double ap = std::chrono::duration<double, std::micro>(hclk::now() - t_f).count();
        c->ht_wait += wt;
        c->ht_apply += ap;
        busy += ap;
        c->ht_batches += 1;
        c->ht_max_busy = std::max(c->ht_max_busy, busy);
        c->ht_busy_hist[std::min(7, (int)(busy / 100.0))] += 1;   // 100-us bins
      }
      c->stats.pods += committed;
      c->stats_all_pods += committed;
      i += committed;
      inflight = false;
      if (spec) {
        if (!host_work && committed == cur_b) {
          if (!c->dirty_list.empty() || c->prep_stale) {
            drain();
            return fail(c, GS_ESTATE, "speculative batch ran while host rows were pending");
          }
          bind_slot(c, 1 - c->cur_slot);
          cur_b = nb;
          cur_special = false;
          inflight = true;   // (when it is the next run's first batch, i == run.n: the top of the loop moves there)
        } else {
          drain();   // its commit kernel was a no-op
        }
      }
    }
    if ((rc = apply_pending())) return rc;
    return flush_rows(c);
  };
  int rc = body();
  if (rc && pend.active) {   // a batch the device committed: its placements reach the outputs and the host state
    drain();
    (void)apply_pending();
  }
  if (rc) {
    run_done(run, rc);
    if (have_nxt) run_done(nxt, GS_ESTATE);
  }
  return rc;
}

}  // namespace

namespace {
void async_worker(gs_ctx* c) {
  AsyncQueue& q = *c->aq;
  (void)hipSetDevice(c->cfg.device);
  std::unique_lock<std::mutex> lk(q.mu);
  for (;;) {
    q.cv_work.wait(lk, [&] { return q.stop || !q.pending.empty(); });
    if (q.pending.empty()) return;   // stop
    std::shared_ptr<AsyncRun> first = q.pending.front();
    q.pending.pop_front();
    q.busy = true;
    lk.unlock();
    std::vector<std::shared_ptr<AsyncRun>> taken{first};   // keeps the runs alive while the loop reads them
    auto as_run = [](const std::shared_ptr<AsyncRun>& r) {
      PodRun p;
      p.pods = r->pods.data();
      p.seq = r->seq.data();
      p.out = r->out;
      p.n = (uint32_t)r->pods.size();
      p.tag = r.get();
      return p;
    };
    auto next = [&](PodRun* out) -> bool {
      std::lock_guard<std::mutex> g(q.mu);
      if (q.pending.empty()) return false;
      taken.push_back(q.pending.front());
      q.pending.pop_front();
      *out = as_run(taken.back());
      return true;
    };
    auto done = [&](const PodRun& r, int rc) {
      AsyncRun* a = static_cast<AsyncRun*>(r.tag);
      std::lock_guard<std::mutex> g(q.mu);
      a->rc = rc;
      if (rc) a->err = c->err;
      q.cv_done.notify_all();
    };
    const int rc = schedule_stream(c, as_run(first), next, done);
    lk.lock();
    if (rc) {   // an error fails every later submission (the stream's order is broken)
      for (auto& r : q.pending) {
        r->rc = GS_ESTATE;
        r->err = "an earlier gs_schedule_submit failed: " + c->err;
      }
      q.pending.clear();
    }
    q.busy = false;
    q.cv_done.notify_all();
  }
}
}  // namespace

// Every other call on the context waits until the submitted runs are complete (the worker is idle).
int quiesce(gs_ctx* c) {
  if (!c || !c->aq) return GS_OK;
  AsyncQueue& q = *c->aq;
  std::unique_lock<std::mutex> lk(q.mu);
  q.cv_done.wait(lk, [&] { return q.pending.empty() && !q.busy; });
  return GS_OK;
}

void async_stop(gs_ctx* c) {
  if (!c->aq) return;
  quiesce(c);
  {
    std::lock_guard<std::mutex> g(c->aq->mu);
    c->aq->stop = true;
  }
  c->aq->cv_work.notify_all();
  if (c->aq->th.joinable()) c->aq->th.join();
  c->aq.reset();
}

}  // extern "C++"

int gs_schedule(gs_ctx* c, const gs_pod* pods, uint32_t npods, const uint64_t* seq, gs_placement* out) {
  if (!c || (npods && (!pods || !out))) return GS_EINVAL;
  quiesce(c);
  int rc = ready(c);
  if (rc) return rc;
  for (uint32_t i = 0; i < npods; ++i)
    if ((rc = validate_pod(c, pods[i]))) return rc;
  PodRun run;
  run.pods = pods;
  run.seq = seq;
  run.out = out;
  run.n = npods;
  return schedule_stream(c, run, [](PodRun*) { return false; }, [](const PodRun&, int) {});
}

int gs_schedule_submit(gs_ctx* c, const gs_pod* pods, uint32_t npods, const uint64_t* seq, gs_placement* out,
                       uint64_t* ticket) {
  if (!c || !ticket || (npods && (!pods || !out))) return GS_EINVAL;
  auto r = std::make_shared<AsyncRun>();
  // checks that write nothing (the worker may be running): on an error, wait for it, then report
  if (c->n_valid != c->N) {
    quiesce(c);
    if (int rc = ready(c)) return rc;
  }
  char msg[256];
  for (uint32_t i = 0; i < npods; ++i) {
    const int rc = validate_pod_msg(c->numa_on, pods[i], msg, sizeof msg);
    if (rc) {
      quiesce(c);
      return fail(c, rc, "%s", msg);
    }
  }
  r->pods.assign(pods, pods + npods);
  r->seq.resize(npods);
  for (uint32_t i = 0; i < npods; ++i) r->seq[i] = seq ? seq[i] : (uint64_t)i;
  r->out = out;
  if (!c->aq) {
    c->aq = std::make_unique<AsyncQueue>();
    c->aq->th = std::thread(async_worker, c);
  }
  {
    std::lock_guard<std::mutex> g(c->aq->mu);
    r->ticket = c->aq->next_ticket++;
    c->aq->runs[r->ticket] = r;
    c->aq->pending.push_back(r);
  }
  c->aq->cv_work.notify_all();
  *ticket = r->ticket;
  return GS_OK;
}

int gs_schedule_wait(gs_ctx* c, uint64_t ticket) {
  if (!c || !c->aq) return GS_EINVAL;
  AsyncQueue& q = *c->aq;
  std::unique_lock<std::mutex> lk(q.mu);
  auto it = q.runs.find(ticket);
  if (it == q.runs.end()) return GS_EINVAL;
  std::shared_ptr<AsyncRun> r = it->second;
  q.cv_done.wait(lk, [&] { return r->rc != 1; });
  q.runs.erase(it);
  if (r->rc) {
    q.cv_done.wait(lk, [&] { return q.pending.empty() && !q.busy; });   // the worker has stopped writing c->err
    c->err = r->err;
  }
  return r->rc;
}

void gs_numa_args_default(gs_numa_args* a) {
  if (!a) return;
  std::memset(a, 0, sizeof(*a));
  a->default_cpu_bind_policy = GS_CPU_BIND_FULL_PCPUS;   // defaults.go:50,103-106
  a->scoring_type = GS_SCORING_LEAST_ALLOCATED;
  a->numa_scoring_type = GS_SCORING_LEAST_ALLOCATED;
  a->resource_weights[GS_RES_CPU] = 1;
  a->resource_weights[GS_RES_MEMORY] = 1;
}

int gs_topology_register(gs_ctx* c, const gs_cpu_topology* t, int32_t* id) {
  if (!c || !t || !id) return GS_EINVAL;
  quiesce(c);
  const char* err = nullptr;
  auto topo = make_topo(*t, &err);
  if (!topo) return fail(c, GS_EUNSUPPORTED, "gs_topology_register: %s", err ? err : "invalid topology");
  c->topos.push_back(topo);
  *id = (int32_t)c->topos.size() - 1;
  // device copy of every registered topology's TopoDev (index = topology id)
  std::vector<TopoDev> all(c->topos.size());
  for (size_t i = 0; i < all.size(); ++i) all[i] = c->topos[i]->dev;
  HIP_TRY(c, host_wait_stream(c->st));
  if (c->d_topos) { (void)hipFree(c->d_topos); c->d_topos = nullptr; }
  HIP_TRY(c, hipMalloc(&c->d_topos, sizeof(TopoDev) * all.size()));
  HIP_TRY(c, hipMemcpy(c->d_topos, all.data(), sizeof(TopoDev) * all.size(), hipMemcpyHostToDevice));
  return GS_OK;
}

int gs_nodes_numa_upsert(gs_ctx* c, const uint32_t* idx, const gs_node_numa* nn, uint32_t n) {
  if (!c || (!nn && n)) return GS_EINVAL;
  quiesce(c);
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t i = idx ? idx[j] : j;
    if (i >= c->N) return fail(c, GS_EINVAL, "node index %u >= %u", i, c->N);
    const gs_node_numa& x = nn[j];
    if (x.num_zones < 0 || x.num_zones > GS_MAX_NUMA)
      return fail(c, GS_EUNSUPPORTED, "node %u: %d NUMA zones (device path supports <= %d)", i, x.num_zones, GS_MAX_NUMA);
    for (int z = 0; z < x.num_zones; ++z) {
      if (x.zones[z].node_id < 0 || x.zones[z].node_id >= 64 || (z && x.zones[z].node_id <= x.zones[z - 1].node_id))
        return fail(c, GS_EINVAL, "node %u: NUMA zones must be sorted by distinct node id in [0,64)", i);
      if (x.zones[z].cpu_milli < 0 || x.zones[z].memory < 0 || x.zones[z].cpu_milli >= kMaxExact || x.zones[z].memory >= kMaxExact)
        return fail(c, GS_EUNSUPPORTED, "node %u: NUMA zone quantity outside [0, 2^53)", i);
    }
    if (x.numa_topology_policy < 0 || x.numa_topology_policy > 3 || x.node_cpu_bind_policy < 0 ||
        x.node_cpu_bind_policy > 2 || x.numa_allocate_strategy < 0 || x.numa_allocate_strategy > 3)
      return fail(c, GS_EINVAL, "node %u: policy enum out of range", i);
    if (x.has_options && x.topology >= (int32_t)c->topos.size())
      return fail(c, GS_EINVAL, "node %u: topology id %d not registered", i, x.topology);
    NumaNode& st = c->numa[i];
    if (st.cfg.numa_topology_policy != x.numa_topology_policy) c->numa_idx_stale = c->xnuma_stale = true;
    st.cfg = x;
    if (c->devs[i].has_device) dev_mark(c, i);   // its GPUs' zone slots (dev_image)
    st.topo = !x.has_options ? nullptr : (x.topology >= 0 ? c->topos[x.topology] : c->empty_topo);
    mark_dirty(c, i);
  }
  return flush_rows(c);
}

int gs_numa_allocations_update(gs_ctx* c, const uint32_t* node_idx, const gs_pod_allocation* a, uint32_t n) {
  if (!c || (n && (!node_idx || !a))) return GS_EINVAL;
  quiesce(c);
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t i = node_idx[j];
    if (i >= c->N) return fail(c, GS_EINVAL, "node index %u >= %u", i, c->N);
    NumaNode& st = c->numa[i];
    if (!st.topo_valid()) continue;   // resourceManager.Update (resource_manager.go:362-373)
    PodAllocRec rec;
    rec.uid = a[j].uid;
    for (int w = 0; w < GS_CPU_WORDS; ++w) rec.cpus.w[w] = a[j].cpuset[w];
    rec.excl = a[j].cpu_exclusive_policy;
    if (a[j].num_numa < 0 || a[j].num_numa > GS_MAX_NUMA) return fail(c, GS_EINVAL, "num_numa out of range");
    for (int z = 0; z < a[j].num_numa; ++z) rec.numa.push_back(a[j].numa[z]);
    numa_release(st, rec.uid);
    numa_add(st, rec);
    c->numa_uid_node[rec.uid] = i;
    mark_dirty(c, i);
  }
  return flush_rows(c);
}

int gs_numa_allocations_release(gs_ctx* c, const uint32_t* node_idx, const uint64_t* uids, uint32_t n) {
  if (!c || (n && (!node_idx || !uids))) return GS_EINVAL;
  quiesce(c);
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t i = node_idx[j];
    if (i >= c->N) return fail(c, GS_EINVAL, "node index %u >= %u", i, c->N);
    numa_release(c->numa[i], uids[j]);
    auto it = c->numa_uid_node.find(uids[j]);
    if (it != c->numa_uid_node.end() && it->second == i) c->numa_uid_node.erase(it);
    mark_dirty(c, i);
  }
  return flush_rows(c);
}

int gs_numa_allocation_get(gs_ctx* c, uint32_t node, uint64_t uid, gs_pod_allocation* out) {
  if (!c || !out || node >= c->N) return GS_EINVAL;
  quiesce(c);
  const NumaNode& st = c->numa[node];
  auto it = st.pods.find(uid);
  if (it == st.pods.end()) return 0;
  std::memset(out, 0, sizeof(*out));
  out->uid = uid;
  for (int w = 0; w < GS_CPU_WORDS; ++w) out->cpuset[w] = it->second.cpus.w[w];
  out->cpu_exclusive_policy = it->second.excl;
  out->num_numa = (int32_t)std::min<size_t>(it->second.numa.size(), GS_MAX_NUMA);
  for (int z = 0; z < out->num_numa; ++z) out->numa[z] = it->second.numa[z];
  return 1;
}

int gs_comm_unique_id(uint8_t out[128]) {
  if (!out) return GS_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return GS_ECOMM;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out, &id, 128);
  return GS_OK;
}

int gs_comm_init_rccl(gs_ctx* c, const uint8_t id[128], int nranks, int rank) {
  if (!c || !id || nranks < 1 || nranks > MAX_RANKS || rank < 0 || rank >= nranks) return GS_EINVAL;
  quiesce(c);
  // node sampling's rotation window needs every node's Filter verdict on every rank: the score rows carry them
  if (c->window_k && nranks > 1 && xchg_levels())
    return fail(c, GS_EUNSUPPORTED, "node sampling on several ranks needs the score-row exchange");
  if (nranks > 1) {
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    HIP_TRY(c, hipSetDevice(c->cfg.device));
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) return fail(c, GS_ECOMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
  }
  c->nranks = nranks;
  c->rank = rank;
  set_shard(c);
  c->numa_idx_stale = c->xnuma_stale = true;
  return alloc_exchange(c);
}

int gs_comm_init_callback(gs_ctx* c, int nranks, int rank, gs_allgather_fn fn, void* user) {
  if (!c || !fn || nranks < 1 || nranks > MAX_RANKS || rank < 0 || rank >= nranks) return GS_EINVAL;
  quiesce(c);
  // node sampling's rotation window needs every node's Filter verdict on every rank: the score rows carry them
  if (c->window_k && nranks > 1 && xchg_levels())
    return fail(c, GS_EUNSUPPORTED, "node sampling on several ranks needs the score-row exchange");
  c->cb = fn;
  c->cb_user = user;
  c->nranks = nranks;
  c->rank = rank;
  set_shard(c);
  c->numa_idx_stale = c->xnuma_stale = true;
  return alloc_exchange(c);
}

int gs_local_group_create(int nranks, gs_local_group** out) {
  if (!out || nranks < 1 || nranks > MAX_RANKS) return GS_EINVAL;
  gs_local_group* g = new gs_local_group;
  g->n = nranks;
  g->send.assign(nranks, nullptr);
  g->bytes.assign(nranks, 0);
  g->ready.assign(nranks, nullptr);
  g->done.assign(nranks, nullptr);
  *out = g;
  return GS_OK;
}

int gs_local_group_destroy(gs_local_group* g) {
  delete g;
  return GS_OK;
}

int gs_comm_init_local(gs_ctx* c, gs_local_group* g, int rank) {
  if (!c || !g || rank < 0 || rank >= g->n) return GS_EINVAL;
  quiesce(c);
  if (c->window_k && g->n > 1 && xchg_levels())
    return fail(c, GS_EUNSUPPORTED, "node sampling on several ranks needs the score-row exchange");
  HIP_TRY(c, hipSetDevice(c->cfg.device));
  if (!c->lg_ready) HIP_TRY(c, hipEventCreateWithFlags(&c->lg_ready, hipEventDisableTiming));
  if (!c->lg_done) HIP_TRY(c, hipEventCreateWithFlags(&c->lg_done, hipEventDisableTiming));
  c->lg = g;
  c->nranks = g->n;
  c->rank = rank;
  set_shard(c);
  c->numa_idx_stale = c->xnuma_stale = true;
  return alloc_exchange(c);
}

int gs_get_stats(gs_ctx* c, gs_stats* out) {
  if (!c || !out) return GS_EINVAL;
  quiesce(c);
  *out = c->stats;
  out->next_start_node_index = c->next_start;
  return GS_OK;
}

int gs_reset_stats(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  quiesce(c);
  uint64_t rb = c->stats.node_row_bytes;   // keep
  c->stats = gs_stats{};
  c->stats.node_row_bytes = rb;
  c->stats.shard_begin = c->n0;
  c->stats.shard_end = c->n1;
  return GS_OK;
}

int gs_synchronize(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  quiesce(c);
  HIP_TRY(c, host_wait_stream(c->st_ev));
  HIP_TRY(c, host_wait_stream(c->st));
  HIP_TRY(c, host_wait_stream(c->st_rb));
  return GS_OK;
}

// Device-error recovery (a GPU error becomes framework.Error, then the mirror is rebuilt from the
// host snapshot): drain the streams, re-derive every node row from the host state into HBM, re-run node prep.
int gs_reset(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  quiesce(c);
  (void)host_wait_stream(c->st);
  (void)host_wait_stream(c->st_ev);
  (void)host_wait_stream(c->st2);
  (void)host_wait_stream(c->st_rb);
  (void)hipGetLastError();
  for (uint32_t i = 0; i < c->N; ++i)
    if (c->nodes[i].valid) mark_dirty(c, i);
  c->numa_idx_stale = c->xnuma_stale = true;
  if (c->d_dev)
    for (uint32_t i = 0; i < c->N; ++i) dev_mark(c, i);
  int rc = flush_rows(c);
  if (!rc) rc = ext_flush_devices(c);
  if (rc) return rc;
  if ((rc = node_prep(c))) return rc;
  hipError_t e = host_wait_stream(c->st);
  if (e != hipSuccess) return fail(c, GS_EDEVICE, "reset: the device is unusable (%s): destroy and recreate the context",
                                   hipGetErrorString(e));
  c->err.clear();
  return GS_OK;
}

int gs_debug_verify_cpuset(gs_ctx* c, int on) {
  if (!c) return GS_EINVAL;
  quiesce(c);
  c->verify_cpuset = on != 0;
  return GS_OK;
}

// Cycle cost of the commit kernel's pair evaluations on mirror rows (gs_probe.hip): n probes, probe i on node
// nodes[i] with pod pod_of[i] (modes 0, 2) or with pods 0..min(npods,64)-1 one per lane (mode 1).
int gs_debug_pair_probe(gs_ctx* c, const gs_pod* pods, uint32_t npods, const uint32_t* nodes, const int32_t* pod_of,
                        uint32_t n, int mode, int32_t* scores, uint64_t* cycles) {
  if (!c || !pods || !nodes || !pod_of || !scores || !cycles || npods == 0 || npods > 64 || mode < 0 || mode > 2)
    return GS_EINVAL;
  quiesce(c);
  int rc = ready(c);
  if (rc) return rc;
  if ((rc = flush_rows(c))) return rc;
  if (c->prep_stale && (rc = node_prep(c))) return rc;
  for (uint32_t i = 0; i < n; ++i)
    if (nodes[i] >= c->N || pod_of[i] < 0 || (uint32_t)pod_of[i] >= npods) return GS_EINVAL;
  std::vector<PodVec> pv(npods);
  int prod_cols = 0;
  for (uint32_t i = 0; i < npods; ++i) {
    if ((rc = validate_pod(c, pods[i]))) return rc;
    pv[i] = prep_pod(c, pods[i]);
    prod_cols |= (pv[i].flags & PF_PROD_SCORE) ? 1 : 0;
  }
  PodVec* d_p = nullptr;
  uint32_t* d_n = nullptr;
  int32_t *d_o = nullptr, *d_s = nullptr;
  uint64_t* d_c = nullptr;
  const size_t ns = (size_t)n * (mode == 1 ? 64 : 1);
  hipError_t e = hipMalloc(&d_p, sizeof(PodVec) * npods);
  if (e == hipSuccess) e = hipMalloc(&d_n, 4 * n);
  if (e == hipSuccess) e = hipMalloc(&d_o, 4 * n);
  if (e == hipSuccess) e = hipMalloc(&d_s, 4 * ns);
  if (e == hipSuccess) e = hipMalloc(&d_c, 80 * n);
  if (e == hipSuccess) e = hipMemset(d_c, 0, 80 * n);
  if (e == hipSuccess) e = hipMemcpy(d_p, pv.data(), sizeof(PodVec) * npods, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_n, nodes, 4 * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_o, pod_of, 4 * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = host_wait_stream(c->st);
  if (e == hipSuccess) e = launch_probe(mode, c->mv, c->pf, d_p, (int)npods, d_n, d_o, n, prod_cols, d_s, d_c, c->st);
  if (e == hipSuccess) e = host_wait_stream(c->st);
  if (e == hipSuccess) e = hipMemcpy(scores, d_s, 4 * ns, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(cycles, d_c, 80 * n, hipMemcpyDeviceToHost);
  (void)hipFree(d_p); (void)hipFree(d_n); (void)hipFree(d_o); (void)hipFree(d_s); (void)hipFree(d_c);
  if (e != hipSuccess) return fail(c, GS_EDEVICE, "probe: %s", hipGetErrorString(e));
  return GS_OK;
}

// The device merge on given hint lists (gs_probe.hip merge_probe_kernel).
int gs_debug_numa_merge(gs_ctx* c, const gs_merge_case* cases, uint32_t n, gs_merge_result* out) {
  if (!c || (n && (!cases || !out))) return GS_EINVAL;
  quiesce(c);
  for (uint32_t i = 0; i < n; ++i)
    if (cases[i].nz < 1 || cases[i].nz > 4 || cases[i].policy < GS_NUMA_POLICY_NONE ||
        cases[i].policy > GS_NUMA_POLICY_SINGLE_NUMA_NODE)
      return GS_EINVAL;
  if (!n) return GS_OK;   // (no mirror state involved: the merge's inputs are the cases)
  gs_merge_case* d_c = nullptr;
  gs_merge_result* d_o = nullptr;
  hipError_t e = hipMalloc(&d_c, sizeof(gs_merge_case) * n);
  if (e == hipSuccess) e = hipMalloc(&d_o, sizeof(gs_merge_result) * n);
  if (e == hipSuccess) e = hipMemcpy(d_c, cases, sizeof(gs_merge_case) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = host_wait_stream(c->st);
  if (e == hipSuccess) e = launch_merge_probe(d_c, (int)n, d_o, c->st);
  if (e == hipSuccess) e = host_wait_stream(c->st);
  if (e == hipSuccess) e = hipMemcpy(out, d_o, sizeof(gs_merge_result) * n, hipMemcpyDeviceToHost);
  (void)hipFree(d_c);
  (void)hipFree(d_o);
  if (e != hipSuccess) return fail(c, GS_EDEVICE, "merge probe: %s", hipGetErrorString(e));
  return GS_OK;
}

// Compares every HBM mirror row against a fresh host derivation; returns the number of mismatching rows.
int gs_debug_mirror_check(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  quiesce(c);
  int rc = flush_rows(c);
  if (rc) return rc;
  std::vector<int64_t> d64((size_t)c->npad * NUM_I64_COLS);
  std::vector<int32_t> d32((size_t)c->npad * NUM_I32_COLS);
  HIP_TRY(c, host_wait_stream(c->st));
  HIP_TRY(c, hipMemcpy(d64.data(), c->d_i64, d64.size() * 8, hipMemcpyDeviceToHost));
  HIP_TRY(c, hipMemcpy(d32.data(), c->d_i32, d32.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  std::vector<int64_t> row(ROW_WORDS);
  for (uint32_t i = 0; i < c->N; ++i) {
    derive_row(c, i, row.data());
    bool ok = true;
    derive_row_numa(c, i, row.data());
    for (int k = 0; k < NUM_I64_COLS; ++k) ok &= d64[(size_t)k * c->npad + i] == row[k];
    for (int k = 0; k < NUM_I32_COLS; ++k)
      if (k != C_DFLAGS) ok &= d32[(size_t)k * c->npad + i] == (int32_t)row[NUM_I64_COLS + k];
    if (!ok) {
      if (bad < 4) fprintf(stderr, "gpuscore: mirror row %u differs from its host derivation\n", i);
      ++bad;
    }
  }
  return bad;
}

}  // extern "C"

// ---- Reservation + DeviceShare ----------------------------------------------------------------
extern "C" {

void gs_ext_args_default(gs_ext_args* a) {
  if (!a) return;
  std::memset(a, 0, sizeof(*a));
  a->enabled = GS_EXT_DEVICESHARE | GS_EXT_RESERVATION;
  a->device_scoring_type = GS_SCORING_LEAST_ALLOCATED;   // v1beta2 SetDefaults_DeviceShareArgs (defaults.go:187-203)
  a->device_weights[GS_GPU_MEMORY_RATIO] = 1;            // (its rdma weight has no GPU counterpart)
  a->weight_deviceshare = 1;                              // config/manager/scheduler-config.yaml:80-89
  a->weight_reservation = 5000;
}

int gs_ext_configure(gs_ctx* c, const gs_ext_args* a) {
  if (!c || !a) return GS_EINVAL;
  quiesce(c);
  if (a->enabled & ~(GS_EXT_DEVICESHARE | GS_EXT_RESERVATION)) return fail(c, GS_EINVAL, "unknown extension plugin bits");
  if (a->fit_ignored_gpu_names & ~0x1Fu) return fail(c, GS_EINVAL, "fit_ignored_gpu_names outside the GPU names");
  if (a->fit_ignored_xres & ~((1u << GS_MAX_XRES) - 1u))
    return fail(c, GS_EINVAL, "fit_ignored_xres outside the registered extended resources");
  if (a->device_scoring_type != GS_SCORING_LEAST_ALLOCATED && a->device_scoring_type != GS_SCORING_MOST_ALLOCATED)
    return fail(c, GS_EINVAL, "DeviceShare scoring strategy not supported");
  for (int r = 0; r < GS_NUM_GPU_RES; ++r)
    if (a->device_weights[r] < 0 || a->device_weights[r] > 100) return fail(c, GS_EINVAL, "DeviceShare weight out of range");
  if (a->weight_deviceshare < 0 || a->weight_reservation < 0 || a->weight_deviceshare > 100000 ||
      a->weight_reservation > 100000)
    return fail(c, GS_EINVAL, "extension plugin weights out of range");
  const bool rs_changed = (c->ext.enabled ^ a->enabled) & GS_EXT_RESERVATION;
  c->ext = *a;
  if (rs_changed)   // the mirror rows carry the unmatched restore only with the Reservation plugin on
    for (uint32_t i = 0; i < c->N; ++i)
      if (c->nodes[i].valid) mark_dirty(c, i);
  return GS_OK;
}

int gs_node_devices_upsert(gs_ctx* c, const uint32_t* idx, const gs_node_devices* d, uint32_t n) {
  if (!c || (n && !d)) return GS_EINVAL;
  quiesce(c);
  for (uint32_t k = 0; k < n; ++k) {
    const uint32_t i = idx ? idx[k] : k;
    if (i >= c->N) return fail(c, GS_EINVAL, "node index %u out of range", i);
    if (d[k].num_gpus < 0 || d[k].num_gpus > GS_MAX_GPUS) return fail(c, GS_EINVAL, "num_gpus out of range");
    for (int g = 0; g < d[k].num_gpus; ++g) {
      for (int h = 0; h < g; ++h)
        if (d[k].gpus[h].minor == d[k].gpus[g].minor) return fail(c, GS_EINVAL, "duplicate GPU minor on node %u", i);
      if (d[k].gpus[g].minor < 0 || d[k].gpus[g].minor > 31) return fail(c, GS_EUNSUPPORTED, "GPU minor outside 0..31");
      for (int r = 0; r < GS_NUM_GPU_RES; ++r)
        if (d[k].gpus[g].total[r] < 0 || d[k].gpus[g].used[r] < 0 || d[k].gpus[g].total[r] >= (1LL << 53))
          return fail(c, GS_EUNSUPPORTED, "GPU quantity outside [0, 2^53)");
    }
    for (int x = 0; x < GS_MAX_XRES; ++x)
      if (!in_range(d[k].xres_allocatable[x]) || !in_range(d[k].xres_requested[x]))
        return fail(c, GS_EUNSUPPORTED, "extended resource quantity outside the exact range (-2^53, 2^53)");
    c->devs[i] = d[k];
    dev_mark(c, i);
  }
  return GS_OK;
}

int gs_node_devices_get(gs_ctx* c, uint32_t node, gs_node_devices* out) {
  if (!c || !out || node >= c->N) return GS_EINVAL;
  quiesce(c);
  *out = c->devs[node];
  return GS_OK;
}

namespace {
void rsv_unindex(gs_ctx* c, const gs_reservation& r) {
  auto& v = c->rsv_node[r.node];
  v.erase(std::remove(v.begin(), v.end(), r.uid), v.end());
  auto it = c->rsv_owner.find(r.owner_key);
  if (it != c->rsv_owner.end()) {
    auto& o = it->second;
    o.erase(std::remove(o.begin(), o.end(), r.uid), o.end());
    if (o.empty()) c->rsv_owner.erase(it);
  }
  mark_dirty(c, r.node);
}
}  // namespace

int gs_reservations_upsert(gs_ctx* c, const gs_reservation* r, uint32_t n) {
  if (!c || (n && !r)) return GS_EINVAL;
  quiesce(c);
  for (uint32_t k = 0; k < n; ++k) {
    const gs_reservation& x = r[k];
    if (x.node >= c->N) return fail(c, GS_EINVAL, "reservation node %u out of range", x.node);
    if (x.allocate_policy < GS_RSV_POLICY_DEFAULT || x.allocate_policy > GS_RSV_POLICY_RESTRICTED)
      return fail(c, GS_EINVAL, "reservation allocate policy out of range");
    if ((x.allocatable_mask | x.allocated_mask | x.resource_names_mask) & ~0x7Fu)
      return fail(c, GS_EINVAL, "reservation resource keys outside slots 0..6");
    for (int s = 0; s < GS_NUM_RES; ++s)
      if (x.allocatable[s] < 0 || x.allocated[s] < 0 || x.allocatable[s] >= (1LL << 50) || x.allocated[s] >= (1LL << 50))
        return fail(c, GS_EUNSUPPORTED, "reservation quantity outside [0, 2^50)");
    auto it = c->rsv.find(x.uid);
    if (it != c->rsv.end()) rsv_unindex(c, it->second);
    c->rsv[x.uid] = x;
    auto& v = c->rsv_node[x.node];
    v.insert(std::lower_bound(v.begin(), v.end(), x.uid), x.uid);
    if (x.owner_key) {
      auto& o = c->rsv_owner[x.owner_key];
      o.insert(std::lower_bound(o.begin(), o.end(), x.uid), x.uid);
    }
    mark_dirty(c, x.node);
  }
  return GS_OK;
}

int gs_reservations_remove(gs_ctx* c, const uint64_t* uids, uint32_t n) {
  if (!c || (n && !uids)) return GS_EINVAL;
  quiesce(c);
  for (uint32_t k = 0; k < n; ++k) {
    auto it = c->rsv.find(uids[k]);
    if (it == c->rsv.end()) continue;
    rsv_unindex(c, it->second);
    c->rsv.erase(it);
  }
  return GS_OK;
}

int gs_reservation_get(gs_ctx* c, uint64_t uid, gs_reservation* out) {
  if (!c || !out) return GS_EINVAL;
  quiesce(c);
  auto it = c->rsv.find(uid);
  if (it == c->rsv.end()) return 0;
  *out = it->second;
  return 1;
}

int gs_schedule_ext(gs_ctx* c, const gs_pod* pods, const gs_pod_ext* ext, uint32_t npods, const uint64_t* seq,
                    gs_placement* out, gs_ext_placement* ext_out) {
  if (!c || (npods && (!pods || !out))) return GS_EINVAL;
  quiesce(c);
  int rc = ready(c);
  if (rc) return rc;
  for (uint32_t i = 0; i < npods; ++i)
    if ((rc = validate_pod(c, pods[i]))) return rc;
  uint32_t i = 0;
  while (i < npods) {
    // a run of plain pods goes through the batched path (both plugins score 0 for them; the mirror rows carry the
    // unmatched restore), an extension pod through the normalizing path
    uint32_t j = i;
    while (j < npods && !(ext && (c->ext.enabled || ext[j].xres_request_mask) && is_ext_pod(c, ext[j]))) ++j;
    if (j > i) {
      std::vector<uint64_t> sq;
      if (!seq) { sq.resize(j - i); for (uint32_t k = i; k < j; ++k) sq[k - i] = k; }
      const auto hp0 = std::chrono::steady_clock::now();
      if ((rc = gs_schedule(c, pods + i, j - i, seq ? seq + i : sq.data(), out + i))) return rc;
      if (c->host_timing) {
        c->hx_plain += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - hp0).count();
        c->hx_runs += 1;
      }
      if (ext_out) std::memset(ext_out + i, 0, sizeof(gs_ext_placement) * (j - i));
      i = j;
      continue;
    }
    gs_ext_placement eo{};
    if ((rc = ext_schedule_one(c, pods[i], ext[i], seq ? seq[i] : i, &out[i], &eo))) return rc;
    if (ext_out) ext_out[i] = eo;
    ++i;
  }
  rc = flush_rows(c);
  if (!rc) rc = ext_flush_devices(c);
  return rc;
}

}  // extern "C"
