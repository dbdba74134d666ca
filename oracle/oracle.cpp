// oracle.cpp — CPU restatement of the reference Filter/Score path. TEST INFRASTRUCTURE ONLY
// (see oracle.h). Reference paths are relative to hormes/koordinator; "[upstream]" marks
// k8s.io/kubernetes@v1.24.15 code (go.mod:57,276), not vendored in /root/reference, restated
// from its published source — parity for those parts is unpinned by in-repo tests.
#include "oracle.h"
#include "numa.h"

#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <algorithm>
#include <mutex>
#include <chrono>
#include <thread>
#include <vector>

namespace {

constexpr int64_t kMaxNodeScore = 100;                       // [upstream] framework.MaxNodeScore
constexpr int64_t kDefaultMilliCPURequest = 250;             // estimator/default_estimator.go:36
constexpr int64_t kDefaultMemoryRequest = 200 * 1024 * 1024; // estimator/default_estimator.go:38
constexpr int64_t kDefaultReportIntervalNs = 60LL * 1000000000LL; // loadaware/load_aware.go:56
constexpr int64_t kZeroTime = INT64_MIN;                     // Go time.Time{} (UpdateTime == nil)

// A corev1.ResourceList restricted to {cpu, memory} (+ "some other key" for len()).
struct ResList {
  int64_t v[2] = {0, 0};
  uint32_t mask = 0;
  bool has(int r) const { return mask & (1u << r); }
  bool empty() const { return mask == 0; }
  int64_t get(int r) const { return has(r) ? v[r] : 0; }
  void add(int r, int64_t x) { v[r] = get(r) + x; mask |= (1u << r); }
};

ResList from_usage(const gs_usage& u) {
  ResList l;
  if (u.mask & GS_USAGE_CPU) { l.v[0] = u.cpu_milli; l.mask |= 1; }
  if (u.mask & GS_USAGE_MEMORY) { l.v[1] = u.memory; l.mask |= 2; }
  if (u.mask & GS_USAGE_OTHER) l.mask |= GS_USAGE_OTHER;
  return l;
}

// Quantity.MilliValue() of the slot value (cpu is stored in milli, memory in units).
int64_t milli_value(int r, int64_t v) { return r == 0 ? v : v * 1000; }

struct AssignInfo {
  int64_t timestamp;
  gs_pod pod;
};

struct PodMetric {
  uint64_t name_key;
  int32_t in_lister, priority_class;
  ResList usage;
};

struct NodeState {
  gs_node node{};
  bool has_node = false;
  gs_node_metric metric{};
  std::vector<PodMetric> pods_metric;
  std::map<uint64_t, AssignInfo> assigned;   // podAssignCache.podInfoItems[node] (pod_assign_cache.go:39)
};

// ---------------------------------------------------------------------------------------------
// selectHost tie-break stream.
// [upstream] schedule_one.go selectHost draws rand.Intn(cntOfMaxScore) from Go's global math/rand,
// seeded by wall clock (cmd/koord-scheduler/main.go:61); that stream cannot be reproduced offline
// (SURVEY.md §7.3). The replacement keeps selectHost's reservoir loop verbatim and draws Intn(cnt)
// from a stream keyed by (seed, pod seq): Intn(cnt) == 0 iff cnt is in the replacement set
// R = {j_1 = 1, j_{i+1} = floor(j_i / U_i) + 1}, U_i in (0,1] from splitmix64(seed, seq, i).
// P(next replacement > m | replacement at j) = j/m, exactly the law of independent
// Bernoulli(1/cnt) events, so the selected node is uniform over the final max ties.
uint64_t mix64(uint64_t x) {
  uint64_t z = x + 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

struct TieBreakRand {
  uint64_t key;
  int64_t cur = 1;      // last replacement position generated
  uint64_t i = 0;
  TieBreakRand(uint64_t seed, uint64_t seq) : key(mix64(seed ^ mix64(seq))) {}
  int64_t next_after(int64_t j) {
    uint64_t h = mix64(key + i);
    ++i;
    double u = (double)((h >> 11) + 1) * 0x1.0p-53;   // (0, 1]
    double x = (double)j / u;
    if (!(x < 4.0e18)) return INT64_MAX;
    return (int64_t)std::floor(x) + 1;
  }
  // Intn(cnt) for cnt = 2, 3, ... called in increasing order within one max run
  // (the set R does not depend on the run, so restarting runs reuse it).
  std::vector<int64_t> R{1};
  int32_t intn(int64_t cnt) {
    while (R.back() < cnt) R.push_back(next_after(R.back()));
    for (int64_t v : R)
      if (v == cnt) return 0;
    return 1;
  }
};

}  // namespace

struct or_cluster {
  gs_config cfg;
  int64_t now = 0;
  std::vector<NodeState> nodes;
  // NodeNUMAResource (oracle/numa.cpp)
  orn::NumaArgs numa_args;
  std::vector<std::shared_ptr<orn::CPUTopology>> topologies;
  std::vector<orn::NodeNUMA> numa;
  bool reverse_hint_order = false;
  uint32_t next_start = 0;   // [upstream] Scheduler.nextStartNodeIndex
  double phase_s[4] = {0, 0, 0, 0};   // or_phase_times
  // Reservation + DeviceShare (the "extension plugins" section at the end of this file)
  gs_ext_args ext{};
  std::map<uint64_t, gs_reservation> reservations;   // reservationCache, by uid (reservation/cache.go)
  std::vector<gs_node_devices> devices;               // nodeDeviceCache (has_device == 0: no Device object)
};

namespace {

// ---- loadaware/estimator/default_estimator.go ------------------------------------------------

// extension.TranslateResourceNameByPriorityClass (apis/extension/resource.go:43-48); -1 = "".
int translate_resource(int32_t prio, int r) {
  if (prio == GS_PRIO_PROD || prio == GS_PRIO_NONE) return r;
  if (prio == GS_PRIO_BATCH) return r == 0 ? GS_RES_BATCH_CPU : GS_RES_BATCH_MEMORY;
  if (prio == GS_PRIO_MID) return r == 0 ? GS_RES_MID_CPU : GS_RES_MID_MEMORY;
  return -1;  // PriorityFree has no ResourceNameMap entry
}

// estimatedUsedByResource (default_estimator.go:73-108)
int64_t estimated_used_by_resource(const gs_pod& pod, int real, int64_t scaling_factor) {
  int64_t limit = real >= 0 ? pod.limits[real] : 0;
  int64_t request = real >= 0 ? pod.requests[real] : 0;
  int64_t quantity;
  if (limit > request) {            // limitQuantity.Cmp(requestQuantity) > 0
    scaling_factor = 100;
    quantity = limit;
  } else {
    quantity = request;
  }
  if (quantity == 0) {
    if (real == GS_RES_CPU || real == GS_RES_BATCH_CPU) return kDefaultMilliCPURequest;
    if (real == GS_RES_MEMORY || real == GS_RES_BATCH_MEMORY) return kDefaultMemoryRequest;
    return 0;
  }
  // cpu: MilliValue; everything else Value — both are the slot's stored unit.
  int64_t est = (int64_t)std::round((double)quantity * (double)scaling_factor / 100);
  if (limit > 0 && est > limit) est = limit;
  return est;
}

// estimatedPodUsed (default_estimator.go:61-70): keys = ResourceWeights keys
ResList estimate_pod(const gs_loadaware_args& a, const gs_pod& pod) {
  ResList out;
  for (int r = 0; r < 2; ++r) {
    if (!(a.resource_weights_mask & (1u << r))) continue;
    int real = translate_resource(pod.priority_class, r);
    int64_t sf = (a.estimated_scaling_factors_mask & (1u << r)) ? a.estimated_scaling_factors[r] : 0;
    out.add(r, estimated_used_by_resource(pod, real, sf));
  }
  return out;
}

// EstimateNode (default_estimator.go:110-129): Allocatable with raw-allocatable keys overriding.
int64_t estimate_node(const gs_node& n, int r) {
  if (n.raw_allocatable_mask & (1u << r)) return n.raw_allocatable[r];
  return n.allocatable[r];
}

// ---- loadaware/helper.go ---------------------------------------------------------------------

// isNodeMetricExpired (helper.go:36-41)
bool is_node_metric_expired(const NodeState& s, int64_t expiration_s, int64_t now) {
  if (!s.metric.exists || !s.metric.has_update_time) return true;
  return expiration_s > 0 && (now - s.metric.update_time_ns) >= expiration_s * 1000000000LL;
}

// getNodeMetricReportInterval (helper.go:43-48)
int64_t report_interval_ns(const gs_node_metric& m) {
  return m.has_report_interval ? m.report_interval_s * 1000000000LL : kDefaultReportIntervalNs;
}

// getTargetAggregatedUsage (helper.go:58-90); duration_ns == 0 stands for nil or 0.
bool target_aggregated_usage(const gs_node_metric& m, int64_t duration_ns, int32_t type, ResList* out) {
  if (!m.has_node_metric || m.n_aggregated == 0) return false;
  if (type < 0 || type >= GS_NUM_AGG_TYPES) return false;   // Usage[""] is an empty ResourceMap
  if (duration_ns == 0) {
    int64_t max_d = 0;
    int max_i = 0;
    for (int i = 0; i < m.n_aggregated; ++i)
      if (m.aggregated[i].duration_ns > max_d) { max_d = m.aggregated[i].duration_ns; max_i = i; }
    const gs_agg_usage& a = m.aggregated[max_i];
    if (a.type_mask & (1u << type)) {
      ResList l = from_usage(a.usage[type]);
      if (!l.empty()) { *out = l; return true; }
    }
  } else {
    for (int i = 0; i < m.n_aggregated; ++i) {
      const gs_agg_usage& a = m.aggregated[i];
      if (a.duration_ns == duration_ns && (a.type_mask & (1u << type))) {
        ResList l = from_usage(a.usage[type]);
        if (!l.empty()) { *out = l; return true; }
      }
    }
  }
  return false;
}

// filterWithAggregation / scoreWithAggregation (helper.go:92-98)
bool filter_with_aggregation(const gs_loadaware_args& a) {
  return a.has_aggregated && a.agg_usage_thresholds_mask != 0 && a.agg_usage_type != GS_AGG_NONE;
}
bool score_with_aggregation(const gs_loadaware_args& a) {
  return a.has_aggregated && a.agg_score_type != GS_AGG_NONE;
}

struct Thresholds {
  int64_t v[2] = {0, 0};
  uint32_t mask = 0;
};
struct FilterProfile {   // extension.CustomUsageThresholds
  Thresholds usage, prod;
  bool has_agg = false;
  Thresholds agg;
  int32_t agg_type = GS_AGG_NONE;
  int64_t agg_duration_ns = 0;
};

// generateUsageThresholdsFilterProfile (helper.go:102-140). A missing or unparsable annotation
// (GetCustomUsageThresholds error) both end in the args-only profile.
FilterProfile filter_profile(const gs_node& n, const gs_loadaware_args& a) {
  FilterProfile p;
  Thresholds args_usage{{a.usage_thresholds[0], a.usage_thresholds[1]}, a.usage_thresholds_mask};
  Thresholds args_prod{{a.prod_usage_thresholds[0], a.prod_usage_thresholds[1]}, a.prod_usage_thresholds_mask};
  bool custom = n.custom_flags & GS_NODE_CUSTOM_THRESHOLDS;
  if (custom) {
    p.usage = {{n.custom_usage_thresholds[0], n.custom_usage_thresholds[1]}, n.custom_usage_mask};
    p.prod = {{n.custom_prod_usage_thresholds[0], n.custom_prod_usage_thresholds[1]}, n.custom_prod_usage_mask};
    if (n.custom_flags & GS_NODE_CUSTOM_AGGREGATED) {
      p.has_agg = true;
      p.agg = {{n.custom_agg_usage_thresholds[0], n.custom_agg_usage_thresholds[1]}, n.custom_agg_usage_mask};
      p.agg_type = n.custom_agg_type;
      p.agg_duration_ns = n.custom_agg_duration_ns;
    }
  }
  if (p.usage.mask == 0) p.usage = args_usage;
  if (p.prod.mask == 0) p.prod = args_prod;
  if (p.has_agg && (p.agg.mask == 0 || p.agg_type == GS_AGG_NONE)) p.has_agg = false;
  if (!p.has_agg && filter_with_aggregation(a)) {
    p.has_agg = true;
    p.agg = {{a.agg_usage_thresholds[0], a.agg_usage_thresholds[1]}, a.agg_usage_thresholds_mask};
    p.agg_type = a.agg_usage_type;
    p.agg_duration_ns = a.agg_usage_duration_ns;
  }
  return p;
}

// buildPodMetricMap (helper.go:153-170): name -> usage (later duplicates overwrite)
std::map<uint64_t, ResList> build_pod_metric_map(const NodeState& s, bool filter_prod) {
  std::map<uint64_t, ResList> m;
  for (const PodMetric& pm : s.pods_metric) {
    if (!pm.in_lister) continue;
    if (filter_prod && pm.priority_class != GS_PRIO_PROD) continue;
    m[pm.name_key] = pm.usage;
  }
  return m;
}

// sumPodUsages (helper.go:172-186)
void sum_pod_usages(const std::map<uint64_t, ResList>& pm, const std::map<uint64_t, bool>* estimated,
                    ResList* pod_usages, ResList* estimated_usages) {
  for (const auto& kv : pm) {
    bool is_est = estimated && estimated->count(kv.first);
    ResList* dst = is_est ? estimated_usages : pod_usages;
    for (int r = 0; r < 2; ++r)
      if (kv.second.has(r)) dst->add(r, kv.second.v[r]);
  }
}

// leastRequestedScore (load_aware.go:388-397) == [upstream] noderesources leastRequestedScore
int64_t least_requested_score(int64_t requested, int64_t capacity) {
  if (capacity == 0) return 0;
  if (requested > capacity) return 0;
  return ((capacity - requested) * kMaxNodeScore) / capacity;
}

// ---- loadaware/load_aware.go -----------------------------------------------------------------

// filterNodeUsage (load_aware.go:173-224); returns 0 or the GS_FAIL_LOADAWARE code with the reason's details
// (the resource named in "node(s) %s usage exceed threshold", the aggregated form); resources are visited in
// the fixed order cpu, memory (the reference ranges over a Go map: with both over, the named one is unpinned)
uint32_t filter_node_usage(const NodeState& s, const FilterProfile& p) {
  if (!s.metric.has_node_metric) return 0;
  const Thresholds& th = p.has_agg ? p.agg : p.usage;
  for (int r = 0; r < 2; ++r) {
    if (!(th.mask & (1u << r))) continue;
    int64_t threshold = th.v[r];
    if (threshold == 0) continue;
    int64_t total = estimate_node(s.node, r);
    if (total == 0) continue;
    ResList usage;
    if (p.has_agg) {
      if (!target_aggregated_usage(s.metric, p.agg_duration_ns, p.agg_type, &usage)) continue;
    } else {
      usage = from_usage(s.metric.node_usage);
    }
    int64_t used = usage.get(r);
    int64_t pct = (int64_t)std::round((double)milli_value(r, used) / (double)milli_value(r, total) * 100);
    if (pct >= threshold)
      return GS_FAIL_LOADAWARE | (r == 1 ? GS_FAIL_LA_MEMORY : 0u) | (p.has_agg ? GS_FAIL_LA_AGGREGATED : 0u);
  }
  return 0;
}

// filterProdUsage (load_aware.go:226-254)
uint32_t filter_prod_usage(const NodeState& s, const Thresholds& prod) {
  if (s.pods_metric.empty()) return 0;
  auto pm = build_pod_metric_map(s, true);
  ResList prod_usages, unused;
  sum_pod_usages(pm, nullptr, &prod_usages, &unused);
  for (int r = 0; r < 2; ++r) {
    if (!(prod.mask & (1u << r))) continue;
    int64_t threshold = prod.v[r];
    if (threshold == 0) continue;
    int64_t total = estimate_node(s.node, r);
    if (total == 0) continue;
    int64_t used = prod_usages.get(r);
    int64_t pct = (int64_t)std::round((double)milli_value(r, used) / (double)milli_value(r, total) * 100);
    if (pct >= threshold) return GS_FAIL_LOADAWARE | (r == 1 ? GS_FAIL_LA_MEMORY : 0u);
  }
  return 0;
}

// Plugin.Filter (load_aware.go:123-171); 0 or the GS_FAIL_LOADAWARE code (Unschedulable) with its details
uint32_t loadaware_filter(const or_cluster& c, const gs_pod& pod, const NodeState& s) {
  const gs_loadaware_args& a = c.cfg.loadaware;
  if (pod.flags & GS_POD_DAEMONSET) return 0;
  if (!s.metric.exists) return 0;  // NotFound: skip the node (load_aware.go:138-140)
  if (a.filter_expired_node_metrics && a.has_node_metric_expiration &&
      is_node_metric_expired(s, a.node_metric_expiration_seconds, c.now))
    return 0;
  FilterProfile p = filter_profile(s.node, a);
  if (p.prod.mask != 0 && pod.priority_class == GS_PRIO_PROD) return filter_prod_usage(s, p.prod);
  const Thresholds& th = p.has_agg ? p.agg : p.usage;
  if (th.mask != 0) return filter_node_usage(s, p);
  return 0;
}

// estimatedAssignedPodUsed (load_aware.go:337-376)
ResList estimated_assigned_pod_used(const or_cluster& c, const NodeState& s,
                                    const std::map<uint64_t, ResList>& pod_metrics, bool filter_prod,
                                    std::map<uint64_t, bool>* estimated_pods) {
  const gs_loadaware_args& a = c.cfg.loadaware;
  ResList used;
  int64_t update_time = s.metric.has_update_time ? s.metric.update_time_ns : kZeroTime;
  int64_t interval = report_interval_ns(s.metric);
  bool agg_missing = false;
  if (score_with_aggregation(a)) {
    ResList tmp;
    agg_missing = !target_aggregated_usage(s.metric, a.agg_score_duration_ns, a.agg_score_type, &tmp);
  }
  for (const auto& kv : s.assigned) {
    const AssignInfo& info = kv.second;
    if (filter_prod && info.pod.priority_class != GS_PRIO_PROD) continue;
    auto it = pod_metrics.find(info.pod.name_key);
    ResList pod_usage;
    if (it != pod_metrics.end()) pod_usage = it->second;
    bool missed_latest = info.timestamp > update_time;                         // helper.go:50-52
    bool in_interval = info.timestamp < update_time && update_time - info.timestamp < interval;  // :54-56
    if (pod_usage.empty() || missed_latest || in_interval || agg_missing) {
      ResList est = estimate_pod(a, info.pod);
      for (int r = 0; r < 2; ++r) {
        if (!est.has(r)) continue;
        int64_t value = est.v[r];
        if (pod_usage.has(r) && pod_usage.v[r] > value) value = pod_usage.v[r];
        used.add(r, value);
      }
      (*estimated_pods)[info.pod.name_key] = true;
    }
  }
  return used;
}

// loadAwareSchedulingScorer (load_aware.go:378-386)
int64_t loadaware_scorer(const gs_loadaware_args& a, const ResList& used, const gs_node& n) {
  int64_t node_score = 0, weight_sum = 0;
  for (int r = 0; r < 2; ++r) {
    if (!(a.resource_weights_mask & (1u << r))) continue;
    int64_t w = a.resource_weights[r];
    node_score += least_requested_score(used.get(r), estimate_node(n, r)) * w;
    weight_sum += w;
  }
  return node_score / weight_sum;
}

// Plugin.Score (load_aware.go:269-335)
int64_t loadaware_score(const or_cluster& c, const gs_pod& pod, const NodeState& s) {
  const gs_loadaware_args& a = c.cfg.loadaware;
  if (!s.metric.exists) return 0;
  if (a.has_node_metric_expiration && is_node_metric_expired(s, a.node_metric_expiration_seconds, c.now)) return 0;
  bool prod_pod = pod.priority_class == GS_PRIO_PROD && a.score_according_prod_usage;
  auto pod_metrics = build_pod_metric_map(s, prod_pod);
  ResList estimated_used = estimate_pod(a, pod);
  std::map<uint64_t, bool> estimated_pods;
  ResList assigned = estimated_assigned_pod_used(c, s, pod_metrics, prod_pod, &estimated_pods);
  for (int r = 0; r < 2; ++r)
    if (assigned.has(r)) estimated_used.add(r, assigned.v[r]);
  ResList pod_actual, est_pod_actual;
  if (!pod_metrics.empty()) sum_pod_usages(pod_metrics, &estimated_pods, &pod_actual, &est_pod_actual);
  if (prod_pod) {
    for (int r = 0; r < 2; ++r)
      if (pod_actual.has(r)) estimated_used.add(r, pod_actual.v[r]);
  } else if (s.metric.has_node_metric) {
    ResList node_usage;
    bool have;
    if (score_with_aggregation(a)) {
      have = target_aggregated_usage(s.metric, a.agg_score_duration_ns, a.agg_score_type, &node_usage);
    } else {
      node_usage = from_usage(s.metric.node_usage);
      have = true;
    }
    if (have) {
      for (int r = 0; r < 2; ++r) {
        if (!node_usage.has(r)) continue;
        int64_t q = node_usage.v[r];
        int64_t e = est_pod_actual.get(r);
        if (e != 0 && q >= e) q -= e;
        estimated_used.add(r, q);
      }
    }
  }
  return loadaware_scorer(a, estimated_used, s.node);
}

// ---- [upstream] noderesources/fit.go fitsRequest ----------------------------------------------
uint32_t fit_filter(const gs_pod& pod, const gs_node& n) {
  uint32_t fail = 0;
  if (n.pod_count + 1 > n.allowed_pod_number) fail |= GS_FAIL_FIT_PODS;
  uint32_t scalar_keys = pod.request_mask & GS_SCALAR_RES_MASK;
  if (pod.requests[GS_RES_CPU] == 0 && pod.requests[GS_RES_MEMORY] == 0 && pod.requests[GS_RES_EPHEMERAL] == 0 &&
      scalar_keys == 0)
    return fail;
  if (pod.requests[GS_RES_CPU] > n.allocatable[GS_RES_CPU] - n.requested[GS_RES_CPU]) fail |= GS_FAIL_FIT_CPU;
  if (pod.requests[GS_RES_MEMORY] > n.allocatable[GS_RES_MEMORY] - n.requested[GS_RES_MEMORY]) fail |= GS_FAIL_FIT_MEMORY;
  if (pod.requests[GS_RES_EPHEMERAL] > n.allocatable[GS_RES_EPHEMERAL] - n.requested[GS_RES_EPHEMERAL])
    fail |= GS_FAIL_FIT_EPHEMERAL;
  for (int r = 0; r < GS_NUM_RES; ++r) {
    if (!(scalar_keys & (1u << r))) continue;
    if (pod.requests[r] > n.allocatable[r] - n.requested[r]) fail |= GS_FAIL_FIT_SCALAR;
  }
  return fail;
}

// ---- [upstream] noderesources/resource_allocation.go + least_allocated.go (LeastAllocated) ----
int64_t fit_score(const gs_fit_args& f, const gs_pod& pod, const gs_node& n) {
  int64_t node_score = 0, weight_sum = 0;
  for (int r = 0; r < GS_NUM_RES; ++r) {
    int64_t w = f.resource_weights[r];
    if (w == 0) continue;
    // calculatePodResourceRequest: non-zero defaults for cpu/memory (LeastAllocated: useRequested=false)
    int64_t pod_request = (r == GS_RES_CPU || r == GS_RES_MEMORY) ? pod.nonzero_requests[r] : pod.requests[r];
    bool scalar = GS_SCALAR_RES_MASK & (1u << r);
    if (pod_request == 0 && scalar) continue;                  // bypass un-requested extended resources
    int64_t alloc, req;
    if (r == GS_RES_CPU || r == GS_RES_MEMORY) {
      alloc = n.allocatable[r];
      req = n.nonzero_requested[r] + pod_request;
    } else {
      alloc = n.allocatable[r];
      req = n.requested[r] + pod_request;
    }
    if (alloc == 0) continue;                                   // only non-zero allocatable is scored
    node_score += least_requested_score(req, alloc) * w;
    weight_sum += w;
  }
  if (weight_sum == 0) return 0;
  return node_score / weight_sum;
}

struct PairResult {
  uint16_t code;
  int64_t fit, la, numa;
};

orn::NodeView node_view(const gs_node& n) {
  return orn::NodeView{n.allocatable[GS_RES_CPU], n.allocatable[GS_RES_MEMORY], n.requested[GS_RES_CPU],
                       n.requested[GS_RES_MEMORY], n.allocatable, n.requested};
}

// NodeNUMAResource Filter of one (pod, node) pair: reason bits + the affinity Admit stored for Score/Reserve
uint16_t numa_filter(const or_cluster& c, const orn::PreState& st, uint32_t i, orn::Hint* aff) {
  bool has = false;
  int reason = orn::filter(c.numa_args, st, c.numa[i], node_view(c.nodes[i].node), aff, &has, c.reverse_hint_order);
  if (!has) *aff = orn::Hint{};
  return (uint16_t)(reason << GS_FAIL_NUMA_SHIFT);
}

PairResult eval_pair(const or_cluster& c, const gs_pod& pod, const orn::PreState& st, uint32_t i) {
  const NodeState& s = c.nodes[i];
  PairResult res{0, 0, 0, 0};
  uint32_t en = c.cfg.enabled;
  if (en & GS_ENABLE_FIT_FILTER) res.code |= (uint16_t)fit_filter(pod, s.node);
  if (en & GS_ENABLE_LA_FILTER) res.code |= loadaware_filter(c, pod, s);
  orn::Hint aff;
  if (en & GS_ENABLE_NUMA_FILTER) res.code |= numa_filter(c, st, i, &aff);
  if (en & GS_ENABLE_FIT_SCORE) res.fit = fit_score(c.cfg.fit, pod, s.node);
  if (en & GS_ENABLE_LA_SCORE) res.la = loadaware_score(c, pod, s);
  // gs_evaluate reports NodeNUMAResource's score as 0 where its own Filter fails (such nodes are never scored)
  if ((en & GS_ENABLE_NUMA_SCORE) && !(res.code & GS_FAIL_NUMA_MASK))
    res.numa = orn::score(c.numa_args, st, c.numa[i], node_view(s.node), aff);
  return res;
}

int64_t weighted_total(const or_cluster& c, const PairResult& r) {
  int64_t t = 0;
  if (c.cfg.enabled & GS_ENABLE_FIT_SCORE) t += r.fit * c.cfg.plugin_weights[GS_PLUGIN_FIT];
  if (c.cfg.enabled & GS_ENABLE_LA_SCORE) t += r.la * c.cfg.plugin_weights[GS_PLUGIN_LOADAWARE];
  if (c.cfg.enabled & GS_ENABLE_NUMA_SCORE) t += r.numa * c.cfg.plugin_weights[GS_PLUGIN_NUMA];
  return t;
}

orn::NumaArgs numa_args_of(const gs_numa_args& a) {
  orn::NumaArgs o;
  o.default_bind = a.default_cpu_bind_policy;
  o.scoring = a.scoring_type;
  o.numa_scoring = a.numa_scoring_type;
  for (int r = 0; r < GS_NUM_RES; ++r) o.weights[r] = a.resource_weights[r];
  return o;
}

orn::PodAllocation pod_allocation_of(const gs_pod_allocation& a) {
  orn::PodAllocation p;
  p.uid = a.uid;
  for (int c = 0; c < GS_MAX_CPUS; ++c)
    if (a.cpuset[c >> 6] >> (c & 63) & 1) p.cpus.insert(c);
  p.excl = a.cpu_exclusive_policy;
  for (int j = 0; j < a.num_numa && j < GS_MAX_NUMA; ++j) {
    orn::NUMANodeResource nr;
    nr.node = a.numa[j].node_id;
    if (a.numa[j].mask & GS_USAGE_CPU) nr.res.set(GS_RES_CPU, a.numa[j].cpu_milli);
    if (a.numa[j].mask & GS_USAGE_MEMORY) nr.res.set(GS_RES_MEMORY, a.numa[j].memory);
    p.numa.push_back(nr);
  }
  return p;
}

void export_allocation(const orn::PodAllocation& p, gs_pod_allocation* out) {
  std::memset(out, 0, sizeof(*out));
  out->uid = p.uid;
  for (int c : p.cpus) out->cpuset[c >> 6] |= 1ull << (c & 63);
  out->cpu_exclusive_policy = p.excl;
  out->num_numa = (int32_t)std::min<size_t>(p.numa.size(), GS_MAX_NUMA);
  for (int j = 0; j < out->num_numa; ++j) {
    out->numa[j].node_id = p.numa[j].node;
    if (p.numa[j].res.has(GS_RES_CPU)) { out->numa[j].mask |= GS_USAGE_CPU; out->numa[j].cpu_milli = p.numa[j].res.v[GS_RES_CPU]; }
    if (p.numa[j].res.has(GS_RES_MEMORY)) { out->numa[j].mask |= GS_USAGE_MEMORY; out->numa[j].memory = p.numa[j].res.v[GS_RES_MEMORY]; }
  }
}

// ---- parallelize.Until emulation (pkg/util/parallelize/parallelism.go:29-49) ------------------
class Pool {
 public:
  explicit Pool(int n) : n_(n) {
    for (int i = 0; i < n_; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    { std::lock_guard<std::mutex> g(mu_); stop_ = true; }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // Until(pieces, doWorkPiece) with chunkSize = max(1, min(sqrt(pieces), pieces/workers+1))
  void until(int pieces, const std::function<void(int)>& fn) {
    int chunk = std::max(1, std::min((int)std::sqrt((double)pieces), pieces / n_ + 1));
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn; pieces_ = pieces; chunk_ = chunk; next_.store(0); active_ = n_; ++gen_;
    }
    cv_.notify_all();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return active_ == 0; });
  }
 private:
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void(int)>* fn = fn_;
      int pieces = pieces_, chunk = chunk_;
      lk.unlock();
      for (;;) {
        int b = next_.fetch_add(chunk);
        if (b >= pieces) break;
        int e = std::min(pieces, b + chunk);
        for (int i = b; i < e; ++i) (*fn)(i);
      }
      lk.lock();
      if (--active_ == 0) done_cv_.notify_all();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int pieces_ = 0, chunk_ = 1, active_ = 0;
  std::atomic<int> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

bool valid_node(const or_cluster* c, uint32_t i) { return c && i < c->nodes.size() && c->nodes[i].has_node; }

}  // namespace

extern "C" {

or_cluster* or_create(const gs_config* cfg) {
  if (!cfg) return nullptr;
  or_cluster* c = new or_cluster();
  c->cfg = *cfg;
  c->nodes.resize(cfg->num_nodes);
  c->numa.resize(cfg->num_nodes);
  c->numa_args = numa_args_of(cfg->numa);
  c->devices.resize(cfg->num_nodes);
  std::memset(c->devices.data(), 0, sizeof(gs_node_devices) * c->devices.size());
  return c;
}

void or_destroy(or_cluster* c) { delete c; }

int or_set_now(or_cluster* c, int64_t now_ns) {
  if (!c) return GS_EINVAL;
  c->now = now_ns;
  return GS_OK;
}

int or_nodes_upsert(or_cluster* c, const uint32_t* idx, const gs_node* nodes, uint32_t n) {
  if (!c) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t k = idx ? idx[i] : i;
    if (k >= c->nodes.size()) return GS_EINVAL;
    c->nodes[k].node = nodes[i];
    c->nodes[k].has_node = true;
  }
  return GS_OK;
}

int or_node_metrics_upsert(or_cluster* c, const uint32_t* idx, const gs_node_metric* m, uint32_t n,
                           const gs_pod_metric* pm, const uint32_t* off) {
  if (!c) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t k = idx ? idx[i] : i;
    if (k >= c->nodes.size()) return GS_EINVAL;
    NodeState& s = c->nodes[k];
    s.metric = m[i];
    s.pods_metric.clear();
    if (pm && off)
      for (uint32_t j = off[i]; j < off[i + 1]; ++j)
        s.pods_metric.push_back({pm[j].name_key, pm[j].in_lister, pm[j].priority_class, from_usage(pm[j].usage)});
  }
  return GS_OK;
}

// podAssignCache.assign (pod_assign_cache.go:53-68)
int or_pods_assign(or_cluster* c, const uint32_t* node_idx, const gs_pod* pods, const int64_t* ts, uint32_t n) {
  if (!c) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    if (node_idx[i] >= c->nodes.size()) return GS_EINVAL;
    if (pods[i].flags & GS_POD_TERMINATED) continue;
    c->nodes[node_idx[i]].assigned[pods[i].uid] = AssignInfo{ts ? ts[i] : c->now, pods[i]};
  }
  return GS_OK;
}

// podAssignCache.unAssign (pod_assign_cache.go:70-80)
int or_pods_unassign(or_cluster* c, const uint32_t* node_idx, const gs_pod* pods, uint32_t n) {
  if (!c) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    if (node_idx[i] >= c->nodes.size()) return GS_EINVAL;
    c->nodes[node_idx[i]].assigned.erase(pods[i].uid);
  }
  return GS_OK;
}

// ForgetPod of an assumed pod after Unreserve: NodeInfo.RemovePod ([upstream] framework/types.go), LoadAware
// podAssignCache.unAssign (load_aware.go:265-267), NodeNUMAResource resourceManager.Release (plugin.go:467-476)
int or_pods_forget(or_cluster* c, const uint32_t* node_idx, const gs_pod* pods, uint32_t n) {
  if (!c || (n && (!node_idx || !pods))) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i)
    if (node_idx[i] >= c->nodes.size()) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    gs_node& nd = c->nodes[node_idx[i]].node;
    for (int r = 0; r < GS_NUM_RES; ++r) nd.requested[r] -= pods[i].requests[r];
    nd.nonzero_requested[0] -= pods[i].nonzero_requests[0];
    nd.nonzero_requested[1] -= pods[i].nonzero_requests[1];
    nd.pod_count -= 1;
    c->nodes[node_idx[i]].assigned.erase(pods[i].uid);
    if (node_idx[i] < c->numa.size()) c->numa[node_idx[i]].alloc.release(pods[i].uid);
  }
  return GS_OK;
}

// podAssignCache.OnAdd / OnUpdate / OnDelete (pod_assign_cache.go:82-117) over assign / unAssign (:53-80)
int or_pods_on_event(or_cluster* c, int event, const int32_t* node_idx, const gs_pod* pods, uint32_t n) {
  if (!c || (n && (!node_idx || !pods))) return GS_EINVAL;
  for (uint32_t j = 0; j < n; ++j) {
    const int32_t i = node_idx[j];
    if (i >= (int32_t)c->nodes.size()) return GS_EINVAL;
    const bool terminated = pods[j].flags & GS_POD_TERMINATED;
    bool do_assign;
    if (event == GS_POD_EVENT_ADD) do_assign = true;
    else if (event == GS_POD_EVENT_UPDATE) do_assign = !terminated;
    else if (event == GS_POD_EVENT_DELETE) do_assign = false;
    else return GS_EINVAL;
    if (i < 0) continue;   // nodeName == ""
    if (do_assign) {
      if (terminated) continue;
      c->nodes[i].assigned[pods[j].uid] = AssignInfo{c->now, pods[j]};
    } else {
      c->nodes[i].assigned.erase(pods[j].uid);
    }
  }
  return GS_OK;
}

int or_assign_cache_get(or_cluster* c, uint32_t node, uint64_t* uids, int64_t* ts, uint32_t cap) {
  if (!c || node >= c->nodes.size()) return GS_EINVAL;
  uint32_t k = 0;
  for (const auto& kv : c->nodes[node].assigned) {   // std::map: uid order
    if (k < cap) {
      if (uids) uids[k] = kv.first;
      if (ts) ts[k] = kv.second.timestamp;
    }
    ++k;
  }
  return (int)k;
}

int or_estimate_pod(const gs_loadaware_args* a, const gs_pod* pod, int64_t out[2], uint32_t* out_mask) {
  if (!a || !pod || !out) return GS_EINVAL;
  ResList e = estimate_pod(*a, *pod);
  out[0] = e.v[0];
  out[1] = e.v[1];
  if (out_mask) *out_mask = e.mask;
  return GS_OK;
}

int or_estimate_node(const gs_node* node, int64_t out[2]) {
  if (!node || !out) return GS_EINVAL;
  out[0] = estimate_node(*node, 0);
  out[1] = estimate_node(*node, 1);
  return GS_OK;
}

int or_loadaware_filter(or_cluster* c, const gs_pod* pod, uint32_t node, int32_t* fail) {
  if (!valid_node(c, node) || !pod || !fail) return GS_EINVAL;
  *fail = loadaware_filter(*c, *pod, c->nodes[node]) ? 1 : 0;
  return GS_OK;
}

int or_loadaware_score(or_cluster* c, const gs_pod* pod, uint32_t node, int64_t* score) {
  if (!valid_node(c, node) || !pod || !score) return GS_EINVAL;
  *score = loadaware_score(*c, *pod, c->nodes[node]);
  return GS_OK;
}

int or_fit_filter(or_cluster* c, const gs_pod* pod, uint32_t node, uint32_t* fail_bits) {
  if (!valid_node(c, node) || !pod || !fail_bits) return GS_EINVAL;
  *fail_bits = fit_filter(*pod, c->nodes[node].node);
  return GS_OK;
}

int or_fit_score(or_cluster* c, const gs_pod* pod, uint32_t node, int64_t* score) {
  if (!valid_node(c, node) || !pod || !score) return GS_EINVAL;
  *score = fit_score(c->cfg.fit, *pod, c->nodes[node].node);
  return GS_OK;
}

int or_evaluate(or_cluster* c, const gs_pod* pods, uint32_t npods, int16_t* scores, uint16_t* codes,
                int16_t* plugin_scores) {
  if (!c) return GS_EINVAL;
  size_t N = c->nodes.size();
  for (uint32_t p = 0; p < npods; ++p) {
    orn::PreState st = orn::prefilter(c->numa_args, pods[p]);
    for (size_t n = 0; n < N; ++n) {
      if (!c->nodes[n].has_node) return GS_ESTATE;
      PairResult r = eval_pair(*c, pods[p], st, (uint32_t)n);
      size_t o = (size_t)p * N + n;
      if (codes) codes[o] = r.code;
      if (scores) scores[o] = r.code ? (int16_t)-1 : (int16_t)weighted_total(*c, r);
      if (plugin_scores) {
        plugin_scores[o * GS_NUM_PLUGINS + GS_PLUGIN_FIT] = (int16_t)r.fit;
        plugin_scores[o * GS_NUM_PLUGINS + GS_PLUGIN_LOADAWARE] = (int16_t)r.la;
        plugin_scores[o * GS_NUM_PLUGINS + GS_PLUGIN_NUMA] = (int16_t)r.numa;
      }
    }
  }
  return GS_OK;
}

int or_topology_register(or_cluster* c, const gs_cpu_topology* t, int32_t* id) {
  if (!c || !t || !id || t->num_cpus < 0 || t->num_cpus > GS_MAX_CPUS) return GS_EINVAL;
  auto topo = orn::build_topology(*t);
  if (topo->num_sockets > 12) return GS_EUNSUPPORTED;
  c->topologies.push_back(topo);
  *id = (int32_t)c->topologies.size() - 1;
  return GS_OK;
}

// TopologyOptionsManager.UpdateTopologyOptions (topology_options.go:76-86) with the node labels resolved
int or_nodes_numa_upsert(or_cluster* c, const uint32_t* idx, const gs_node_numa* nn, uint32_t n) {
  if (!c) return GS_EINVAL;
  for (uint32_t j = 0; j < n; ++j) {
    uint32_t k = idx ? idx[j] : j;
    if (k >= c->numa.size()) return GS_EINVAL;
    const gs_node_numa& x = nn[j];
    orn::TopologyOptions o;
    o.present = x.has_options != 0;
    if (o.present) {
      if (x.topology >= 0) {
        if (x.topology >= (int)c->topologies.size()) return GS_EINVAL;
        o.topo = c->topologies[x.topology];
      } else {
        o.topo = std::make_shared<orn::CPUTopology>();   // reported but empty: non-nil, invalid
      }
      for (int cpu = 0; cpu < GS_MAX_CPUS; ++cpu)
        if (x.reserved_cpus[cpu >> 6] >> (cpu & 63) & 1) o.reserved.insert(cpu);
      o.max_ref = x.max_ref_count ? x.max_ref_count : 1;
      for (int z = 0; z < x.num_zones && z < GS_MAX_NUMA; ++z) {
        orn::NUMANodeResource nr;
        nr.node = x.zones[z].node_id;
        if (x.zones[z].mask & GS_USAGE_CPU) nr.res.set(GS_RES_CPU, x.zones[z].cpu_milli);
        if (x.zones[z].mask & GS_USAGE_MEMORY) nr.res.set(GS_RES_MEMORY, x.zones[z].memory);
        o.numa.push_back(nr);
      }
    }
    o.amp_ratio = x.cpu_amplification_ratio;   // effective ratio after amplifyNUMANodeResources (util.go:62-83)
    o.node_cpu_bind = x.node_cpu_bind_policy;
    o.numa_policy = x.numa_topology_policy;
    o.numa_alloc_strategy = x.numa_allocate_strategy;
    o.node_amp_ratio = x.node_cpu_amplification_ratio;
    o.node_amp_invalid = x.node_amplification_invalid != 0;
    c->numa[k].opts = o;
  }
  return GS_OK;
}

int or_numa_allocations_update(or_cluster* c, const uint32_t* node_idx, const gs_pod_allocation* a, uint32_t n) {
  if (!c) return GS_EINVAL;
  for (uint32_t j = 0; j < n; ++j) {
    if (node_idx[j] >= c->numa.size()) return GS_EINVAL;
    orn::NodeNUMA& nn = c->numa[node_idx[j]];
    if (!(nn.opts.topo && nn.opts.topo->valid())) continue;   // resourceManager.Update skips
    nn.alloc.update(pod_allocation_of(a[j]), nn.opts.topo.get());
  }
  return GS_OK;
}

int or_numa_allocations_release(or_cluster* c, const uint32_t* node_idx, const uint64_t* uids, uint32_t n) {
  if (!c) return GS_EINVAL;
  for (uint32_t j = 0; j < n; ++j) {
    if (node_idx[j] >= c->numa.size()) return GS_EINVAL;
    c->numa[node_idx[j]].alloc.release(uids[j]);
  }
  return GS_OK;
}

int or_numa_allocation_get(or_cluster* c, uint32_t node, uint64_t uid, gs_pod_allocation* out) {
  if (!c || node >= c->numa.size() || !out) return GS_EINVAL;
  auto it = c->numa[node].alloc.pods.find(uid);
  if (it == c->numa[node].alloc.pods.end()) return 0;
  export_allocation(it->second, out);
  return 1;
}

int or_numa_topology_hints(or_cluster* c, const gs_pod* pod, uint32_t node, int32_t* res, uint64_t* masks,
                           uint8_t* preferred, uint32_t cap, uint32_t* count) {
  if (!c || !pod || !count || node >= c->numa.size()) return GS_EINVAL;
  const orn::PreState st = orn::prefilter(c->numa_args, *pod);
  return orn::topology_hints_test(c->numa_args, st, c->numa[node], res, masks, preferred, cap, count);
}

int or_set_hint_order(or_cluster* c, int reverse) {
  if (!c) return GS_EINVAL;
  c->reverse_hint_order = reverse != 0;
  return GS_OK;
}

int or_take_cpus_test(int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core, int max_ref,
                      const uint64_t* available, const int32_t* alloc_ref, const int32_t* alloc_excl, int needed,
                      int bind, int excl, int strategy, uint64_t* result) {
  auto topo = orn::build_test_topology(sockets, nodes_per_socket, cores_per_node, cpus_per_core);
  orn::CPUSet avail;
  orn::CPUDetails details;
  for (auto& kv : topo->details) {
    int cpu = kv.first;
    if (available[cpu >> 6] >> (cpu & 63) & 1) avail.insert(cpu);
    if (alloc_ref && alloc_ref[cpu] >= 0) {
      orn::CPUInfo info = kv.second;
      info.ref = alloc_ref[cpu];
      info.excl = alloc_excl ? alloc_excl[cpu] : 0;
      details[cpu] = info;
    }
  }
  orn::CPUSet out;
  bool ok = orn::take_cpus(*topo, max_ref, avail, details, needed, bind, excl, strategy, &out);
  for (int w = 0; w < GS_CPU_WORDS; ++w) result[w] = 0;
  for (int cpu : out) result[cpu >> 6] |= 1ull << (cpu & 63);
  return ok ? 0 : -1;
}

// NodeAllocation (node_allocation.go:32-177) on a buildCPUTopologyForTest topology (the CoreID = socket<<16 | core
// form node_allocation_test.go uses): a script of ops. op 0: addCPUs(uid, set, excl); op 1: release(uid);
// op 2: getAvailableCPUs(maxRef = arg, reserved = none, preferred = set) -> out (4 words per op).
// refcount[cpu] (256 entries, may be NULL) = allocatedCPUs[cpu].RefCount after the script (-1: no entry).
int or_node_allocation_script(int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core, int nops,
                              const int32_t* op, const uint64_t* uid, const uint64_t* set, const int32_t* arg,
                              uint64_t* out, int32_t* refcount) {
  auto topo = orn::build_test_topology(sockets, nodes_per_socket, cores_per_node, cpus_per_core);
  orn::NodeAllocation na;
  for (int k = 0; k < nops; ++k) {
    orn::CPUSet cs;
    for (int cpu = 0; cpu < GS_MAX_CPUS; ++cpu)
      if (set[4 * k + (cpu >> 6)] >> (cpu & 63) & 1) cs.insert(cpu);
    for (int w = 0; w < 4; ++w) out[4 * k + w] = 0;
    if (op[k] == 0) {
      orn::PodAllocation pa;
      pa.uid = uid[k];
      pa.cpus = cs;
      pa.excl = arg[k];
      na.add(pa, topo.get());
    } else if (op[k] == 1) {
      na.release(uid[k]);
    } else if (op[k] == 2) {
      orn::CPUSet avail;
      orn::CPUDetails alloc;
      na.available_cpus(*topo, arg[k], orn::CPUSet{}, cs, &avail, &alloc);
      for (int cpu : avail) out[4 * k + (cpu >> 6)] |= 1ull << (cpu & 63);
    } else {
      return GS_EINVAL;
    }
  }
  if (refcount)
    for (int cpu = 0; cpu < GS_MAX_CPUS; ++cpu) {
      auto it = na.allocated_cpus.find(cpu);
      refcount[cpu] = it == na.allocated_cpus.end() ? -1 : it->second.ref;
    }
  return GS_OK;
}

// getAvailableNUMANodeResources (node_allocation.go:141-177) for two NUMA nodes of a buildCPUTopologyForTest topology:
// zone resources zone_cpu/zone_mem, AmplificationRatios[cpu] = amp (<= 1: none), allocatedResources[0] cpu =
// alloc_cpu0 (0: no entry), the first n_cpuset CPUs in allocatedCPUs. avail / alloc: [zone][cpu, mem], masks bit
// 2*zone + r = key present (alloc_mask bit 4 = zone entry present).
int or_available_numa_test(int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core, double amp,
                           int64_t zone_cpu, int64_t zone_mem, int64_t alloc_cpu0, int n_cpuset, int64_t* avail,
                           uint32_t* avail_mask, int64_t* alloc, uint32_t* alloc_mask) {
  orn::TopologyOptions o;
  o.present = true;
  o.topo = orn::build_test_topology(sockets, nodes_per_socket, cores_per_node, cpus_per_core);
  o.max_ref = 1;
  o.amp_ratio = amp;
  for (int z = 0; z < 2; ++z) {
    orn::NUMANodeResource r;
    r.node = z;
    r.res.set(GS_RES_CPU, zone_cpu);
    r.res.set(GS_RES_MEMORY, zone_mem);
    o.numa.push_back(r);
  }
  orn::NodeAllocation na;
  if (alloc_cpu0) {
    orn::NUMANodeResource r;
    r.node = 0;
    r.res.set(GS_RES_CPU, alloc_cpu0);
    na.allocated_res[0] = r;
  }
  for (int cpu = 0; cpu < n_cpuset; ++cpu) na.allocated_cpus[cpu] = o.topo->details[cpu];
  std::map<int, orn::RL> ta, tl;
  na.available_numa(o, &ta, &tl);
  *avail_mask = *alloc_mask = 0;
  for (int z = 0; z < 2; ++z)
    for (int r = 0; r < 2; ++r) {
      avail[2 * z + r] = alloc[2 * z + r] = 0;
      if (ta.count(z) && ta[z].has(r)) { avail[2 * z + r] = ta[z].v[r]; *avail_mask |= 1u << (2 * z + r); }
      if (tl.count(z)) {
        *alloc_mask |= 1u << (4 + z);
        if (tl[z].has(r)) { alloc[2 * z + r] = tl[z].v[r]; *alloc_mask |= 1u << (2 * z + r); }
      }
    }
  return GS_OK;
}

// [upstream] Scheduler.numFeasibleNodesToFind (schedule_one.go): minFeasibleNodesToFind = 100,
// minFeasibleNodesPercentageToFind = 5, adaptive percentage 50 - N/125 when pct <= 0 (int32 arithmetic).
uint32_t or_num_feasible_nodes_to_find(uint32_t num_all_nodes, int32_t pct) {
  const int32_t n = (int32_t)num_all_nodes;
  if (n < 100 || pct >= 100) return num_all_nodes;
  int32_t adaptive = pct;
  if (adaptive <= 0) {
    adaptive = 50 - n / 125;
    if (adaptive < 5) adaptive = 5;
  }
  const int32_t nodes = n * adaptive / 100;
  return nodes < 100 ? 100u : (uint32_t)nodes;
}

uint32_t or_next_start_node_index(const or_cluster* c) { return c ? c->next_start : 0; }

int32_t or_tiebreak_intn(uint64_t seed, uint64_t seq, int64_t cnt) {
  TieBreakRand rnd(seed, seq);
  return rnd.intn(cnt);
}

// [upstream] scheduleOne for each pod: findNodesThatFitPod -> prioritizeNodes -> selectHost -> assume + Reserve.
int or_schedule_replay(or_cluster* c, const gs_pod* pods, uint32_t npods, const uint64_t* seq,
                       const int32_t* given, gs_placement* out, int nthreads);

int or_schedule(or_cluster* c, const gs_pod* pods, uint32_t npods, const uint64_t* seq, gs_placement* out,
                int nthreads) {
  return or_schedule_replay(c, pods, npods, seq, nullptr, out, nthreads);
}

// Replay (test infrastructure for full-size parity): a pod with given[p] >= 0 is not scheduled but placed on
// that node — its Filter runs on that node alone (the topologymanager affinity Reserve consumes; a node that
// fails Filter is an error), then Reserve + assume exactly as for a scheduled pod; only node and flags are
// reported for it. given[p] == -2 replays a FitError (nothing assumed); pods with given[p] == -1 run the full
// scheduleOne below on the replayed state.
int or_schedule_replay(or_cluster* c, const gs_pod* pods, uint32_t npods, const uint64_t* seq,
                       const int32_t* given, gs_placement* out, int nthreads) {
  if (!c || !out) return GS_EINVAL;
  int N = (int)c->nodes.size();
  for (int n = 0; n < N; ++n)
    if (!c->nodes[n].has_node) return GS_ESTATE;
  std::vector<uint8_t> feasible(N);
  std::vector<int64_t> score(N);
  std::vector<orn::Hint> affinity(N);   // topologymanager Store of the cycle (store.go:55-66)
  std::vector<int> feasible_list;
  feasible_list.reserve(N);
  std::unique_ptr<Pool> pool;
  if (nthreads > 1) pool.reset(new Pool(nthreads));
  using clk = std::chrono::steady_clock;
  auto lap = [](clk::time_point& t0) {   // seconds since t0, t0 advanced
    const clk::time_point t = clk::now();
    const double d = std::chrono::duration<double>(t - t0).count();
    t0 = t;
    return d;
  };
  for (uint32_t p = 0; p < npods; ++p) {
    clk::time_point tp = clk::now();
    const gs_pod& pod = pods[p];
    const orn::PreState st = orn::prefilter(c->numa_args, pod);
    gs_placement& o = out[p];
    int selected = -1;
    if (given && given[p] == -2) {   // replayed FitError: nothing assumed
      o.feasible = 0; o.flags = 0; o.node = -1; o.score = 0; o.ties = 0;
      continue;
    }
    if (given && given[p] >= 0) {
      if (given[p] >= N) return GS_EINVAL;
      if (c->cfg.sample_nodes) return GS_EUNSUPPORTED;   // a replayed pod's processedNodes is unknown
      selected = given[p];
      const NodeState& s = c->nodes[selected];
      uint16_t code = 0;
      if (c->cfg.enabled & GS_ENABLE_FIT_FILTER) code |= (uint16_t)fit_filter(pod, s.node);
      if (c->cfg.enabled & GS_ENABLE_LA_FILTER) code |= loadaware_filter(*c, pod, s);
      affinity[selected] = orn::Hint{};
      if (!code && (c->cfg.enabled & GS_ENABLE_NUMA_FILTER))
        code |= numa_filter(*c, st, (uint32_t)selected, &affinity[selected]);
      if (code) return GS_ESTATE;
      o.feasible = 0; o.flags = 0; o.node = selected; o.score = 0; o.ties = 0;
    } else {
    auto check = [&](int n) {
      const NodeState& s = c->nodes[n];
      uint16_t code = 0;
      if (c->cfg.enabled & GS_ENABLE_FIT_FILTER) code |= (uint16_t)fit_filter(pod, s.node);
      if (c->cfg.enabled & GS_ENABLE_LA_FILTER) code |= loadaware_filter(*c, pod, s);
      affinity[n] = orn::Hint{};
      if (!code && (c->cfg.enabled & GS_ENABLE_NUMA_FILTER)) code |= numa_filter(*c, st, (uint32_t)n, &affinity[n]);
      feasible[n] = code == 0;
    };
    feasible_list.clear();
    if (!c->cfg.sample_nodes) {
      // findNodesThatPassFilters with percentageOfNodesToScore = 100: every node is checked and
      // nextStartNodeIndex = (start + N) % N stays put: feasible order = node index order.
      if (pool) pool->until(N, check);
      else for (int n = 0; n < N; ++n) check(n);
      for (int n = 0; n < N; ++n)
        if (feasible[n]) feasible_list.push_back(n);
      c->phase_s[0] += lap(tp);
    } else {
      // findNodesThatPassFilters with node sampling, parallelism-1 order: nodes are checked in rotation order
      // from nextStartNodeIndex; the (K+1)-th feasible node cancels the search uncounted (feasibleNodesLen is
      // decremented), processedNodes = feasible + diagnosed, nextStartNodeIndex advances by it (mod N)
      const int K = (int)or_num_feasible_nodes_to_find((uint32_t)N, c->cfg.percentage_of_nodes_to_score);
      int diagnosed = 0;
      for (int i = 0; i < N; ++i) {
        const int n = (int)((c->next_start + (uint32_t)i) % (uint32_t)N);
        check(n);
        if (!feasible[n]) { ++diagnosed; continue; }
        if ((int)feasible_list.size() >= K) break;
        feasible_list.push_back(n);
      }
      c->next_start = (uint32_t)((c->next_start + feasible_list.size() + (uint32_t)diagnosed) % (uint32_t)N);
    }
    o.feasible = (uint32_t)feasible_list.size();
    o.flags = 0;
    if (feasible_list.empty()) {   // FitError: nothing is assumed
      o.node = -1; o.score = 0; o.ties = 0;
      continue;
    }
    // prioritizeNodes: RunScorePlugins over the feasible list, weight and sum.
    auto score_one = [&](int i) {
      int n = feasible_list[i];
      PairResult r{0, 0, 0, 0};
      if (c->cfg.enabled & GS_ENABLE_FIT_SCORE) r.fit = fit_score(c->cfg.fit, pod, c->nodes[n].node);
      if (c->cfg.enabled & GS_ENABLE_LA_SCORE) r.la = loadaware_score(*c, pod, c->nodes[n]);
      if (c->cfg.enabled & GS_ENABLE_NUMA_SCORE)
        r.numa = orn::score(c->numa_args, st, c->numa[n], node_view(c->nodes[n].node), affinity[n]);
      score[n] = weighted_total(*c, r);
    };
    int F = (int)feasible_list.size();
    if (pool) pool->until(F, score_one);
    else for (int i = 0; i < F; ++i) score_one(i);
    c->phase_s[1] += lap(tp);
    // selectHost ([upstream] schedule_one.go)
    TieBreakRand rnd(c->cfg.seed, seq ? seq[p] : p);
    selected = feasible_list[0];
    int64_t max_score = score[selected];
    int64_t cnt = 1;
    for (int i = 1; i < F; ++i) {
      int n = feasible_list[i];
      if (score[n] > max_score) {
        max_score = score[n]; selected = n; cnt = 1;
      } else if (score[n] == max_score) {
        ++cnt;
        if (rnd.intn(cnt) == 0) selected = n;
      }
    }
    o.node = selected; o.score = max_score; o.ties = (uint32_t)cnt;
    c->phase_s[2] += lap(tp);
    }
    // Reserve: NodeNUMAResource (plugin.go:375-422) on the pre-assume NodeInfo
    if (c->cfg.enabled & (GS_ENABLE_NUMA_FILTER | GS_ENABLE_NUMA_SCORE)) {
      orn::PodAllocation pa;
      if (orn::reserve(c->numa_args, st, c->numa[selected], pod, affinity[selected], &pa) != 0) return GS_ESTATE;
      if (!pa.numa.empty()) o.flags |= GS_PLACED_NUMA;
      // the Filter-time affinity hint (topologymanager store) as a mask over the node's zone slots
      const orn::Hint& h = affinity[selected];
      if (h.has_mask) {
        const auto& zones = c->numa[selected].opts.numa;
        for (size_t z = 0; z < zones.size() && z < 4; ++z)
          if (zones[z].node >= 0 && zones[z].node < 64 && ((h.mask >> zones[z].node) & 1))
            o.flags |= 1u << (GS_PLACED_AFFINITY_SHIFT + z);
      }
      if (!pa.cpus.empty()) o.flags |= GS_PLACED_CPUSET;
    }
    // assume: NodeInfo.AddPod ([upstream] framework/types.go calculateResource)
    gs_node& nd = c->nodes[selected].node;
    for (int r = 0; r < GS_NUM_RES; ++r) nd.requested[r] += pod.requests[r];
    nd.nonzero_requested[0] += pod.nonzero_requests[0];
    nd.nonzero_requested[1] += pod.nonzero_requests[1];
    nd.pod_count += 1;
    // Reserve: LoadAware podAssignCache.assign(node, pod) with timestamp = now (load_aware.go:260-263)
    if (!(pod.flags & GS_POD_TERMINATED))
      c->nodes[selected].assigned[pod.uid] = AssignInfo{c->now, pod};
    c->phase_s[3] += lap(tp);
  }
  return GS_OK;
}

// seconds spent per scheduleOne phase since the last call: Filter (findNodesThatPassFilters), Score
// (prioritizeNodes), selectHost, Reserve + assume (cpu_baseline breakdown)
int or_phase_times(or_cluster* c, double out[4]) {
  if (!c || !out) return GS_EINVAL;
  for (int i = 0; i < 4; ++i) { out[i] = c->phase_s[i]; c->phase_s[i] = 0; }
  return GS_OK;
}

}  // extern "C"

// =============================================================================================
// Extension plugins: Reservation + DeviceShare. Restated with
// ResourceList-shaped maps keyed by resource slot / GPU resource name; reservations iterate in uid order
// (the reference walks a Go map, reservation/cache.go forEachAvailableReservationOnNode — the harness fixes the
// order, as for the NUMA hint providers).
// =============================================================================================
namespace {

// corev1.ResourceList over the node resource slots (key presence kept: quotav1 semantics depend on it)
struct RList {
  std::map<int, int64_t> m;
  int64_t get(int r) const { auto it = m.find(r); return it == m.end() ? 0 : it->second; }
  bool has(int r) const { return m.count(r) != 0; }
  bool is_zero() const { for (auto& kv : m) if (kv.second != 0) return false; return true; }   // quotav1.IsZero
};
RList rlist_of(const int64_t* v, uint32_t mask) {
  RList l;
  for (int r = 0; r < GS_NUM_RES; ++r)
    if (mask & (1u << r)) l.m[r] = v[r];
  return l;
}
RList rl_add(const RList& a, const RList& b) {   // quotav1.Add
  RList o = a;
  for (auto& kv : b.m) o.m[kv.first] = a.get(kv.first) + kv.second;
  return o;
}
RList rl_sub(const RList& a, const RList& b) {   // quotav1.Subtract
  RList o = a;
  for (auto& kv : b.m) o.m[kv.first] = a.get(kv.first) - kv.second;
  return o;
}
RList rl_sub_nonneg(const RList& a, const RList& b) {   // quotav1.SubtractWithNonNegativeResult
  RList o;
  for (auto& kv : a.m) o.m[kv.first] = std::max<int64_t>(0, kv.second - b.get(kv.first));
  for (auto& kv : b.m)
    if (!a.has(kv.first)) o.m[kv.first] = std::max<int64_t>(0, -kv.second);
  return o;
}
RList rl_mask(const RList& a, uint32_t names) {   // quotav1.Mask
  RList o;
  for (auto& kv : a.m)
    if (names & (1u << kv.first)) o.m[kv.first] = kv.second;
  return o;
}
uint32_t rl_names(const RList& a) { uint32_t n = 0; for (auto& kv : a.m) n |= 1u << kv.first; return n; }
RList rl_remove_zeros(const RList& a) { RList o; for (auto& kv : a.m) if (kv.second) o.m[kv.first] = kv.second; return o; }

// [upstream] schedutil.GetNonzeroRequests of a container with these requests: cpu 100m / memory 200MiB when unset
void nonzero_of(const RList& req, int64_t* cpu, int64_t* mem) {
  *cpu = req.has(GS_RES_CPU) ? req.get(GS_RES_CPU) : 100;
  *mem = req.has(GS_RES_MEMORY) ? req.get(GS_RES_MEMORY) : 200LL * 1024 * 1024;
}

// transformer.go:294-307 updateNodeInfoRequested (a one-container pod with `req`)
void update_requested(gs_node& n, const RList& req, int64_t sign) {
  for (auto& kv : req.m) n.requested[kv.first] += sign * kv.second;
  int64_t c, m;
  nonzero_of(req, &c, &m);
  n.nonzero_requested[0] += sign * c;
  n.nonzero_requested[1] += sign * m;
}

struct NodeRState {               // reservation/plugin.go nodeReservationState
  std::vector<const gs_reservation*> matched;
  gs_node restored{};             // NodeInfo after BeforePreFilter
  gs_node pod_requested{};        // Requested after the unmatched trim (podRequested)
  RList r_allocated;              // Σ matched Allocated
  bool has = false;
};

// ---- DeviceShare (deviceshare/*.go), GPU device type ----
struct GpuReq {                   // ConvertDeviceRequest result: keys of gs_gpu_res present
  int64_t v[GS_NUM_GPU_RES] = {0, 0, 0};
  uint32_t mask = 0;
};
// GetPodDeviceRequests (utils.go:232-252) for the GPU type: 0 ok (req->mask == 0: no GPU request), <0 invalid
int gpu_pod_request(const gs_pod_ext& e, GpuReq* req) {
  *req = GpuReq{};
  const uint32_t m = e.gpu_request_mask & 0x1Fu;   // after RemoveZeros (the caller passes non-zero keys only)
  if (!m) return 0;
  for (int n = 0; n < GS_NUM_GPU_NAMES; ++n) {     // ValidatePercentageResource for koord gpu, core, ratio
    if (!(m & (1u << n))) continue;
    const int64_t q = e.gpu_requests[n];
    if ((n == GS_GPU_NAME_KOORD_GPU || n == GS_GPU_NAME_CORE || n == GS_GPU_NAME_MEMORY_RATIO) && q > 100 && q % 100)
      return -1;
  }
  const uint32_t NV = 1u << GS_GPU_NAME_NVIDIA, KG = 1u << GS_GPU_NAME_KOORD_GPU, CO = 1u << GS_GPU_NAME_CORE,
                 ME = 1u << GS_GPU_NAME_MEMORY, RA = 1u << GS_GPU_NAME_MEMORY_RATIO;
  // ValidDeviceResourceCombinations (utils.go:69-79) + ResourceCombinationsMapper (:89-144)
  if (m == NV) {
    req->v[GS_GPU_CORE] = req->v[GS_GPU_MEMORY_RATIO] = e.gpu_requests[GS_GPU_NAME_NVIDIA] * 100;
    req->mask = 3;
  } else if (m == KG) {
    req->v[GS_GPU_CORE] = req->v[GS_GPU_MEMORY_RATIO] = e.gpu_requests[GS_GPU_NAME_KOORD_GPU];
    req->mask = 3;
  } else if (m == ME) {
    req->v[GS_GPU_MEMORY] = e.gpu_requests[GS_GPU_NAME_MEMORY]; req->mask = 4;
  } else if (m == RA) {
    req->v[GS_GPU_MEMORY_RATIO] = e.gpu_requests[GS_GPU_NAME_MEMORY_RATIO]; req->mask = 2;
  } else if (m == (CO | ME)) {
    req->v[GS_GPU_CORE] = e.gpu_requests[GS_GPU_NAME_CORE];
    req->v[GS_GPU_MEMORY] = e.gpu_requests[GS_GPU_NAME_MEMORY]; req->mask = 5;
  } else if (m == (CO | RA)) {
    req->v[GS_GPU_CORE] = e.gpu_requests[GS_GPU_NAME_CORE];
    req->v[GS_GPU_MEMORY_RATIO] = e.gpu_requests[GS_GPU_NAME_MEMORY_RATIO]; req->mask = 3;
  } else {
    return -1;
  }
  return 0;
}

struct GpuRes {                   // one device's ResourceList over gs_gpu_res (all three keys, as a Device reports)
  int64_t v[GS_NUM_GPU_RES] = {0, 0, 0};
  bool zero() const { return !v[0] && !v[1] && !v[2]; }
};
struct NodeDev {                  // nodeDevice after filterNodeDevice (device_allocator.go:139-163): minors with info
  std::map<int, GpuRes> total, free;
};
// numaNodes: the allocator's NUMA affinity (the topology manager's store entry; nullptr / no mask = none): only the
// minors whose Topology.NodeID it holds are candidates (device_allocator.go:148-152)
bool on_numa(const gs_gpu_device& g, const orn::Hint* numa) {
  if (!numa || !numa->has_mask) return true;
  return g.numa_node >= 0 && g.numa_node < 64 && (numa->mask >> g.numa_node & 1u);
}
NodeDev filtered_node_device(const gs_node_devices& d, const orn::Hint* numa = nullptr) {
  NodeDev o;
  std::map<int, GpuRes> free_all;   // resetDeviceFree (device_cache.go:157-174)
  bool all_zero = true;
  for (int g = 0; g < d.num_gpus && g < GS_MAX_GPUS; ++g) {
    GpuRes f;
    for (int r = 0; r < GS_NUM_GPU_RES; ++r) f.v[r] = std::max<int64_t>(0, d.gpus[g].total[r] - d.gpus[g].used[r]);
    free_all[d.gpus[g].minor] = f;
    if (!f.zero()) all_zero = false;
  }
  if (all_zero) return o;           // nodeDevice.filter: freeDevices.isZero() -> the type is dropped (device_cache.go:361)
  for (int g = 0; g < d.num_gpus && g < GS_MAX_GPUS; ++g) {
    if (!d.gpus[g].has_info || !on_numa(d.gpus[g], numa)) continue;
    GpuRes t;
    for (int r = 0; r < GS_NUM_GPU_RES; ++r) t.v[r] = d.gpus[g].total[r];
    o.total[d.gpus[g].minor] = t;
    o.free[d.gpus[g].minor] = free_all[d.gpus[g].minor];
  }
  return o;
}

// GPUHandler.CalcDesiredRequestsAndCount (devicehandler_gpu.go:38-64): per-instance request (keys: mask) and count.
// <0: UnschedulableAndUnresolvable (no GPU devices / no healthy GPU)
int gpu_desired(const gs_node_devices& d, const GpuReq& pod, GpuReq* inst, int64_t* count) {
  if (d.num_gpus <= 0) return -1;                       // len(deviceTotal[gpu]) == 0
  int64_t total_mem = -1;                               // fillGPUTotalMem: the first healthy device (all GPUs of a
  for (int g = 0; g < d.num_gpus && g < GS_MAX_GPUS; ++g) {   // node are one model: the same memory)
    bool z = !d.gpus[g].total[0] && !d.gpus[g].total[1] && !d.gpus[g].total[2];
    if (!z) { total_mem = d.gpus[g].total[GS_GPU_MEMORY]; break; }
  }
  if (total_mem < 0) return -2;
  GpuReq r = pod;
  if (r.mask & (1u << GS_GPU_MEMORY)) {
    r.v[GS_GPU_MEMORY_RATIO] = (int64_t)((double)r.v[GS_GPU_MEMORY] / (double)total_mem * 100);   // memoryBytesToRatio
  } else {
    r.v[GS_GPU_MEMORY] = r.v[GS_GPU_MEMORY_RATIO] * total_mem / 100;                           // memoryRatioToBytes
  }
  r.mask |= (1u << GS_GPU_MEMORY) | (1u << GS_GPU_MEMORY_RATIO);
  *count = 1;
  const int64_t ratio = r.v[GS_GPU_MEMORY_RATIO];
  if (ratio > 100 && ratio % 100 == 0) {
    const int64_t n = ratio / 100;
    *count = n;
    GpuReq o;
    o.v[GS_GPU_CORE] = r.v[GS_GPU_CORE] / n;
    o.v[GS_GPU_MEMORY] = r.v[GS_GPU_MEMORY] / n;
    o.v[GS_GPU_MEMORY_RATIO] = ratio / n;
    o.mask = 7;
    r = o;
  }
  *inst = r;
  return 0;
}

bool le_request(const GpuReq& req, const GpuRes& free) {   // quotav1.LessThanOrEqual(request, free) over request keys
  for (int r = 0; r < GS_NUM_GPU_RES; ++r)
    if ((req.mask & (1u << r)) && req.v[r] > free.v[r]) return false;
  return true;
}

int64_t ds_least(int64_t req, int64_t cap) { return cap == 0 || req > cap ? 0 : (cap - req) * kMaxNodeScore / cap; }
int64_t ds_most(int64_t req, int64_t cap) {
  if (cap == 0) return 0;
  if (req > cap) req = cap;
  return req * kMaxNodeScore / cap;
}
// resourceAllocationScorer (scoring.go:186-243): requested = total - free + request (total >= free)
int64_t ds_scorer(const gs_ext_args& a, const int64_t* total, const int64_t* free, const GpuReq& req) {
  int64_t ns = 0, ws = 0;
  for (int r = 0; r < GS_NUM_GPU_RES; ++r) {
    if (!a.device_weights[r]) continue;       // resourceToWeightMap keys
    if (total[r] == 0) continue;
    int64_t rq = total[r];
    if (total[r] >= free[r]) rq = total[r] - free[r] + ((req.mask & (1u << r)) ? req.v[r] : 0);
    ns += (a.device_scoring_type == GS_SCORING_MOST_ALLOCATED ? ds_most(rq, total[r]) : ds_least(rq, total[r])) *
          a.device_weights[r];
    ws += a.device_weights[r];
  }
  return ws ? ns / ws : 0;
}

// DeviceShare Filter (plugin.go:272-322) on a node with a Device object: 0 ok, else GS_EXT_FAIL_DEVICE
// (numa: the node's NUMA affinity; the same check is DeviceShare.Allocate in the topology manager's Admit,
// topology_hint.go:57-106)
uint32_t ds_filter(const gs_node_devices& d, const GpuReq& pod, const orn::Hint* numa = nullptr) {
  GpuReq inst;
  int64_t count;
  if (gpu_desired(d, pod, &inst, &count) < 0) return GS_EXT_FAIL_DEVICE;
  NodeDev nd = filtered_node_device(d, numa);
  int64_t ok = 0;                              // defaultAllocateDevices (device_allocator.go:397-467), no scorer
  for (auto& kv : nd.free) {
    if (kv.second.zero()) continue;
    if (!le_request(inst, kv.second)) continue;
    if (++ok == count) break;
  }
  return ok < count ? GS_EXT_FAIL_DEVICE : 0u;
}

// DeviceShare Score (scoring.go:34-89) -> allocator.score (device_allocator.go:513-536)
int64_t ds_score(const gs_ext_args& a, const gs_node_devices& d, const GpuReq& pod, const orn::Hint* numa = nullptr) {
  GpuReq inst;
  int64_t count;
  if (gpu_desired(d, pod, &inst, &count) < 0) return 0;
  NodeDev nd = filtered_node_device(d, numa);
  if (nd.total.empty()) return 0;
  int64_t tot[GS_NUM_GPU_RES] = {0, 0, 0}, fr[GS_NUM_GPU_RES] = {0, 0, 0};
  for (auto& kv : nd.total)
    for (int r = 0; r < GS_NUM_GPU_RES; ++r) tot[r] += kv.second.v[r];
  for (auto& kv : nd.free)
    for (int r = 0; r < GS_NUM_GPU_RES; ++r) fr[r] += kv.second.v[r];
  return ds_scorer(a, tot, fr, inst);
}

// DeviceShare Reserve (plugin.go:377-430): defaultAllocateDevices with the scorer; minors sorted by device score
// descending, then minor (sortDeviceResourcesByMinor, device_resources.go:187-208). Returns the minors.
int ds_reserve(const gs_ext_args& a, gs_node_devices& d, const GpuReq& pod, gs_ext_placement* eo,
               const orn::Hint* numa = nullptr) {
  GpuReq inst;
  int64_t count;
  if (gpu_desired(d, pod, &inst, &count) < 0) return -1;
  NodeDev nd = filtered_node_device(d, numa);
  struct Pair { int minor; int64_t score; GpuRes free; };
  std::vector<Pair> ps;
  for (auto& kv : nd.free) ps.push_back({kv.first, ds_scorer(a, nd.total[kv.first].v, kv.second.v, inst), kv.second});
  std::stable_sort(ps.begin(), ps.end(), [](const Pair& x, const Pair& y) {
    if (x.score != y.score) return x.score > y.score;
    return x.minor < y.minor;
  });
  std::vector<int> minors;
  for (auto& p : ps) {
    if (p.free.zero() || !le_request(inst, p.free)) continue;
    minors.push_back(p.minor);
    if ((int64_t)minors.size() == count) break;
  }
  if ((int64_t)minors.size() < count) return -1;
  for (int mnr : minors) {                     // nodeDevice.updateCacheUsed -> updateDeviceUsed (device_cache.go:176-201)
    for (int g = 0; g < d.num_gpus; ++g) {
      if (d.gpus[g].minor != mnr) continue;
      for (int r = 0; r < GS_NUM_GPU_RES; ++r)
        if (inst.mask & (1u << r)) d.gpus[g].used[r] += inst.v[r];
    }
    eo->gpu_minor_mask |= 1u << mnr;
  }
  eo->gpu_count = (int32_t)count;
  for (int r = 0; r < GS_NUM_GPU_RES; ++r) eo->gpu_per_instance[r] = (inst.mask & (1u << r)) ? inst.v[r] : 0;
  return 0;
}

// DeviceShare as a NUMATopologyHintProvider: GetPodTopologyHints -> generateTopologyHints (topology_hint.go:33-55,
// 108-214), GPU type. false: the provider returns no hints (no Device object, Prepare fails, or no mask holds enough
// devices: an empty map, i.e. filterProvidersHints' preferred any-numa hint). true: *lists = one list per resource name
// of the per-instance request (gpu-core / gpu-memory-ratio / gpu-memory: identical lists, possibly empty), *names =
// those names (gs_gpu_res bits).
bool ds_topology_hints(const gs_node_devices& d, const GpuReq& pod, std::vector<std::vector<orn::Hint>>* lists,
                       uint32_t* names = nullptr) {
  lists->clear();
  if (names) *names = 0;
  if (!d.has_device || !pod.mask) return false;
  std::vector<int> ids;   // numaTopology.nodes keys (devices with a Topology), sorted (topology_hint.go:123-127)
  for (int g = 0; g < d.num_gpus && g < GS_MAX_GPUS; ++g)
    if (d.gpus[g].has_info && d.gpus[g].numa_node >= 0 && d.gpus[g].numa_node < 64) ids.push_back(d.gpus[g].numa_node);
  std::sort(ids.begin(), ids.end());
  ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
  GpuReq inst;
  int64_t count;
  if (gpu_desired(d, pod, &inst, &count) < 0) return false;   // allocator.Prepare fails for every mask
  int min_size = -1;
  std::vector<orn::Hint> hs;
  // bitmask.IterateBitMasks (util/bitmask/bitmask.go:206-222): sizes 1..n, combinations in lexicographic order
  std::vector<int> acc;
  std::function<void(size_t, int)> it = [&](size_t from, int size) {
    if ((int)acc.size() == size) {
      uint64_t m = 0;
      for (int id : acc) m |= 1ull << id;
      int64_t total = 0;   // calcTotalDevicesByNUMA (topology_hint.go:216-227)
      for (int g = 0; g < d.num_gpus && g < GS_MAX_GPUS; ++g)
        if (d.gpus[g].has_info && d.gpus[g].numa_node >= 0 && d.gpus[g].numa_node < 64 && (m >> d.gpus[g].numa_node & 1u))
          ++total;
      if (total < count) return;
      if (min_size < 0) min_size = (int)ids.size();   // minAffinitySize: len(numaNodes), then the smallest mask
      if (size < min_size) min_size = size;
      const orn::Hint aff{true, m, false, 0};
      if (ds_filter(d, pod, &aff) != 0) return;   // allocator.Allocate within the mask
      hs.push_back(aff);
      return;
    }
    for (size_t i = from; i < ids.size(); ++i) {
      acc.push_back(ids[i]);
      it(i + 1, size);
      acc.pop_back();
    }
  };
  for (int k = 1; k <= (int)ids.size(); ++k) it(0, k);
  if (min_size < 0) return false;   // minAffinitySize nil: no resource name gets a list
  for (orn::Hint& h : hs) h.preferred = __builtin_popcountll(h.mask) == min_size;
  for (int r = 0; r < GS_NUM_GPU_RES; ++r)   // one (identical) list per name: their order does not matter
    if (inst.mask >> r & 1u) lists->push_back(hs);
  if (names) *names = inst.mask;
  return true;
}

// ---- Reservation (reservation/*.go) ----
bool rsv_usable(const gs_reservation& r) {   // transformer.go:102-111
  if (!r.available) return false;
  if (r.allocate_once && r.assigned_pods > 0) return false;
  return true;
}
RList rsv_allocatable(const gs_reservation& r) { return rlist_of(r.allocatable, r.allocatable_mask); }
RList rsv_allocated(const gs_reservation& r) { return rlist_of(r.allocated, r.allocated_mask); }

// scoreReservation (scoring.go:183-203): MostAllocated over the non-zero Allocatable, milli values
int64_t score_reservation(const gs_pod& pod, const gs_reservation& r, const RList& allocated) {
  RList requested = rl_add(rlist_of(pod.requests, pod.request_mask), allocated);
  RList resources = rl_remove_zeros(rsv_allocatable(r));
  const int64_t w = (int64_t)resources.m.size();
  if (w <= 0) return 0;
  int64_t s = 0;
  for (auto& kv : resources.m) {
    const int64_t req = requested.get(kv.first);
    if (req <= kv.second) s += kMaxNodeScore * milli_value(kv.first, req) / milli_value(kv.first, kv.second);
  }
  return s / w;
}

// fitsNode (plugin.go:444-496) with preemptible = 0: the insufficient resource count
int fits_node(const gs_pod& pod, const gs_node& restored, const NodeRState& ns, const gs_reservation* r) {
  int bad = 0;
  if (restored.pod_count - (int64_t)ns.matched.size() + 1 > restored.allowed_pod_number) ++bad;
  const uint32_t scalars = pod.request_mask & GS_SCALAR_RES_MASK;
  if (!pod.requests[0] && !pod.requests[1] && !pod.requests[2] && !scalars) return bad;
  RList rem = r ? rl_sub(rsv_allocatable(*r), rsv_allocated(*r)) : RList{};
  for (int s = 0; s < GS_NUM_RES; ++s) {
    if (s >= 3 && !(scalars & (1u << s))) continue;
    if (s == GS_RES_RESERVED) continue;
    const int64_t avail = restored.allocatable[s] - (ns.pod_requested.requested[s] - rem.get(s) - ns.r_allocated.get(s));
    if (pod.requests[s] > avail) ++bad;
  }
  return bad;
}

// filterWithReservations (plugin.go:377-440): true = some reservation satisfies the pod
bool filter_with_reservations(const gs_pod& pod, const NodeRState& ns, const std::vector<const gs_reservation*>& rs) {
  const uint32_t pod_names = pod.request_mask;
  for (const gs_reservation* r : rs) {
    if (!(r->resource_names_mask & pod_names)) continue;
    const bool node_fits = fits_node(pod, ns.restored, ns, r) == 0;
    if (r->allocate_policy == GS_RSV_POLICY_DEFAULT || r->allocate_policy == GS_RSV_POLICY_ALIGNED) {
      if (node_fits) return true;
    } else if (r->allocate_policy == GS_RSV_POLICY_RESTRICTED) {
      RList allocated = rl_mask(rsv_allocated(*r), r->resource_names_mask);
      RList remained = rl_sub_nonneg(rsv_allocatable(*r), allocated);
      RList req = rl_mask(rlist_of(pod.requests, pod.request_mask), r->resource_names_mask);
      bool fits = true;
      for (auto& kv : req.m)
        if (kv.second > remained.get(kv.first)) fits = false;
      if (fits && node_fits) return true;
    }
  }
  return false;
}

// NominateReservation (nominator.go:140-190): filter each matched reservation (RunReservationFilterPlugins: the
// Reservation plugin's FilterReservation, plugin.go:503-530, and DeviceShare's, deviceshare/plugin.go:324-375), then
// the lowest order label, else the highest ScoreReservation (ties: the first in reservation order).
// device_pod: the pod requests devices (DeviceShare's PreFilter state is not skip). DeviceShare's FilterReservation
// then looks the reservation up in its restore state, which keeps only reservations holding device allocations
// (RestoreReservation's filterFn, deviceshare/reservation.go:133-162); a reservation without one fails with "impossible,
// there is no relevant Reservation information in deviceShare" and is not nominated. The reservations modelled here
// hold no devices, so a device pod nominates none.
const gs_reservation* nominate(const gs_pod& pod, const NodeRState& ns, bool device_pod = false) {
  if (device_pod) return nullptr;
  std::vector<const gs_reservation*> ok;
  for (const gs_reservation* r : ns.matched) {
    if (r->allocate_once && r->assigned_pods > 0) continue;
    if (!filter_with_reservations(pod, ns, {r})) continue;
    ok.push_back(r);
  }
  if (ok.empty()) return nullptr;
  const gs_reservation* best = nullptr;
  int64_t order = INT64_MAX;
  for (const gs_reservation* r : ok)   // findMostPreferredReservationByOrder (scoring.go:162-181)
    if (r->order != 0 && order > r->order) { order = r->order; best = r; }
  if (best) return best;
  int64_t bs = INT64_MIN;
  for (const gs_reservation* r : ok) {
    const int64_t s = score_reservation(pod, *r, rsv_allocated(*r));
    if (s > bs) { bs = s; best = r; }
  }
  return best;
}

// [upstream] pluginhelper.DefaultNormalizeScore(MaxNodeScore, false) / frameworkext.DefaultReservationNormalizeScore
void default_normalize(int64_t max_priority, bool reverse, std::vector<int64_t>& s) {
  int64_t mx = 0;
  for (int64_t v : s) mx = std::max(mx, v);
  if (mx == 0) {
    if (reverse) for (auto& v : s) v = max_priority;
    return;
  }
  for (auto& v : s) {
    v = max_priority * v / mx;
    if (reverse) v = max_priority - v;
  }
}

}  // namespace

extern "C" {

void or_ext_args_default(gs_ext_args* a) {
  std::memset(a, 0, sizeof(*a));
  a->enabled = GS_EXT_DEVICESHARE | GS_EXT_RESERVATION;
  a->device_scoring_type = GS_SCORING_LEAST_ALLOCATED;
  a->device_weights[GS_GPU_MEMORY_RATIO] = 1;
  a->weight_deviceshare = 1;
  a->weight_reservation = 5000;
}

int or_ext_configure(or_cluster* c, const gs_ext_args* a) {
  if (!c || !a) return GS_EINVAL;
  c->ext = *a;
  return GS_OK;
}

int or_node_devices_upsert(or_cluster* c, const uint32_t* idx, const gs_node_devices* d, uint32_t n) {
  if (!c || (n && !d)) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t k = idx ? idx[i] : i;
    if (k >= c->devices.size() || d[i].num_gpus < 0 || d[i].num_gpus > GS_MAX_GPUS) return GS_EINVAL;
    c->devices[k] = d[i];
  }
  return GS_OK;
}

int or_node_devices_get(or_cluster* c, uint32_t node, gs_node_devices* out) {
  if (!c || !out || node >= c->devices.size()) return GS_EINVAL;
  *out = c->devices[node];
  return GS_OK;
}

int or_reservations_upsert(or_cluster* c, const gs_reservation* r, uint32_t n) {
  if (!c || (n && !r)) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) {
    if (r[i].node >= c->nodes.size()) return GS_EINVAL;
    c->reservations[r[i].uid] = r[i];
  }
  return GS_OK;
}

int or_reservations_remove(or_cluster* c, const uint64_t* uids, uint32_t n) {
  if (!c || (n && !uids)) return GS_EINVAL;
  for (uint32_t i = 0; i < n; ++i) c->reservations.erase(uids[i]);
  return GS_OK;
}

int or_reservation_get(or_cluster* c, uint64_t uid, gs_reservation* out) {
  if (!c || !out) return GS_EINVAL;
  auto it = c->reservations.find(uid);
  if (it == c->reservations.end()) return 0;
  *out = it->second;
  return 1;
}

int64_t or_score_reservation(const gs_pod* pod, const gs_reservation* r) {
  return score_reservation(*pod, *r, rsv_allocated(*r));
}

int or_default_normalize_score(int64_t max_priority, int reverse, int64_t* scores, uint32_t n) {
  std::vector<int64_t> s(scores, scores + n);
  default_normalize(max_priority, reverse != 0, s);
  for (uint32_t i = 0; i < n; ++i) scores[i] = s[i];
  return GS_OK;
}

// Reservation PreScore + Score of one pod over `nnodes` nodes: node k's matched reservations are rsv[off[k]..off[k+1]),
// its restored NodeInfo nodes[k] and its podRequested view pod_requested[k] (fitsNode). raw[k] = Score (1000 for
// PreScore's preferred node, else the nominated reservation's scoreReservation, else 0).
int or_reservation_node_scores(const gs_pod* pod, const gs_reservation* rsv, const uint32_t* off, uint32_t nnodes,
                               const gs_node* nodes, const gs_node* pod_requested, int64_t* raw) {
  if (!pod || !off || !nodes || !pod_requested || !raw) return GS_EINVAL;
  int preferred = -1;
  int64_t sel = INT64_MAX;
  std::vector<NodeRState> ns(nnodes);
  for (uint32_t k = 0; k < nnodes; ++k) {
    ns[k].restored = nodes[k];
    ns[k].pod_requested = pod_requested[k];
    int64_t order = INT64_MAX;
    for (uint32_t j = off[k]; j < off[k + 1]; ++j) {
      ns[k].matched.push_back(&rsv[j]);
      ns[k].r_allocated = rl_add(ns[k].r_allocated, rsv_allocated(rsv[j]));
      if (rsv[j].order != 0 && order > rsv[j].order) order = rsv[j].order;
    }
    if (order != INT64_MAX && sel > order) { sel = order; preferred = (int)k; }
  }
  for (uint32_t k = 0; k < nnodes; ++k) {
    raw[k] = 0;
    if ((int)k == preferred) { raw[k] = 1000; continue; }
    const gs_reservation* r = ns[k].matched.empty() ? nullptr : nominate(*pod, ns[k]);
    if (r) raw[k] = score_reservation(*pod, *r, rsv_allocated(*r));
  }
  return GS_OK;
}

// DeviceShare Score of one pod on one node (PreFilter conversion + allocator.score)
int64_t or_device_score(const gs_ext_args* a, const gs_node_devices* d, const gs_pod_ext* e) {
  GpuReq q;
  if (gpu_pod_request(*e, &q) < 0 || !q.mask || !d->has_device) return 0;
  return ds_score(*a, *d, q);
}

// DeviceShare Filter of one pod on one node: 0 = pass, else GS_EXT_FAIL_DEVICE / GS_EXT_FAIL_POD
uint32_t or_device_filter(const gs_node_devices* d, const gs_pod_ext* e) {
  GpuReq q;
  if (gpu_pod_request(*e, &q) < 0) return GS_EXT_FAIL_POD;
  if (!q.mask || !d->has_device) return 0;
  return ds_filter(*d, q);
}

// DeviceShare GetPodTopologyHints on one node (topology_hint_test.go TestPlugin_GetPodTopologyHints, GPU cases):
// returns -1 invalid request, 0 no hints (an empty map), 1 hints: *names = resource names (gs_gpu_res bits) that each
// get the list (masks[k], preferred[k]) k < *count (over NUMA node ids)
int or_device_topology_hints(const gs_node_devices* d, const gs_pod_ext* e, uint64_t* masks, uint8_t* preferred,
                             uint32_t cap, uint32_t* count, uint32_t* names) {
  *count = 0;
  *names = 0;
  GpuReq q;
  if (gpu_pod_request(*e, &q) < 0) return -1;
  std::vector<std::vector<orn::Hint>> lists;
  if (!ds_topology_hints(*d, q, &lists, names)) return 0;
  const std::vector<orn::Hint>& l = lists[0];
  for (size_t k = 0; k < l.size(); ++k)
    if (k < cap) { masks[k] = l[k].mask; preferred[k] = l[k].preferred ? 1 : 0; }
  *count = (uint32_t)l.size();
  return 1;
}

// DeviceShare.Allocate with an affinity (topology_hint.go:57-106; TestPlugin_Allocate GPU cases): 0 ok, else
// GS_EXT_FAIL_DEVICE / GS_EXT_FAIL_POD
uint32_t or_device_allocate(const gs_node_devices* d, const gs_pod_ext* e, int has_mask, uint64_t mask) {
  GpuReq q;
  if (gpu_pod_request(*e, &q) < 0) return GS_EXT_FAIL_POD;
  if (!q.mask || !d->has_device) return 0;
  const orn::Hint aff{has_mask != 0, mask, false, 0};
  return ds_filter(*d, q, &aff);
}

int64_t or_device_score_node(const gs_ext_args* a, const int64_t* total, const int64_t* free, const int64_t* request,
                             uint32_t request_mask) {
  GpuReq q;
  for (int r = 0; r < GS_NUM_GPU_RES; ++r) q.v[r] = request[r];
  q.mask = request_mask;
  return ds_scorer(*a, total, free, q);
}

// scheduleOne with the extension plugins (one pod at a time, every node checked, no replay).
int or_schedule_ext(or_cluster* c, const gs_pod* pods, const gs_pod_ext* ext, uint32_t npods, const uint64_t* seq,
                    gs_placement* out, gs_ext_placement* ext_out) {
  if (!c || !out || (npods && !pods)) return GS_EINVAL;
  if (c->cfg.sample_nodes) return GS_EUNSUPPORTED;
  const int N = (int)c->nodes.size();
  for (int n = 0; n < N; ++n)
    if (!c->nodes[n].has_node) return GS_ESTATE;
  const uint32_t en = c->cfg.enabled;
  const bool ds_on = c->ext.enabled & GS_EXT_DEVICESHARE, rs_on = c->ext.enabled & GS_EXT_RESERVATION;
  std::vector<int64_t> base(N), dsr(N), rsr(N);
  std::vector<uint8_t> feasible(N);
  std::vector<orn::Hint> affinity(N);
  std::vector<NodeRState> rstate(N);
  std::vector<const gs_reservation*> nominated(N);
  // reservations by node, uid order
  std::vector<std::vector<gs_reservation*>> by_node(N);
  for (auto& kv : c->reservations) by_node[kv.second.node].push_back(&kv.second);
  for (uint32_t p = 0; p < npods; ++p) {
    const gs_pod& pod = pods[p];
    gs_pod_ext e{};
    if (ext) e = ext[p];
    gs_placement& o = out[p];
    gs_ext_placement eo{};
    o = gs_placement{-1, 0, 0, 0, 0};
    GpuReq gpu;
    if (ds_on && gpu_pod_request(e, &gpu) < 0) {   // DeviceShare PreFilter: UnschedulableAndUnresolvable
      eo.fail_code = GS_EXT_FAIL_POD;
      if (ext_out) ext_out[p] = eo;
      continue;
    }
    if (!ds_on) gpu = GpuReq{};
    const bool gpu_pod = gpu.mask != 0;
    const uint32_t gpu_names = gpu_pod ? (e.gpu_request_mask & 0x1Fu) : 0u;
    const uint32_t xres_names = e.xres_request_mask & ((1u << GS_MAX_XRES) - 1u);   // the caller's extended resources
    const orn::PreState st = orn::prefilter(c->numa_args, pod);
    // Reservation BeforePreFilter (transformer.go:50-235)
    bool any_state = false;
    for (int n = 0; n < N; ++n) {
      NodeRState& ns = rstate[n];
      ns = NodeRState{};
      ns.restored = c->nodes[n].node;
      if (!rs_on) continue;
      std::vector<const gs_reservation*> unmatched;
      for (const gs_reservation* r : by_node[n]) {
        if (!rsv_usable(*r)) continue;
        if (!r->unschedulable && e.reservation_owner != 0 && r->owner_key == e.reservation_owner) ns.matched.push_back(r);
        else if (r->assigned_pods > 0) unmatched.push_back(r);
      }
      if (ns.matched.empty() && unmatched.empty()) continue;
      if (e.reservation_required && ns.matched.empty()) continue;
      for (const gs_reservation* r : unmatched) {   // restoreUnmatchedReservations (:266-292)
        update_requested(ns.restored, rsv_allocatable(*r), -1);
        RList rem = rl_sub_nonneg(rsv_allocatable(*r), rsv_allocated(*r));
        if (!rem.is_zero()) update_requested(ns.restored, rem, +1);
      }
      ns.pod_requested = ns.restored;
      for (const gs_reservation* r : ns.matched) {   // restoreMatchedReservation (:241-264): RemovePod(reservePod)
        update_requested(ns.restored, rsv_allocatable(*r), -1);
        ns.restored.pod_count -= 1;
        ns.r_allocated = rl_add(ns.r_allocated, rsv_allocated(*r));
      }
      ns.has = true;
      any_state = true;
    }
    if (rs_on && e.reservation_required && !any_state) {   // PreFilter: ErrReasonReservationAffinity
      if (ext_out) ext_out[p] = eo;
      continue;
    }
    // Filter
    std::vector<int> fl;
    for (int n = 0; n < N; ++n) {
      const NodeState& s = c->nodes[n];
      const gs_node& nd = rstate[n].restored;
      uint32_t code = 0;
      if (en & GS_ENABLE_FIT_FILTER) {
        code |= fit_filter(pod, nd);
        if (gpu_pod || xres_names) {   // GPU names / extended resources are scalars ([upstream] fit.go fitsRequest)
          const gs_node_devices& d = c->devices[n];
          if (!pod.requests[0] && !pod.requests[1] && !pod.requests[2] && !(pod.request_mask & GS_SCALAR_RES_MASK)) {
            // fit_filter returned early on an all-zero request: the scalar GPU names make it non-zero
            if (pod.requests[0] > nd.allocatable[0] - nd.requested[0]) code |= GS_FAIL_FIT_CPU;
            if (pod.requests[1] > nd.allocatable[1] - nd.requested[1]) code |= GS_FAIL_FIT_MEMORY;
            if (pod.requests[2] > nd.allocatable[2] - nd.requested[2]) code |= GS_FAIL_FIT_EPHEMERAL;
          }
          for (int g = 0; g < GS_NUM_GPU_NAMES; ++g) {
            if (!(gpu_names & (1u << g))) continue;
            if (c->ext.fit_ignored_gpu_names & (1u << g)) continue;   // IgnoredResources / IgnoredResourceGroups
            const int64_t a = d.allocatable[g], r = d.requested[g];
            if (e.gpu_requests[g] > a - r) code |= GS_FAIL_FIT_SCALAR;
          }
          for (int x = 0; x < GS_MAX_XRES; ++x) {
            if (!(xres_names & (1u << x)) || (c->ext.fit_ignored_xres & (1u << x))) continue;
            if (e.xres_requests[x] > d.xres_allocatable[x] - d.xres_requested[x]) code |= GS_FAIL_FIT_SCALAR;
          }
        }
      }
      if (en & GS_ENABLE_LA_FILTER) code |= loadaware_filter(*c, pod, s);
      affinity[n] = orn::Hint{};
      if (!code && (en & GS_ENABLE_NUMA_FILTER)) {
        bool has = false;
        std::vector<std::vector<orn::Hint>> p2;   // DeviceShare's hints (the second provider) on NUMA-policy nodes
        if (gpu_pod && c->numa[n].opts.numa_policy != GS_NUMA_POLICY_NONE) ds_topology_hints(c->devices[n], gpu, &p2);
        int reason = orn::filter(c->numa_args, st, c->numa[n], node_view(nd), &affinity[n], &has, c->reverse_hint_order,
                                 &p2);
        if (!has) affinity[n] = orn::Hint{};
        code |= (uint32_t)reason << GS_FAIL_NUMA_SHIFT;
      }
      if (!code && gpu_pod && c->devices[n].has_device) code |= ds_filter(c->devices[n], gpu, &affinity[n]);
      if (!code && rs_on) {   // Reservation Filter (plugin.go:311-375), non-reserve pods
        const NodeRState& ns = rstate[n];
        if (ns.matched.empty()) {
          if (e.reservation_required) code |= GS_EXT_FAIL_RESERVATION;
        } else if (e.reservation_required && !filter_with_reservations(pod, ns, ns.matched)) {
          code |= GS_EXT_FAIL_RESERVATION;
        }
      }
      feasible[n] = code == 0;
      if (!code) fl.push_back(n);
    }
    o.feasible = (uint32_t)fl.size();
    if (fl.empty()) {
      if (ext_out) ext_out[p] = eo;
      continue;
    }
    // PreScore (Reservation, scoring.go:42-101): nominations + the preferred node (lowest order, first in feasible order)
    int preferred = -1;
    int64_t sel_order = INT64_MAX;
    for (int n : fl) {
      nominated[n] = nullptr;
      const NodeRState& ns = rstate[n];
      if (!rs_on || ns.matched.empty()) continue;
      int64_t order = INT64_MAX;
      for (const gs_reservation* r : ns.matched)
        if (r->order != 0 && order > r->order) order = r->order;
      if (order != INT64_MAX && order != 0 && sel_order > order) { sel_order = order; preferred = n; }
      nominated[n] = nominate(pod, ns, gpu_pod);
    }
    // Score + NormalizeScore + weights
    const int F = (int)fl.size();
    std::vector<int64_t> dsl(F), rsl(F);
    for (int i = 0; i < F; ++i) {
      const int n = fl[i];
      const gs_node& nd = rstate[n].restored;
      PairResult r{0, 0, 0, 0};
      if (en & GS_ENABLE_FIT_SCORE) r.fit = fit_score(c->cfg.fit, pod, nd);
      if (en & GS_ENABLE_LA_SCORE) r.la = loadaware_score(*c, pod, c->nodes[n]);
      if (en & GS_ENABLE_NUMA_SCORE) r.numa = orn::score(c->numa_args, st, c->numa[n], node_view(nd), affinity[n]);
      base[n] = weighted_total(*c, r);
      dsl[i] = (gpu_pod && c->devices[n].has_device) ? ds_score(c->ext, c->devices[n], gpu, &affinity[n]) : 0;
      int64_t rs = 0;
      if (rs_on) {
        if (n == preferred) rs = 1000;   // mostPreferredScore
        else if (nominated[n]) rs = score_reservation(pod, *nominated[n], rsv_allocated(*nominated[n]));
      }
      rsl[i] = rs;
    }
    if (ds_on) default_normalize(kMaxNodeScore, false, dsl);
    if (rs_on) default_normalize(kMaxNodeScore, false, rsl);
    std::vector<int64_t> total(F);
    for (int i = 0; i < F; ++i)
      total[i] = base[fl[i]] + (ds_on ? dsl[i] * c->ext.weight_deviceshare : 0) +
                 (rs_on ? rsl[i] * c->ext.weight_reservation : 0);
    // selectHost
    TieBreakRand rnd(c->cfg.seed, seq ? seq[p] : p);
    int si = 0;
    int64_t mx = total[0], cnt = 1;
    for (int i = 1; i < F; ++i) {
      if (total[i] > mx) { mx = total[i]; si = i; cnt = 1; }
      else if (total[i] == mx) { ++cnt; if (rnd.intn(cnt) == 0) si = i; }
    }
    const int selected = fl[si];
    o.node = selected; o.score = mx; o.ties = (uint32_t)cnt;
    eo.deviceshare_score = (int32_t)dsl[si];
    eo.reservation_score = (int32_t)rsl[si];
    // Reserve: NodeNUMAResource, DeviceShare, Reservation; then assume
    if (en & (GS_ENABLE_NUMA_FILTER | GS_ENABLE_NUMA_SCORE)) {
      orn::PodAllocation pa;
      if (orn::reserve(c->numa_args, st, c->numa[selected], pod, affinity[selected], &pa) != 0) return GS_ESTATE;
      if (!pa.numa.empty()) o.flags |= GS_PLACED_NUMA;
      if (!pa.cpus.empty()) o.flags |= GS_PLACED_CPUSET;
    }
    gs_node_devices& dv = c->devices[selected];
    if (gpu_pod && dv.has_device && ds_reserve(c->ext, dv, gpu, &eo, &affinity[selected]) != 0) return GS_ESTATE;
    if (rs_on) {
      const gs_reservation* nr = nominated[selected];
      if (nr) {   // reservationCache.assumePod -> ReservationInfo.AddAssignedPod (reservation_info.go:379-388)
        gs_reservation& rr = c->reservations[nr->uid];
        RList add = rl_mask(rlist_of(pod.requests, pod.request_mask), rr.resource_names_mask);
        RList na = rl_add(rsv_allocated(rr), add);
        for (auto& kv : na.m) rr.allocated[kv.first] = kv.second;
        rr.allocated_mask |= rl_names(na);
        rr.assigned_pods += 1;
        eo.reservation_uid = rr.uid;
      }
    }
    gs_node& nd = c->nodes[selected].node;   // NodeInfo.AddPod
    for (int r = 0; r < GS_NUM_RES; ++r) nd.requested[r] += pod.requests[r];
    nd.nonzero_requested[0] += pod.nonzero_requests[0];
    nd.nonzero_requested[1] += pod.nonzero_requests[1];
    nd.pod_count += 1;
    for (int g = 0; g < GS_NUM_GPU_NAMES; ++g)
      if (gpu_names & (1u << g)) dv.requested[g] += e.gpu_requests[g];
    for (int x = 0; x < GS_MAX_XRES; ++x)
      if (xres_names & (1u << x)) dv.xres_requested[x] += e.xres_requests[x];
    if (!(pod.flags & GS_POD_TERMINATED)) c->nodes[selected].assigned[pod.uid] = AssignInfo{c->now, pod};
    if (ext_out) ext_out[p] = eo;
  }
  return GS_OK;
}

}  // extern "C"
