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
