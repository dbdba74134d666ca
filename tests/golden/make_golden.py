"""Writes tests/golden/loadaware.json: the reference's own LoadAware test vectors, transcribed.

The reference (Go) cannot run here (no Go toolchain), so these fixtures are transcriptions of the
table-driven tests in hormes/koordinator — inputs as Kubernetes-shaped specs, expected outputs as the
tests assert them. Each case carries the file:line of its source. Times are relative to `now`
(seconds); the Go tests build them from time.Now() in struct-literal order, which is reproduced
with sub-microsecond offsets where the order matters (see "just assigned" cases).

Run: python tests/golden/make_golden.py   (regenerates the JSON; the JSON is what tests read)
"""
import json
import os

LA = "pkg/scheduler/plugins/loadaware/load_aware_test.go"
EST = "pkg/scheduler/plugins/loadaware/estimator/default_estimator_test.go"

NODE_96 = {"allocatable": {"cpu": "96", "memory": "512Gi"}}


def c(req=None, lim=None):
    d = {}
    if req is not None:
        d["requests"] = req
    if lim is not None:
        d["limits"] = lim
    return d


G16 = {"cpu": "16", "memory": "32Gi"}
POD_16 = {"namespace": "default", "name": "test-pod-1", "containers": [c(G16, G16)]}


def metric(update=0.0, node_usage=None, aggregated=None, pods_metric=None, node_metric=True):
    m = {"update_time_rel": update, "report_interval_s": 60}
    if node_metric:
        m["node_metric"] = {"node_usage": node_usage or {}, "aggregated": aggregated or []}
    if pods_metric:
        m["pods_metric"] = pods_metric
    return m


def usage(cpu, mem):
    return {"cpu": cpu, "memory": mem}


estimate_pod = [
    {"src": f"{EST}:40-56", "name": "estimate empty pod",
     "pod": {"containers": [c()]}, "want": [250, 209715200]},
    {"src": f"{EST}:57-81", "name": "estimate guaranteed pod",
     "pod": {"containers": [c({"cpu": "4", "memory": "8Gi"}, {"cpu": "4", "memory": "8Gi"})]},
     "want": [3400, 6012954214]},
    {"src": f"{EST}:82-106", "name": "estimate burstable pod",
     "pod": {"containers": [c({"cpu": "4", "memory": "8Gi"}, {"cpu": "8", "memory": "8Gi"})]},
     "want": [8000, 6012954214]},
    {"src": f"{EST}:107-134", "name": "estimate guaranteed pod and zoomed cpu factors",
     "scaling": {"cpu": 110},
     "pod": {"containers": [c({"cpu": "4", "memory": "8Gi"}, {"cpu": "4", "memory": "8Gi"})]},
     "want": [4000, 6012954214]},
    {"src": f"{EST}:135-162", "name": "estimate guaranteed pod and zoomed memory factors",
     "scaling": {"memory": 110},
     "pod": {"containers": [c({"cpu": "4", "memory": "8Gi"}, {"cpu": "4", "memory": "8Gi"})]},
     "want": [3400, 8589934592]},
    {"src": f"{EST}:163-193", "name": "estimate Batch pod",
     "pod": {"labels": {"koordinator.sh/qosClass": "BE"}, "priority": 5000,
             "containers": [c({"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"},
                              {"kubernetes.io/batch-cpu": "4000", "kubernetes.io/batch-memory": "8Gi"})]},
     "want": [3400, 6012954214]},
    {"src": f"{EST}:194-222", "name": "estimate pod only has request",
     "scaling": {"cpu": 80, "memory": 80},
     "pod": {"labels": {"koordinator.sh/qosClass": "LS"}, "priority": 9999,
             "containers": [c({"cpu": "4", "memory": "8Gi"})]},
     "want": [3200, 6871947674]},
]

estimate_node = [
    {"src": f"{EST}:258-272", "name": "estimate empty node",
     "node": {"allocatable": {"cpu": "32"}}, "want": [32000, 0]},
    {"src": f"{EST}:273-292", "name": "estimate node with original allocatable",
     "node": {"allocatable": {"cpu": "32", "memory": "42Gi"},
              "annotations": {"raw_allocatable": {"cpu": 28, "memory": "32Gi"}}},
     "want": [28000, 34359738368]},
    {"src": f"{EST}:293-312", "name": "estimate node with original allocatable and sames",
     "node": {"allocatable": {"cpu": "32", "memory": "42Gi"},
              "annotations": {"raw_allocatable": {"cpu": 32, "memory": "42Gi"}}},
     "want": [32000, 45097156608]},
]

filter_expired = [
    {"src": f"{LA}:147-164", "name": "filter healthy nodeMetrics",
     "metric": {"update_time_rel": 0.0, "report_interval_s": 60}, "want_fail": False},
    {"src": f"{LA}:165-178", "name": "filter unhealthy nodeMetric with nil updateTime",
     "metric": {"update_time_rel": None, "report_interval_s": 60}, "want_fail": False},
    {"src": f"{LA}:179-197", "name": "filter unhealthy nodeMetric with expired updateTime",
     "metric": {"update_time_rel": -180.0, "report_interval_s": 60}, "want_fail": False},
]

PROD_PODS = [{"namespace": "default", "name": "prod-pod-1", "priority": 9999},
             {"namespace": "default", "name": "prod-pod-2", "priority": 9999}]
PROD_METRICS = [{"name": "prod-pod-1", "usage": usage("30", "200Gi")},
                {"name": "prod-pod-2", "usage": usage("33", "300Gi")}]
PROD_TEST_POD = {"namespace": "default", "name": "prod-pod-3", "priority": 9999}

filter_usage = [
    {"src": f"{LA}:275-301", "name": "filter normal usage",
     "metric": metric(node_usage=usage("60", "256Gi")), "want_fail": False},
    {"src": f"{LA}:302-306", "name": "filter node missing NodeMetrics", "metric": None, "want_fail": False},
    {"src": f"{LA}:307-333", "name": "filter exceed cpu usage",
     "metric": metric(node_usage=usage("70", "256Gi")), "want_fail": True,
     "want_msg": "node(s) cpu usage exceed threshold"},
    {"src": f"{LA}:334-380", "name": "filter exceed p95 cpu usage",
     "args": {"aggregated": {"usageThresholds": {"cpu": 60}, "usageAggregationType": "p95",
                             "usageAggregatedDurationSeconds": 300}},
     "metric": metric(node_usage=usage("30", "100Gi"),
                      aggregated=[{"duration_s": 300, "usage": {"p95": usage("70", "256Gi")}}]),
     "want_fail": True, "want_msg": "node(s) cpu aggregated usage exceed threshold"},
    {"src": f"{LA}:381-407", "name": "filter exceed memory usage",
     "metric": metric(node_usage=usage("30", "500Gi")), "want_fail": True,
     "want_msg": "node(s) memory usage exceed threshold"},
    {"src": f"{LA}:408-437", "name": "filter exceed memory usage by custom usage thresholds",
     "custom": {"usageThresholds": {"memory": 60}},
     "metric": metric(node_usage=usage("30", "316Gi")), "want_fail": True,
     "want_msg": "node(s) memory usage exceed threshold"},
    {"src": f"{LA}:438-482", "name": "filter exceed p95 cpu usage by custom usage",
     "custom": {"aggregatedUsage": {"usageThresholds": {"cpu": 60}, "usageAggregationType": "p95",
                                    "usageAggregatedDurationSeconds": 300}},
     "metric": metric(node_usage=usage("30", "100Gi"),
                      aggregated=[{"duration_s": 300, "usage": {"p95": usage("70", "256Gi")}}]),
     "want_fail": True, "want_msg": "node(s) cpu aggregated usage exceed threshold"},
    {"src": f"{LA}:483-509", "name": "disable filter exceed memory usage",
     "args": {"usageThresholds": {"memory": 0}},
     "metric": metric(node_usage=usage("30", "500Gi")), "want_fail": False},
    {"src": f"{LA}:510-556", "name": "prod usage filter is not enabled by default",
     "args": {"usageThresholds": {"cpu": 100, "memory": 100}},
     "metric": metric(node_usage=usage("63", "500Gi"), pods_metric=PROD_METRICS),
     "lister": PROD_PODS, "want_fail": False},
    {"src": f"{LA}:557-609", "name": "filter prod cpu usage",
     "args": {"usageThresholds": {"cpu": 100, "memory": 100}, "prodUsageThresholds": {"cpu": 50, "memory": 100}},
     "metric": metric(node_usage=usage("63", "500Gi"), pods_metric=PROD_METRICS),
     "lister": PROD_PODS, "pod": PROD_TEST_POD, "want_fail": True, "want_msg": "node(s) cpu usage exceed threshold"},
    {"src": f"{LA}:610-662", "name": "filter prod memory usage",
     "args": {"usageThresholds": {"cpu": 100, "memory": 100}, "prodUsageThresholds": {"cpu": 100, "memory": 50}},
     "metric": metric(node_usage=usage("63", "500Gi"), pods_metric=PROD_METRICS),
     "lister": PROD_PODS, "pod": PROD_TEST_POD, "want_fail": True, "want_msg": "node(s) memory usage exceed threshold"},
    {"src": f"{LA}:663-719", "name": "filter prod memory usage with custom usage configuration",
     "args": {"usageThresholds": {"cpu": 100, "memory": 100}, "prodUsageThresholds": {"cpu": 100, "memory": 100}},
     "custom": {"prodUsageThresholds": {"cpu": 100, "memory": 50}},
     "metric": metric(node_usage=usage("63", "500Gi"), pods_metric=PROD_METRICS),
     "lister": PROD_PODS, "pod": PROD_TEST_POD, "want_fail": True, "want_msg": "node(s) memory usage exceed threshold"},
    {"src": f"{LA}:720-746", "name": "filter daemonset pod exceed cpu usage",
     "metric": metric(node_usage=usage("70", "256Gi")),
     "pod": {"namespace": "default", "name": "test-pod", "priority": 9999, "daemonset": True},
     "want_fail": False},
]
# want_msg: the wantStatus message of the case (load_aware_test.go:335,383,411,442,490,642,705,772)
for case in filter_usage:   # TestFilterUsage runs with FilterExpiredNodeMetrics = false (:748)
    case.setdefault("args", {})["filterExpiredNodeMetrics"] = False

ASSIGNED_16 = {"namespace": "default", "name": "assigned-pod-1", "containers": [c(G16, G16)]}

score = [
    {"src": f"{LA}:925-944", "name": "score node with expired nodeMetric",
     "metric": {"update_time_rel": -180.0, "report_interval_s": 60}, "pod": {}, "want": 0},
    {"src": f"{LA}:945-987", "name": "score empty node",
     "metric": metric(node_metric=False), "pod": POD_16, "want": 90},
    {"src": f"{LA}:988-1019", "name": "score node missing NodeMetrics",
     "metric": None, "pod": POD_16, "want": 0},
    {"src": f"{LA}:1020-1070", "name": "score load node",
     "metric": metric(node_usage=usage("32", "10Gi")), "pod": POD_16, "want": 72},
    {"src": f"{LA}:1071-1137", "name": "score load node with p95",
     "args": {"aggregated": {"scoreAggregationType": "p95", "scoreAggregatedDurationSeconds": 300}},
     "metric": metric(node_usage=usage("0", "0Gi"),
                      aggregated=[{"duration_s": 300, "usage": {"p95": usage("32", "10Gi"),
                                                                "p99": usage("50", "70Gi")}}]),
     "pod": POD_16, "want": 72},
    {"src": f"{LA}:1138-1186", "name": "score load node with p95 but have not reported usage",
     "args": {"aggregated": {"scoreAggregationType": "p95", "scoreAggregatedDurationSeconds": 300}},
     "metric": metric(node_usage=usage("0", "0Gi")), "pod": POD_16, "want": 90},
    {"src": f"{LA}:1187-1299",
     "name": "score load node with p95 but have not reported usage and have assigned pods",
     "args": {"aggregated": {"scoreAggregationType": "p95", "scoreAggregatedDurationSeconds": 300}},
     "assigned": [{"pod": ASSIGNED_16, "ts_rel": -600.0}],
     "metric": metric(node_usage=usage("0", "0Gi"),
                      pods_metric=[{"name": "assigned-pod-1", "usage": usage("1", "1Gi")}]),
     "pod": POD_16, "want": 81},
    {"src": f"{LA}:1300-1379", "name": "score load node with just assigned pod",
     "assigned": [{"pod": ASSIGNED_16, "ts_rel": -1e-6}],
     "metric": metric(node_usage=usage("32", "10Gi")), "pod": POD_16, "want": 63},
    {"src": f"{LA}:1380-1459", "name": "score load node with just assigned pod where after updateTime",
     "assigned": [{"pod": ASSIGNED_16, "ts_rel": 0.0}],
     "metric": metric(update=-10.0, node_usage=usage("32", "10Gi")), "pod": POD_16, "want": 63},
    {"src": f"{LA}:1460-1539", "name": "score load node with just assigned pod where before updateTime",
     "assigned": [{"pod": ASSIGNED_16, "ts_rel": -10.0}],
     "metric": metric(node_usage=usage("32", "10Gi")), "pod": POD_16, "want": 63},
    {"src": f"{LA}:1540-1583", "name": "score batch Pod",
     "metric": metric(node_metric=False),
     "pod": {"namespace": "default", "name": "test-pod-1", "priority": 5000,
             "containers": [c({"kubernetes.io/batch-cpu": "16000", "kubernetes.io/batch-memory": "32Gi"},
                              {"kubernetes.io/batch-cpu": "16000", "kubernetes.io/batch-memory": "32Gi"})]},
     "want": 90},
    {"src": f"{LA}:1584-1663", "name": "score prod Pod",
     "args": {"scoreAccordingProdUsage": True},
     "assigned": [{"pod": {"namespace": "default", "name": "assign-prod-pod-1", "priority": 9999,
                           "containers": [c(G16, G16)]}, "ts_rel": -1e-6}],
     "metric": metric(node_metric=False,
                      pods_metric=[{"name": "assign-prod-pod-1", "usage": usage("30", "100Gi")}]),
     "pod": {"namespace": "default", "name": "prod-pod-1", "priority": 9999,
             "containers": [c({"cpu": "16000", "memory": "32Gi"}, {"cpu": "16000", "memory": "32Gi"})]},
     "want": 38},
    {"src": f"{LA}:1664-1701", "name": "score request less than limit",
     "metric": metric(node_metric=False),
     "pod": {"namespace": "default", "name": "test-pod-1",
             "containers": [c({"cpu": "8", "memory": "16Gi"}, G16)]},
     "want": 88},
    {"src": f"{LA}:1702-1733", "name": "score empty pod",
     "metric": metric(node_metric=False),
     "pod": {"namespace": "default", "name": "test-pod-1", "containers": [c()]}, "want": 99},
]
for case in score:   # TestScore: the scheduled pod and every assigned pod are in the pod lister (:1804-1814)
    case["node"] = NODE_96

for case in filter_usage + filter_expired:
    case.setdefault("node", NODE_96 if case in filter_usage else {"allocatable": {}})

fixtures = {
    "estimate_pod": estimate_pod,
    "estimate_node": estimate_node,
    "filter_expired": filter_expired,
    "filter_usage": filter_usage,
    "score": score,
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "loadaware.json")
    with open(out, "w") as f:
        json.dump(fixtures, f, indent=1)
    print("wrote", out, {k: len(v) for k, v in fixtures.items()})
