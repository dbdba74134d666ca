"""Writes tests/golden/quota.json: the ElasticQuota vectors of the reference's own tests, transcribed as data
(inputs and the asserted outputs). cpu in milli (createResourceList: NewMilliQuantity(cpu*1000)), memory and
GPUs as Value(). Run from the repo root: python tests/golden/make_golden_quota.py"""
import json
import os


def rl(cpu=None, mem=None, gpu=None):
    out = {}
    if cpu is not None:
        out["cpu"] = cpu * 1000
    if mem is not None:
        out["memory"] = mem
    if gpu is not None:
        out["nvidia.com/gpu"] = gpu
    return out


G = {
    # core/runtime_quota_calculator_test.go:132-154 TestRuntimeQuotaCalculator_Iteration4AdjustQuota:
    # insert(name, sharedWeight, request, min, guarantee, allowLent), total cpu 100 milli
    "redistribution": [
        {"name": "Iteration4AdjustQuota", "total": 100,
         "nodes": [[40, 5, 10, 0, True], [60, 20, 15, 0, True], [50, 40, 20, 0, True], [80, 70, 15, 0, True]],
         "runtime": [5, 20, 35, 40]},
    ],
    # two quotas under one parent (the calculator tests drive one RuntimeQuotaCalculator directly):
    # core/runtime_quota_calculator_test.go:328-379 (UpdateOneGroupRuntimeQuota, three steps) and :381-422
    # (UpdateOneGroupRuntimeQuota2). sharedWeight (1, 1) in all of them.
    "runtime": [
        {"name": "UpdateOneGroupRuntimeQuota/step1", "total": rl(100, 1000),
         "quotas": [{"name": "test1", "max": rl(80, 800), "min": rl(60, 600), "shared_weight": rl(1, 1), "request": {}},
                    {"name": "test2", "max": rl(100, 1000), "min": rl(50, 500), "shared_weight": rl(1, 1),
                     "request": rl(90, 900)}],
         "runtime": {"test1": rl(0, 0), "test2": rl(90, 900)}},
        {"name": "UpdateOneGroupRuntimeQuota/step2", "total": rl(100, 1000),
         "quotas": [{"name": "test1", "max": rl(80, 800), "min": rl(60, 600), "shared_weight": rl(1, 1),
                     "request": rl(30, 300)},
                    {"name": "test2", "max": rl(100, 1000), "min": rl(50, 500), "shared_weight": rl(1, 1),
                     "request": rl(90, 900)}],
         "runtime": {"test1": rl(30, 300), "test2": rl(70, 700)}},
        {"name": "UpdateOneGroupRuntimeQuota/step3", "total": rl(100, 1000),
         "quotas": [{"name": "test1", "max": rl(80, 800), "min": rl(60, 600), "shared_weight": rl(1, 1),
                     "request": rl(60, 600)},
                    {"name": "test2", "max": rl(100, 1000), "min": rl(50, 500), "shared_weight": rl(1, 1),
                     "request": rl(90, 900)}],
         "runtime": {"test1": rl(60, 600), "test2": rl(50, 500)}},
        {"name": "UpdateOneGroupRuntimeQuota2/alone", "total": rl(120, 1200),
         "quotas": [{"name": "test1", "max": rl(80, 800), "min": rl(50, 500), "shared_weight": rl(1, 1),
                     "request": rl(100, 1000)}],
         "runtime": {"test1": rl(80, 800)}},
        {"name": "UpdateOneGroupRuntimeQuota2/both", "total": rl(120, 1200),
         "quotas": [{"name": "test1", "max": rl(80, 800), "min": rl(50, 500), "shared_weight": rl(1, 1),
                     "request": rl(100, 1000)},
                    {"name": "test2", "max": rl(100, 1000), "min": rl(50, 500), "shared_weight": rl(1, 1),
                     "request": rl(150, 1500)}],
         "runtime": {"test1": rl(60, 600), "test2": rl(60, 600)}},
    ],
    # plugin_test.go:603-699 TestPlugin_PreFilter (runtime set directly on the default quota, used empty)
    "prefilter_runtime": [
        {"name": "default", "request": rl(1, 2, 1), "runtime": rl(0, 20, 10), "max": None, "runtime_quota": True,
         "code": "Unschedulable", "exceed": ["cpu"]},
        {"name": "used dimension larger than runtime, but value is enough", "request": rl(1, 2, 1),
         "runtime": rl(10, 20, 10), "max": None, "runtime_quota": True, "code": "Success", "exceed": []},
        {"name": "value not enough", "request": rl(1, 3, 1), "runtime": rl(1, 2), "max": None,
         "runtime_quota": True, "code": "Unschedulable", "exceed": ["memory"]},
        {"name": "runtime not enough, but disable runtime", "request": rl(1, 3, 1), "runtime": rl(1, 2),
         "max": rl(1, 3), "runtime_quota": False, "code": "Success", "exceed": []},
    ],
    # plugin_test.go:701-767 TestPlugin_PreFilter_CheckParent
    "prefilter_check_parent": [
        {"name": "parent reject", "request": rl(1, 3, 1),
         "child": {"name": "test-child", "max": rl(10, 30, 10), "min": rl(0, 0, 0), "runtime": rl(1, 3, 1)},
         "parent": {"name": "test", "max": rl(10, 30, 10), "min": rl(0, 0, 0), "runtime": rl(1, 2, 1)},
         "code": "Unschedulable", "failed": "test", "topo": ["test", "test-child"], "exceed": ["memory"]},
    ],
    # plugin_test.go:769-876 TestPlugin_Prefilter_QuotaNonPreempt: pods (name, quota, priority, cpu, mem,
    # nonPreempt); init pods assigned, the pod under test added unassigned, then PreFilter with runtime refresh.
    "prefilter_non_preemptible": [
        {"name": "default", "total": rl(10, 10),
         "quota": {"name": "test1", "max": rl(10, 10), "min": rl(5, 5)},
         "init_pods": [[2, 1, False], [1, 1, False], [1, 1, False]], "pod": [2, 2, True],
         "code": "Success", "exceed": [], "runtime": rl(6, 5)},
        {"name": "non-preemptible pod used larger than min", "total": rl(8, 5),
         "quota": {"name": "test1", "max": rl(10, 8), "min": rl(5, 5)},
         "init_pods": [[2, 1, False], [2, 1, True], [2, 1, True]], "pod": [2, 2, True],
         "code": "Unschedulable", "reason": "Insufficient non-preemptible quotas", "exceed": ["cpu"],
         "message": "Insufficient non-preemptible quotas, quotaName: test1, min: cpu:5,memory:5, "
                    "nonPreemptibleUsed: cpu:4,memory:2, pod's request: cpu:2,memory:2, exceedDimensions: [cpu]"},
        {"name": "non-preemptible pod will not be evicted", "total": rl(7, 5),
         "quota": {"name": "test1", "max": rl(10, 8), "min": rl(5, 5)},
         "init_pods": [[2, 1, False], [2, 1, False], [2, 2, True]], "pod": [2, 1, True],
         "code": "Unschedulable", "reason": "Insufficient quotas", "exceed": ["cpu"], "runtime": rl(7, 5),
         "message": "Insufficient quotas, quotaName: test1, runtime: cpu:7,memory:5, used: cpu:6,memory:4, "
                    "pod's request: cpu:2,memory:1, exceedDimensions: [cpu]"},
    ],
}

if __name__ == "__main__":
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "quota.json")
    with open(path, "w") as f:
        json.dump(G, f, indent=1)
    print("wrote", path)
