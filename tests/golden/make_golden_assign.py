"""Generates tests/golden/assign_cache.json: the podAssignCache informer-handler vectors of
pkg/scheduler/plugins/loadaware/pod_assign_cache_test.go, transcribed by hand into data. A pod is (node: 0 for
Spec.NodeName "test-node", -1 for ""; terminated: Status.Phase Failed; uid); the cache is the list of uids on
"test-node", each stamped with timeNowFn (the injected now).

    python tests/golden/make_golden_assign.py
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assign_cache.json")
UID = 123456789


def main():
    cases = [
        {"name": "OnAdd update pending pod", "src": "loadaware/pod_assign_cache_test.go:42-46", "event": "add",
         "pod": {"node": -1, "terminated": False, "uid": 1}, "cache": [], "want": []},
        {"name": "OnAdd update terminated pod", "src": "loadaware/pod_assign_cache_test.go:47-58", "event": "add",
         "pod": {"node": 0, "terminated": True, "uid": 2}, "cache": [], "want": []},
        {"name": "OnAdd update scheduled running pod", "src": "loadaware/pod_assign_cache_test.go:59-92",
         "event": "add", "pod": {"node": 0, "terminated": False, "uid": UID}, "cache": [], "want": [UID]},
        {"name": "OnUpdate update pending pod", "src": "loadaware/pod_assign_cache_test.go:117-121",
         "event": "update", "pod": {"node": -1, "terminated": False, "uid": 1}, "cache": [], "want": []},
        {"name": "OnUpdate update terminated pod", "src": "loadaware/pod_assign_cache_test.go:122-159",
         "event": "update", "pod": {"node": 0, "terminated": True, "uid": UID}, "cache": [UID], "want": []},
        {"name": "OnUpdate update scheduled running pod", "src": "loadaware/pod_assign_cache_test.go:160-193",
         "event": "update", "pod": {"node": 0, "terminated": False, "uid": UID}, "cache": [], "want": [UID]},
        {"name": "OnDelete", "src": "loadaware/pod_assign_cache_test.go:214-253", "event": "delete",
         "pod": {"node": 0, "terminated": True, "uid": UID}, "cache": [UID], "want": []},
    ]
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)
    print(OUT)


if __name__ == "__main__":
    main()
