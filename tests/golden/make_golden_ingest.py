"""Transcribes the reference's own test vectors for the ingest decoders into tests/golden/ingest.json.

Data only (inputs and expected outputs typed in from the Go tests); no reference code is copied or run.
Sources:
  apis/extension/node_resource_amplification_test.go
    TestGetNodeResourceAmplificationRatios :28-87   (cpu entry of the returned map; error flag)
    TestGetNodeResourceAmplificationRatio  :89-180  (resource cpu; -1 when unset; error flag)
    TestGetNodeRawAllocatable              :372-433 (ResourceList; error flag)
  pkg/util/cpuset/cpuset_test.go
    TestParse                              :326-353
Run: python tests/golden/make_golden_ingest.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
RATIO = "node.koordinator.sh/resource-amplification-ratio"
RAW = "node.koordinator.sh/raw-allocatable"

ratios = [
    # TestGetNodeResourceAmplificationRatios :35-78
    {"name": "ratios/no annotation", "annotations": {}, "cpu": -1, "err": False},
    {"name": "ratios/no ratio annotation", "annotations": {"xxx": "yyy"}, "cpu": -1, "err": False},
    {"name": "ratios/valid", "annotations": {"xxx": "yyy", RATIO: '{"cpu":1.22}'}, "cpu": 1.22, "err": False},
    {"name": "ratios/invalid", "annotations": {"xxx": "yyy", RATIO: "invalid"}, "cpu": -1, "err": True},
    # TestGetNodeResourceAmplificationRatio :100-171
    {"name": "ratio/no annotation", "annotations": {}, "cpu": -1, "err": False},
    {"name": "ratio/no ratio annotation", "annotations": {"xxx": "yyy"}, "cpu": -1, "err": False},
    {"name": "ratio/cpu set", "annotations": {"xxx": "yyy", RATIO: '{"cpu":1.22}'}, "cpu": 1.22, "err": False},
    {"name": "ratio/cpu unset", "annotations": {"xxx": "yyy", RATIO: '{"memory":1.22}'}, "cpu": -1, "err": False},
    {"name": "ratio/invalid", "annotations": {"xxx": "yyy", RATIO: "invalid"}, "cpu": -1, "err": True},
]

raw_allocatable = [
    # TestGetNodeRawAllocatable :379-424 (want: ResourceList in cpu milli / memory units; err)
    {"name": "no annotation", "annotations": {}, "want": None, "err": False},
    {"name": "no raw allocatable annotation", "annotations": {"xxx": "yyy"}, "want": None, "err": False},
    {"name": "valid", "annotations": {"xxx": "yyy", RAW: '{"cpu":"1"}'}, "want": {"cpu": 1000}, "err": False},
    {"name": "invalid", "annotations": {"xxx": "yyy", RAW: "invalid"}, "want": None, "err": True},
]

cpuset_parse = [
    # TestParse :332-338
    {"s": "", "want": [], "err": False},
    {"s": "5", "want": [5], "err": False},
    {"s": "1,2,3,4,5", "want": [1, 2, 3, 4, 5], "err": False},
    {"s": "1-5", "want": [1, 2, 3, 4, 5], "err": False},
    {"s": "1-2,3-5", "want": [1, 2, 3, 4, 5], "err": False},
    {"s": "3-5,1-2", "want": [1, 2, 3, 4, 5], "err": False},
    {"s": "1-3-4", "want": [], "err": True},
]

if __name__ == "__main__":
    out = {"source": "apis/extension/node_resource_amplification_test.go, pkg/util/cpuset/cpuset_test.go",
           "amplification_ratio": ratios, "raw_allocatable": raw_allocatable, "cpuset_parse": cpuset_parse}
    with open(os.path.join(HERE, "ingest.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(ratios) + len(raw_allocatable) + len(cpuset_parse)} cases")
