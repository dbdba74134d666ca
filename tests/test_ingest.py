"""Ingest decoders (include/gpuscore.h gs_decode_*): annotation / label text -> ABI structs.

Pinned: the reference's own vectors in tests/golden/ingest.json (node_resource_amplification_test.go,
cpuset_test.go TestParse). Parity unpinned (upstream libraries, no test in the reference): resource.Quantity
Value/MilliValue, time.ParseDuration, encoding/json corner cases — checked against their published semantics
below. Round trips: synthetic node / topology / cpuset structs -> the annotation JSON the reference reads ->
the decoders -> the same structs. Pure host functions of libgpuscore: no GPU needed."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi, ingest

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ingest.json")))
RAW = "node.koordinator.sh/raw-allocatable"
THR = "scheduling.koordinator.sh/usage-thresholds"
RATIO = "node.koordinator.sh/resource-amplification-ratio"


@pytest.mark.parametrize("case", G["amplification_ratio"], ids=lambda c: c["name"])
def test_golden_amplification_ratio(case):
    _, numa = ingest.node_annotations(case["annotations"])
    assert numa.node_cpu_amplification_ratio == case["cpu"]
    assert bool(numa.node_amplification_invalid) == case["err"]


@pytest.mark.parametrize("case", G["raw_allocatable"], ids=lambda c: c["name"])
def test_golden_raw_allocatable(case):
    node, _ = ingest.node_annotations(case["annotations"])
    if case["want"] is None:   # absent, or an error EstimateNode ignores (default_estimator.go:111-114)
        assert node.raw_allocatable_mask == 0
    else:
        assert node.raw_allocatable_mask == abi.GS_USAGE_CPU
        assert node.raw_allocatable[0] == case["want"]["cpu"]


@pytest.mark.parametrize("case", G["cpuset_parse"], ids=lambda c: repr(c["s"]))
def test_golden_cpuset_parse(case):
    if case["err"]:
        with pytest.raises(ingest.DecodeError):
            ingest.cpuset(case["s"])
    else:
        assert ingest.cpuset(case["s"]) == case["want"]


# resource.Quantity: (text, Value(), MilliValue()) — both round up (ScaledValue ceil)
QUANTITIES = [
    ("1", 1, 1000), ("100m", 1, 100), ("1500m", 2, 1500), ("1.5", 2, 1500), ("0.0001", 1, 1), ("0", 0, 0),
    ("1Ki", 1024, 1024000), ("1Gi", 1 << 30, (1 << 30) * 1000), ("16Gi", 16 << 30, (16 << 30) * 1000),
    ("5G", 5 * 10**9, 5 * 10**12), ("1e3", 1000, 10**6), ("1E-3", 1, 1), ("-0", 0, 0), ("+2", 2, 2000),
    ("128974848", 128974848, 128974848000), ("129e6", 129 * 10**6, 129 * 10**9), ("123Mi", 123 << 20, (123 << 20) * 1000),
    ("0.5Ki", 512, 512000), ("1n", 1, 1), ("250u", 1, 1), ("3k", 3000, 3 * 10**6), (".5", 1, 500),
]


@pytest.mark.parametrize("text,value,milli", QUANTITIES)
def test_quantity(text, value, milli):
    assert ingest.quantity(text) == (value, milli)


@pytest.mark.parametrize("text", ["", "abc", "1Gb", "1.2.3", "--1", "1e", "Mi", "1 Gi"])
def test_quantity_malformed(text):
    with pytest.raises(ingest.DecodeError):
        ingest.quantity(text)


@pytest.mark.parametrize("text", ["-1.5", "-1", "-100m", "-1Ki", "-0.5"])
def test_quantity_negative_refused(text):
    """Negative quantities: apimachinery rounds an inexact negative Value() one way on its int64Amount path and
    another on its inf.Dec path; no valid request / allocatable / annotation is negative, so the decoder refuses
    them (parity unpinned: no reference fixture holds a negative quantity)."""
    with pytest.raises(ingest.DecodeError) as e:
        ingest.quantity(text)
    assert e.value.rc == abi.GS_EUNSUPPORTED


def test_quantity_outside_int64():
    with pytest.raises(ingest.DecodeError) as e:
        ingest.quantity("10E")   # 10^19 > 2^63
    assert e.value.rc == abi.GS_EUNSUPPORTED


@pytest.mark.parametrize("dur,ns", [("5m", 300 * 10**9), ("1h30m", 5400 * 10**9), ("300s", 300 * 10**9),
                                     ("1.5h", 5400 * 10**9), ("0", 0), ("100ms", 10**8), ("2m3.5s", 123_500_000_000)])
def test_usage_thresholds_aggregated_duration(dur, ns):
    text = json.dumps({"aggregatedUsage": {"usageThresholds": {"cpu": 70}, "usageAggregationType": "p95",
                                           "usageAggregatedDuration": dur}})
    node, _ = ingest.node_annotations({THR: text})
    assert node.custom_flags == abi.GS_NODE_CUSTOM_THRESHOLDS | abi.GS_NODE_CUSTOM_AGGREGATED
    assert node.custom_agg_duration_ns == ns and node.custom_agg_type == abi.GS_AGG_P95


@pytest.mark.parametrize("text", ['{"usageThresholds":{"cpu":"65"}}', '{"usageThresholds":{"cpu":65.5}}',
                                  'not json', '{"aggregatedUsage":{"usageAggregatedDuration":"5x"}}',
                                  '{"usageThresholds":[]}'])
def test_usage_thresholds_malformed_means_args(text):
    """json.Unmarshal fails -> generateUsageThresholdsFilterProfile uses the args (helper.go:104-117): no flags"""
    node, _ = ingest.node_annotations({THR: text})
    assert node.custom_flags == 0


def test_usage_thresholds_keys():
    text = '{"usageThresholds":{"cpu":65,"memory":80,"nvidia.com/gpu":10},"prodUsageThresholds":{"memory":70}}'
    node, _ = ingest.node_annotations({THR: text})
    assert node.custom_flags == abi.GS_NODE_CUSTOM_THRESHOLDS
    assert list(node.custom_usage_thresholds) == [65, 80]
    assert node.custom_usage_mask == abi.GS_USAGE_CPU | abi.GS_USAGE_MEMORY | abi.GS_USAGE_OTHER
    assert list(node.custom_prod_usage_thresholds) == [0, 70] and node.custom_prod_usage_mask == abi.GS_USAGE_MEMORY


def test_resource_spec():
    pod = ingest.resource_spec('{"requiredCPUBindPolicy":"FullPCPUs","preferredCPUExclusivePolicy":"PCPULevel"}')
    assert (pod.required_cpu_bind_policy, pod.preferred_cpu_bind_policy, pod.preferred_cpu_exclusive_policy) == \
        (abi.CPU_BIND["FullPCPUs"], abi.CPU_BIND[""], abi.CPU_EXCLUSIVE["PCPULevel"])
    pod = ingest.resource_spec('{"preferredCPUBindPolicy":"SpreadByPCPUs"}')
    assert pod.preferred_cpu_bind_policy == abi.CPU_BIND["SpreadByPCPUs"]
    pod = ingest.resource_spec(None)   # annotation absent: an empty ResourceSpec
    assert pod.required_cpu_bind_policy == pod.preferred_cpu_bind_policy == abi.CPU_BIND[""]
    with pytest.raises(ingest.DecodeError):
        ingest.resource_spec('{"preferredCPUBindPolicy":1}')   # json.Unmarshal error: PreFilter fails


def test_node_labels_and_kubelet_policy():
    numa = ingest.node_labels({"node.koordinator.sh/numa-topology-policy": "SingleNUMANode",
                               "node.koordinator.sh/numa-allocate-strategy": "LeastAllocated"})
    assert numa.numa_topology_policy == abi.NUMA_POLICY["SingleNUMANode"]
    assert numa.numa_allocate_strategy == abi.NUMA_ALLOC["LeastAllocated"]
    assert numa.node_cpu_bind_policy == abi.NODE_CPU_BIND["None"]
    kubelet = '{"policy":"static","options":{"full-pcpus-only":"true"},"reservedCPUs":"0-1"}'
    numa = ingest.node_labels({}, kubelet, "Restricted")
    assert numa.node_cpu_bind_policy == abi.NODE_CPU_BIND["FullPCPUsOnly"]   # numa_aware.go:316-318
    assert numa.numa_topology_policy == abi.NUMA_POLICY["Restricted"]          # util.go:52-58 fallback
    numa = ingest.node_labels({"node.koordinator.sh/cpu-bind-policy": "SpreadByPCPUs"},
                              '{"policy":"none"}')
    assert numa.node_cpu_bind_policy == abi.NODE_CPU_BIND["SpreadByPCPUs"]


def test_round_trip_random_annotations():
    """Seeded random raw-allocatable / usage-threshold / amplification annotations (the JSON the reference reads)
    -> the decoders -> the values they were built from"""
    rng = np.random.default_rng(7)
    names = {abi.GS_AGG_AVG: "avg", abi.GS_AGG_P50: "p50", abi.GS_AGG_P90: "p90", abi.GS_AGG_P95: "p95",
             abi.GS_AGG_P99: "p99"}
    for _ in range(400):
        ann = {}
        raw = {}
        if rng.random() < 0.5:
            raw["cpu"] = f"{int(rng.integers(1, 200_000))}m"
        if rng.random() < 0.5:
            raw["memory"] = f"{int(rng.integers(1, 1 << 20))}Mi"
        if raw:
            ann[RAW] = json.dumps(raw)
        thr = {}
        if rng.random() < 0.5:
            thr["usageThresholds"] = {"cpu": int(rng.integers(1, 100))}
        if rng.random() < 0.3:
            t = int(rng.choice(list(names)))
            thr["aggregatedUsage"] = {"usageThresholds": {"memory": int(rng.integers(1, 100))},
                                      "usageAggregationType": names[t], "usageAggregatedDuration": "10m0s"}
        if thr or rng.random() < 0.2:
            ann[THR] = json.dumps(thr)
        ratio = round(float(rng.uniform(1, 3)), 3) if rng.random() < 0.3 else None
        if ratio is not None:
            ann[RATIO] = json.dumps({"cpu": ratio})
        node, numa = ingest.node_annotations(ann)
        if raw:
            mask = (abi.GS_USAGE_CPU if "cpu" in raw else 0) | (abi.GS_USAGE_MEMORY if "memory" in raw else 0)
            assert node.raw_allocatable_mask == mask
            if "cpu" in raw:
                assert node.raw_allocatable[0] == int(raw["cpu"][:-1])
            if "memory" in raw:
                assert node.raw_allocatable[1] == int(raw["memory"][:-2]) << 20
        else:
            assert node.raw_allocatable_mask == 0
        assert bool(node.custom_flags & abi.GS_NODE_CUSTOM_THRESHOLDS) == (THR in ann)
        assert bool(node.custom_flags & abi.GS_NODE_CUSTOM_AGGREGATED) == ("aggregatedUsage" in thr)
        if "usageThresholds" in thr:
            assert node.custom_usage_thresholds[0] == thr["usageThresholds"]["cpu"]
        if "aggregatedUsage" in thr:
            assert node.custom_agg_duration_ns == 600 * 10**9
            assert names[node.custom_agg_type] == thr["aggregatedUsage"]["usageAggregationType"]
        assert numa.node_cpu_amplification_ratio == (ratio if ratio is not None else -1)


def test_round_trip_cpu_topology_and_cpusets():
    rng = np.random.default_rng(11)
    for _ in range(50):
        sockets, nodes_per, cores_per, smt = (int(rng.integers(1, 3)), int(rng.integers(1, 3)),
                                              int(rng.integers(1, 17)), int(rng.integers(1, 3)))
        detail, cpu = [], 0
        for s in range(sockets):
            for nn in range(nodes_per):
                for co in range(cores_per):
                    for _t in range(smt):
                        detail.append({"id": cpu, "core": s * nodes_per * cores_per + nn * cores_per + co,
                                       "socket": s, "node": s * nodes_per + nn})
                        cpu += 1
        order = rng.permutation(len(detail))
        t = ingest.cpu_topology(json.dumps({"detail": [detail[j] for j in order]}))
        core, sock, node = ingest.topology_arrays(t)
        assert t.num_cpus == len(detail)
        for d in detail:
            assert core[d["id"]] == (d["socket"] << 16) | d["core"]
            assert sock[d["id"]] == d["socket"] and node[d["id"]] == d["node"]
        ids = sorted(set(int(x) for x in rng.integers(0, abi.GS_MAX_CPUS, int(rng.integers(0, 40)))))
        parts, i = [], 0
        while i < len(ids):   # Linux list format with ranges, as CPUSet.String writes it
            j = i
            while j + 1 < len(ids) and ids[j + 1] == ids[j] + 1:
                j += 1
            parts.append(str(ids[i]) if i == j else f"{ids[i]}-{ids[j]}")
            i = j + 1
        assert ingest.cpuset(",".join(parts)) == ids


def test_decoder_throughput_smoke():
    """The decoders are host code on the ingest path: a 10k-node annotation batch decodes well under a second."""
    import time
    ann = {RAW: '{"cpu":"96","memory":"512Gi"}', THR: '{"usageThresholds":{"cpu":65,"memory":95}}',
           RATIO: '{"cpu":1.5}'}
    t0 = time.perf_counter()
    for _ in range(10_000):
        ingest.node_annotations(ann)
    assert time.perf_counter() - t0 < 5.0


def test_quantity_matches_python_restatement():
    """The C++ Quantity decoder against the independent exact-rational restatement in koordinator_amd.objects
    (Decimal mantissa x suffix, ceil), on seeded random quantities across every suffix."""
    from koordinator_amd import objects
    rng = np.random.default_rng(5)
    sufs = sorted(objects._SUFFIX)
    for _ in range(3000):
        whole = int(rng.integers(0, 10**6))
        frac = "" if rng.random() < 0.5 else "." + str(int(rng.integers(0, 10**4))).rjust(int(rng.integers(1, 5)), "0")
        text = f"{whole}{frac}{sufs[int(rng.integers(0, len(sufs)))]}"
        want_v = objects._ceil(objects.parse_quantity(text))
        want_mv = objects._ceil(objects.parse_quantity(text) * 1000)
        if max(abs(want_v), abs(want_mv)) >= 2**63:
            continue
        assert ingest.quantity(text) == (want_v, want_mv), text
