"""NodeNUMAResource plugin-level vectors of the reference (tests/golden/numa_plugin.json, transcribed from
plugin_test.go by make_golden_numa.py): Filter verdicts (TestPlugin_Filter, TestFilterWithAmplifiedCPUs), the
Filter-time NUMA affinity (TestFilterWithNUMANodeScoring) and the cpuset Reserve allocates (TestPlugin_Reserve); and
resourceManager.Allocate (resource_manager_test.go TestResourceManagerAllocate): the NUMA split and the cpuset of the
hint the test hands Allocate, or Allocate's failure (the pod then finds no node); resourceManager.GetTopologyHints
(TestResourceManagerGetTopologyHint) on the oracle.

The oracle is checked on the CPU; the same cases run through the HIP path (gs_evaluate codes, and gs_schedule on a
one-node cluster for the affinity bits and the cpuset the commit kernel selects) under -m gpu."""
import numpy as np
import pytest

from koordinator_amd import abi, numa
from oracle import oracle as orc
from tests import numa_util as nu

G = nu.load("numa_plugin.json")
REASON = {"INVALID_REQUESTED_CPUS": 1, "INVALID_AMP_RATIO": 2, "AVAILABLE_CPUS_ERROR": 3, "INSUFFICIENT_AMP_CPU": 4,
          "INVALID_TOPOLOGY": 5, "BIND_POLICY_CONFLICT": 6, "SMT_ALIGNMENT": 7}


def cases(kind):
    return [c for c in G["cases"] if c["kind"] == kind]


def ids(c):
    return c["name"].replace(" ", "_")


def check_filter(case, cls):
    e, pod = nu.build(case, cls)
    _, codes, _ = e.evaluate(np.array([pod], abi.POD_DTYPE))
    reason = (int(codes[0, 0]) & abi.GS_FAIL_NUMA_MASK) >> abi.GS_FAIL_NUMA_SHIFT
    want = REASON[case["want_reason"]] if case["want_reason"] else 0
    assert reason == want, f"{case['src']}: NodeNUMAResource reason {abi.NUMA_REASONS[reason]}, want {case['want_reason']}"


def schedule_one(case, cls):
    e, pod = nu.build(case, cls)
    if hasattr(e, "verify_cpusets"):
        e.verify_cpusets(True)
    out = e.schedule(np.array([pod], abi.POD_DTYPE), np.zeros(1, np.uint64))
    assert out["node"][0] == 0, f"{case['src']}: pod not placed"
    return e, pod, int(out["flags"][0])


def check_affinity(case, cls):
    _, _, flags = schedule_one(case, cls)
    got = [z for z in range(4) if (flags >> (abi.GS_PLACED_AFFINITY_SHIFT + z)) & 1]
    assert got == case["want_affinity"], f"{case['src']}: affinity {got}, want {case['want_affinity']}"


def check_reserve(case, cls):
    e, pod, _ = schedule_one(case, cls)
    a = e.allocation(0, int(pod["uid"]))
    got = [] if a is None else numa.cpus_of(a["cpuset"])
    assert got == case["want_cpuset"], f"{case['src']}: cpuset {got}, want {case['want_cpuset']}"


def check_allocate(case, cls):
    e, pod = nu.build(case, cls)
    if hasattr(e, "verify_cpusets"):
        e.verify_cpusets(True)
    out = e.schedule(np.array([pod], abi.POD_DTYPE), np.zeros(1, np.uint64))
    placed = int(out["node"][0]) == 0
    assert placed == case["want_placed"], f"{case['src']}: placed {placed}, want {case['want_placed']}"
    if not placed:
        return
    flags = int(out["flags"][0])
    aff = [z for z in range(4) if (flags >> (abi.GS_PLACED_AFFINITY_SHIFT + z)) & 1]
    assert aff == case["want_affinity"], f"{case['src']}: hint {aff}, want {case['want_affinity']}"
    a = e.allocation(0, int(pod["uid"]))
    assert a is not None, f"{case['src']}: no allocation recorded"
    assert numa.cpus_of(a["cpuset"]) == case["want_cpuset"], \
        f"{case['src']}: cpuset {numa.cpus_of(a['cpuset'])}, want {case['want_cpuset']}"
    got = {str(int(z["node_id"])): int(z["cpu_milli"]) for z in a["numa"][:int(a["num_numa"])] if z["cpu_milli"]}
    assert got == case["want_numa_cpu"], f"{case['src']}: NUMA cpu {got}, want {case['want_numa_cpu']}"


@pytest.mark.parametrize("case", cases("hints"), ids=ids)
def test_topology_hints_golden_oracle(case):
    """resourceManager.GetTopologyHints (oracle only: the device builds the same hints per zone subset inside
    eval_numa_kernel, where they are pinned through the Filter / affinity / Allocate vectors and full-size parity)."""
    e, pod = nu.build(case, orc.Oracle)
    got = e.topology_hints(pod)
    assert got is not None, f"{case['src']}: nil hints"
    names = {abi.GS_RES_CPU: "cpu", abi.GS_RES_MEMORY: "memory"}
    got = {names[r]: [[[z for z in range(4) if m >> z & 1], p] for m, p in lst] for r, lst in got.items()}
    assert got == case["want_hints"], f"{case['src']}: hints {got}, want {case['want_hints']}"


@pytest.mark.parametrize("case", cases("allocate"), ids=ids)
def test_allocate_golden_oracle(case):
    check_allocate(case, orc.Oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("case", cases("allocate"), ids=ids)
def test_allocate_golden_gpu(case):
    check_allocate(case, engine_cls())


@pytest.mark.parametrize("case", cases("filter"), ids=ids)
def test_filter_golden_oracle(case):
    check_filter(case, orc.Oracle)


@pytest.mark.parametrize("case", cases("affinity"), ids=ids)
def test_affinity_golden_oracle(case):
    check_affinity(case, orc.Oracle)


@pytest.mark.parametrize("case", cases("reserve"), ids=ids)
def test_reserve_golden_oracle(case):
    check_reserve(case, orc.Oracle)


def engine_cls():
    from koordinator_amd.engine import Engine
    return Engine


@pytest.mark.gpu
@pytest.mark.parametrize("case", cases("filter"), ids=ids)
def test_filter_golden_gpu(case):
    check_filter(case, engine_cls())


@pytest.mark.gpu
@pytest.mark.parametrize("case", cases("affinity"), ids=ids)
def test_affinity_golden_gpu(case):
    check_affinity(case, engine_cls())


@pytest.mark.gpu
@pytest.mark.parametrize("case", cases("reserve"), ids=ids)
def test_reserve_golden_gpu(case):
    check_reserve(case, engine_cls())
