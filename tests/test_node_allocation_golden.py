"""NodeAllocation (nodenumaresource/node_allocation.go:32-177) restatement in the oracle against the reference's own
tests in nodenumaresource/node_allocation_test.go, transcribed inline (each case cites its lines). Topology:
buildCPUTopologyForTest(2, 1, 4, 2) = 16 CPUs (node_allocation_test.go uses CoreID = socket<<16 | core)."""
import pytest

from koordinator_amd import abi
from oracle import oracle as orc

TOPO = (2, 1, 4, 2)
PCPU = abi.CPU_EXCLUSIVE["PCPULevel"]


def r(a, b):
    return list(range(a, b + 1))


def test_node_allocation_add_cpus():
    """TestNodeAllocationAddCPUs (node_allocation_test.go:33-97): add 1-4 (PCPULevel) -> RefCount 1 on 1-4 and
    getAvailableCPUs(maxRef 2) = 0-15; adding the same pod again changes nothing; another pod on 2-5 -> RefCount 2
    on 2-4, 1 on 1 and 5."""
    avail, ref = orc.node_allocation_script(TOPO, [("add", 1, r(1, 4), PCPU), ("available", 2, [])])
    assert avail == [r(0, 15)] and ref == {c: 1 for c in r(1, 4)}
    avail, ref = orc.node_allocation_script(TOPO, [("add", 1, r(1, 4), PCPU), ("add", 1, r(1, 4), PCPU),
                                                   ("available", 2, [])])
    assert avail == [r(0, 15)] and ref == {c: 1 for c in r(1, 4)}
    _, ref = orc.node_allocation_script(TOPO, [("add", 1, r(1, 4), PCPU), ("add", 2, r(2, 5), PCPU)])
    assert ref == {1: 1, 2: 2, 3: 2, 4: 2, 5: 1}


def test_node_allocation_release_cpus():
    """TestNodeAllocationStateReleaseCPUs (node_allocation_test.go:99-120): release leaves no allocated CPU."""
    _, ref = orc.node_allocation_script(TOPO, [("add", 1, r(1, 4), PCPU), ("release", 1)])
    assert ref == {}


def test_get_available_cpus():
    """Test_cpuAllocation_getAvailableCPUs (node_allocation_test.go:122-149)."""
    avail, _ = orc.node_allocation_script(TOPO, [
        ("add", 1, r(1, 4), PCPU), ("available", 2, []),
        ("add", 2, r(2, 5), PCPU), ("available", 2, []),
        ("release", 1), ("available", 1, [])])
    assert avail == [r(0, 15), [0, 1] + r(5, 15), [0, 1] + r(6, 15)]


def test_get_available_cpus_with_preferred_cpus():
    """Test_cpuAllocation_getAvailableCPUs_with_preferred_cpus (node_allocation_test.go:151-169)."""
    avail, _ = orc.node_allocation_script(TOPO, [("add", 1, r(0, 4), PCPU), ("available", 1, []),
                                                 ("available", 1, [1, 2])])
    assert avail == [r(5, 15), [1, 2] + r(5, 15)]


GI = 1 << 30


@pytest.mark.parametrize("name,amp,zone_cpu,alloc0,ncs,want_avail0,want_alloc", [
    # Test_getAvailableNUMANodeResources (node_allocation_test.go:171-303), topology buildCPUTopologyForTest(2,1,8,2)
    ("normal node", 0.0, 16000, 0, 0, 16000, {}),
    ("normal node with amplification ratios", 1.5, 24000, 0, 0, 24000, {}),
    ("amplification ratios and allocated CPUSets", 1.5, 24000, 4000, 4, 18000, {0: {0: 6000}}),
    ("amplification ratios, allocated CPUSets and CPU shares", 1.5, 24000, 8000, 4, 14000, {0: {0: 10000}}),
])
def test_get_available_numa_node_resources(name, amp, zone_cpu, alloc0, ncs, want_avail0, want_alloc):
    avail, alloc = orc.available_numa_test((2, 1, 8, 2), amp, zone_cpu, 32 * GI, alloc0, ncs)
    assert avail == {0: {0: want_avail0, 1: 32 * GI}, 1: {0: zone_cpu, 1: 32 * GI}}, name
    assert alloc == want_alloc, name
