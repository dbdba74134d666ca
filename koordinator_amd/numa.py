"""Host-side builders of the NodeNUMAResource ABI records (include/gpuscore.h gs_cpu_topology,
gs_node_numa, gs_pod_allocation) from NodeResourceTopology-shaped inputs.

The reference decodes these from the NRT object and node labels/annotations
(pkg/scheduler/plugins/nodenumaresource/topology_options.go:90-211, apis/extension/numa_aware.go);
the caller hands the decoded values over the C-ABI.
"""
from __future__ import annotations

import numpy as np

from . import abi


def cpuset_words(cpus) -> np.ndarray:
    w = np.zeros(abi.GS_CPU_WORDS, np.uint64)
    for c in cpus:
        w[c >> 6] |= np.uint64(1) << np.uint64(c & 63)
    return w


def cpus_of(words) -> list[int]:
    return [c for c in range(abi.GS_MAX_CPUS) if (int(words[c >> 6]) >> (c & 63)) & 1]


def topology(cpus: list[tuple[int, int, int]]) -> np.void:
    """CPUTopology from the reported detail: cpus[i] = (socket, numa node, core) of logical CPU i.
    CoreID = socket<<16 | core (CPUTopologyBuilder.AddCPUInfo, cpu_topology.go:40-45)."""
    t = np.zeros(1, abi.TOPOLOGY_DTYPE)[0]
    t["num_cpus"] = len(cpus)
    for i, (s, n, c) in enumerate(cpus):
        t["core_id"][i] = (s << 16) | c
        t["socket_id"][i] = s
        t["node_id"][i] = n
    return t


def test_topology(sockets: int, nodes_per_socket: int, cores_per_node: int, cpus_per_core: int) -> np.void:
    """buildCPUTopologyForTest (cpu_accumulator_test.go:30-57): CPU ids dense, core ids global, no socket shift."""
    t = np.zeros(1, abi.TOPOLOGY_DTYPE)[0]
    cpu = core = node = 0
    for s in range(sockets):
        for _ in range(nodes_per_socket):
            for _ in range(cores_per_node):
                for _ in range(cpus_per_core):
                    t["core_id"][cpu] = core
                    t["socket_id"][cpu] = s
                    t["node_id"][cpu] = node
                    cpu += 1
                core += 1
            node += 1
    t["num_cpus"] = cpu
    return t


def node_numa(topology_id: int | None = None, zones=(), numa_policy: str = "", node_cpu_bind: str = "",
              numa_allocate_strategy: str = "", cpu_ratio: float = 0.0, node_cpu_ratio: float = -1.0,
              reserved_cpus=(), max_ref_count: int = 1, has_options: bool = True) -> np.void:
    """gs_node_numa: zones = [(numa node id, cpu milli | None, memory | None), ...] sorted by id."""
    r = np.zeros(1, abi.NODE_NUMA_DTYPE)[0]
    r["has_options"] = int(has_options)
    r["topology"] = -1 if topology_id is None else topology_id
    r["max_ref_count"] = max_ref_count
    r["node_cpu_bind_policy"] = abi.NODE_CPU_BIND[node_cpu_bind]
    r["numa_topology_policy"] = abi.NUMA_POLICY[numa_policy]
    r["numa_allocate_strategy"] = abi.NUMA_ALLOC[numa_allocate_strategy]
    r["cpu_amplification_ratio"] = cpu_ratio
    r["node_cpu_amplification_ratio"] = node_cpu_ratio
    zs = sorted(zones, key=lambda z: z[0])
    if len(zs) > abi.GS_MAX_NUMA:
        raise ValueError(f"at most {abi.GS_MAX_NUMA} NUMA nodes per node on this path")
    r["num_zones"] = len(zs)
    for i, (nid, cpu, mem) in enumerate(zs):
        r["zones"][i]["node_id"] = nid
        m = 0
        if cpu is not None:
            r["zones"][i]["cpu_milli"] = cpu
            m |= abi.GS_USAGE_CPU
        if mem is not None:
            r["zones"][i]["memory"] = mem
            m |= abi.GS_USAGE_MEMORY
        r["zones"][i]["mask"] = m
    r["reserved_cpus"] = cpuset_words(reserved_cpus)
    return r


def pod_allocation(uid: int, cpus=(), numa=(), exclusive: str = "") -> np.void:
    """PodAllocation: numa = [(node id, cpu milli | None, memory | None), ...]"""
    a = np.zeros(1, abi.POD_ALLOCATION_DTYPE)[0]
    a["uid"] = uid
    a["cpuset"] = cpuset_words(cpus)
    a["cpu_exclusive_policy"] = abi.CPU_EXCLUSIVE[exclusive]
    a["num_numa"] = len(numa)
    for i, (nid, cpu, mem) in enumerate(numa):
        a["numa"][i]["node_id"] = nid
        m = 0
        if cpu is not None:
            a["numa"][i]["cpu_milli"] = cpu
            m |= abi.GS_USAGE_CPU
        if mem is not None:
            a["numa"][i]["memory"] = mem
            m |= abi.GS_USAGE_MEMORY
        a["numa"][i]["mask"] = m
    return a
