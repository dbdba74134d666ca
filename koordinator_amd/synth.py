"""Deterministic synthetic clusters for the BASELINE.json configurations.

Counter-based splitmix64 streams (seed 0x6b6f6f7264 + config id): every value is a pure function of
(seed, stream, index), so every rank of a multi-GPU run builds the identical cluster without
communication, and the CPU oracle sees exactly the bytes the GPU sees. All quantities are integral
milli-CPU / bytes, so resource.Quantity rounding is inert.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import abi

BASE_SEED = 0x6B6F6F7264
NOW_NS = 1_700_000_000 * 10**9
GiB = 1 << 30
MiB = 1 << 20
SEC = 10**9

CONFIGS = {
    # id: (nodes, pods, description)  — BASELINE.json "configs"
    0: (1_000, 1_000, "C1: 1k nodes x 1k pods, LoadAware + NodeResourcesFit LeastAllocated (CPU bench analogue)"),
    1: (5_000, 10_000, "C2: 5k nodes x 10k pods, synthetic NodeMetric usage, batched pod queue, 1 GPU"),
    2: (50_000, 50_000, "C3: 50k nodes x 50k pods, 1 GPU"),
    3: (100_000, 50_000, "C4: 100k nodes node-sharded across GPUs"),
}

_M1, _M2, _GOLD = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB), np.uint64(0x9E3779B97F4A7C15)


def mix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


class Stream:
    def __init__(self, seed: int):
        self.seed = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)

    def u64(self, stream: int, n: int) -> np.ndarray:
        key = mix64(np.array([self.seed ^ np.uint64(stream)], np.uint64))[0]
        with np.errstate(over="ignore"):
            return mix64(np.arange(n, dtype=np.uint64) + key * np.uint64(0x100000001B3))

    def randint(self, stream: int, n: int, lo, hi) -> np.ndarray:
        """Uniform integers in [lo, hi] (inclusive; lo/hi scalars or arrays)."""
        lo = np.asarray(lo, np.int64)
        hi = np.asarray(hi, np.int64)
        span = (hi - lo + 1).astype(np.uint64)
        return lo + (self.u64(stream, n) % span).astype(np.int64)

    def uniform(self, stream: int, n: int) -> np.ndarray:
        return (self.u64(stream, n) >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


@dataclass
class Cluster:
    now_ns: int
    nodes: np.ndarray        # NODE_DTYPE[N]
    metrics: np.ndarray      # METRIC_DTYPE[N]
    pod_metrics: np.ndarray  # POD_METRIC_DTYPE[M]
    pm_offsets: np.ndarray   # uint32[N+1]
    assigned_node: np.ndarray
    assigned_pods: np.ndarray
    assigned_ts: np.ndarray
    pods: np.ndarray         # POD_DTYPE[P] pending, in scheduling order
    numa: dict | None = None # NodeNUMAResource state: topologies, node_numa, allocations (make_numa)
    ext: dict | None = None  # Reservation + DeviceShare state (make_ext)

    @property
    def num_nodes(self) -> int:
        return len(self.nodes)


def make_pods(s: Stream, n: int, base_stream: int, name_base: int) -> np.ndarray:
    pods = np.zeros(n, abi.POD_DTYPE)
    kind = s.randint(base_stream + 0, n, 0, 99)           # 70% limit=req, 20% limit=2req, 10% no requests
    no_req = kind >= 90
    cpu = s.randint(base_stream + 1, n, 1, 80) * 100       # [100m, 8] step 100m
    mem = s.randint(base_stream + 2, n, 128, 16 * 1024) * MiB
    cpu = np.where(no_req, 0, cpu)
    mem = np.where(no_req, 0, mem)
    lim_mul = np.where(kind < 70, 1, np.where(kind < 90, 2, 0))
    prio_prod = s.randint(base_stream + 3, n, 0, 99) < 40   # 40% Prod priority (9000-9999), 60% none
    req = np.zeros((n, abi.GS_NUM_RES), np.int64)
    lim = np.zeros((n, abi.GS_NUM_RES), np.int64)
    req[:, 0], req[:, 1] = cpu, mem
    lim[:, 0], lim[:, 1] = cpu * lim_mul, mem * lim_mul
    pods["requests"] = req
    pods["limits"] = lim
    nz = np.zeros((n, 2), np.int64)
    nz[:, 0] = np.where(no_req, 100, cpu)                   # schedutil DefaultMilliCPURequest
    nz[:, 1] = np.where(no_req, 200 * MiB, mem)             # schedutil DefaultMemoryRequest
    pods["nonzero_requests"] = nz
    pods["request_mask"] = np.where(no_req, 0, (1 << abi.GS_RES_CPU) | (1 << abi.GS_RES_MEMORY)).astype(np.uint32)
    # GetPodPriorityClassWithDefault: priority 9000-9999 -> Prod; otherwise the QoS default
    # (Guaranteed -> LSR, Burstable -> LS: Prod; BestEffort -> BE: Batch).
    pods["priority_class"] = np.where(prio_prod | ~no_req, abi.GS_PRIO_PROD, abi.GS_PRIO_BATCH)
    pods["uid"] = s.u64(base_stream + 4, n)
    pods["name_key"] = mix64(np.arange(name_base, name_base + n, dtype=np.uint64))
    return pods


def make_cluster(num_nodes: int, num_pods: int, config_id: int = 1, seed: int | None = None) -> Cluster:
    s = Stream((BASE_SEED + config_id) if seed is None else seed)
    N = num_nodes
    now = NOW_NS
    cores = np.array([32, 48, 64, 96, 128], np.int64)[s.randint(1, N, 0, 4)]
    mem_g = np.array([128, 256, 384, 512, 1024], np.int64)[s.randint(2, N, 0, 4)]
    nodes = np.zeros(N, abi.NODE_DTYPE)
    alloc = np.zeros((N, abi.GS_NUM_RES), np.int64)
    alloc[:, 0] = cores * 1000
    alloc[:, 1] = mem_g * GiB
    alloc[:, 2] = 500 * GiB
    nodes["allocatable"] = alloc
    reqd = np.zeros((N, abi.GS_NUM_RES), np.int64)
    reqd[:, 0] = s.randint(3, N, 0, alloc[:, 0] // 100 * 70 // 100) * 100     # U[0,70%] in 100m steps
    reqd[:, 1] = s.randint(4, N, 0, alloc[:, 1] // MiB * 70 // 100) * MiB      # U[0,70%] in 1MiB steps
    reqd[:, 2] = s.randint(5, N, 0, 50) * GiB
    nodes["requested"] = reqd
    pod_count = s.randint(6, N, 0, 60)
    zero_req = s.randint(7, N, 0, pod_count // 10)                           # ~5% zero-request pods
    nz = np.zeros((N, 2), np.int64)
    nz[:, 0] = reqd[:, 0] + zero_req * 100
    nz[:, 1] = reqd[:, 1] + zero_req * 200 * MiB
    nodes["nonzero_requested"] = nz
    nodes["allowed_pod_number"] = 110
    nodes["pod_count"] = pod_count
    # 5% of nodes carry node.koordinator.sh/raw-allocatable (EstimateNode override)
    raw = s.randint(8, N, 0, 99) < 5
    rawv = np.zeros((N, 2), np.int64)
    rawv[:, 0] = np.where(raw, alloc[:, 0] * 9 // 10 // 1000 * 1000, 0)
    rawv[:, 1] = np.where(raw, alloc[:, 1] * 9 // 10, 0)
    nodes["raw_allocatable"] = rawv
    nodes["raw_allocatable_mask"] = np.where(raw, abi.GS_USAGE_CPU | abi.GS_USAGE_MEMORY, 0).astype(np.uint32)
    # 3% custom usage thresholds, 1% custom prod thresholds (scheduling.koordinator.sh/usage-thresholds)
    cu = s.randint(9, N, 0, 99)
    custom = cu < 4
    nodes["custom_flags"] = np.where(custom, abi.GS_NODE_CUSTOM_THRESHOLDS, 0).astype(np.uint32)
    ut = np.zeros((N, 2), np.int64)
    ut[:, 0], ut[:, 1] = 70, 90
    nodes["custom_usage_thresholds"] = ut
    nodes["custom_usage_mask"] = np.where(cu < 3, abi.GS_USAGE_CPU | abi.GS_USAGE_MEMORY, 0).astype(np.uint32)
    pt = np.zeros((N, 2), np.int64)
    pt[:, 0] = 60
    nodes["custom_prod_usage_thresholds"] = pt
    nodes["custom_prod_usage_mask"] = np.where(cu == 3, abi.GS_USAGE_CPU, 0).astype(np.uint32)
    nodes["custom_agg_type"] = abi.GS_AGG_NONE

    # NodeMetric: 2% missing, 1% expired (now - 300s), else now - U[0,120]s (+ ns jitter)
    metrics = np.zeros(N, abi.METRIC_DTYPE)
    mk = s.randint(10, N, 0, 99)
    exists = mk >= 2
    expired = mk == 2
    upd = now - s.randint(11, N, 0, 120) * SEC - s.randint(12, N, 1, 999_999)
    upd = np.where(expired, now - 300 * SEC, upd)
    metrics["exists"] = exists
    metrics["has_update_time"] = exists
    metrics["update_time_ns"] = np.where(exists, upd, 0)
    metrics["has_report_interval"] = exists
    metrics["report_interval_s"] = 60
    metrics["has_node_metric"] = exists
    metrics["node_usage"]["cpu_milli"] = s.randint(13, N, 0, alloc[:, 0] * 80 // 100)
    metrics["node_usage"]["memory"] = s.randint(14, N, 0, alloc[:, 1] * 95 // 100)
    metrics["node_usage"]["mask"] = np.where(exists, abi.GS_USAGE_CPU | abi.GS_USAGE_MEMORY, 0)

    # podAssignCache: 0-3 pods per node, timestamps straddling updateTime (>= 1s from every boundary)
    na = s.randint(15, N, 0, 3)
    A = int(na.sum())
    a_node = np.repeat(np.arange(N, dtype=np.uint32), na)
    a_pods = make_pods(s, A, 100, 10_000_000)
    a_pods["uid"] = s.u64(120, A)
    off_kind = s.randint(16, A, 0, 2)
    off = np.where(off_kind == 0, -s.randint(17, A, 61, 300),         # old: metric may cover it
                   np.where(off_kind == 1, -s.randint(18, A, 1, 59),   # within the report interval
                            s.randint(19, A, 1, 30)))                  # after the last update
    base = np.where(exists[a_node], upd[a_node], now - 100 * SEC)
    a_ts = base + off * SEC + s.randint(20, A, 0, 999) * 1000
    a_ts = np.minimum(a_ts, now)
    # PodsMetric: 70% of assigned pods on nodes with metrics report usage (in the pod lister)
    has_pm = (s.randint(21, A, 0, 99) < 70) & exists[a_node]
    pm_node = a_node[has_pm]
    pm = np.zeros(int(has_pm.sum()), abi.POD_METRIC_DTYPE)
    pm["name_key"] = a_pods["name_key"][has_pm]
    pm["in_lister"] = 1
    pm["priority_class"] = a_pods["priority_class"][has_pm]
    rq = a_pods["requests"][has_pm]
    pm["usage"]["cpu_milli"] = s.randint(22, len(pm), 0, np.maximum(rq[:, 0], 100))
    pm["usage"]["memory"] = s.randint(23, len(pm), 0, np.maximum(rq[:, 1], 128 * MiB))
    pm["usage"]["mask"] = abi.GS_USAGE_CPU | abi.GS_USAGE_MEMORY
    order = np.argsort(pm_node, kind="stable")
    pm = pm[order]
    counts = np.bincount(pm_node, minlength=N)
    offsets = np.zeros(N + 1, np.uint32)
    offsets[1:] = np.cumsum(counts)

    pods = make_pods(s, num_pods, 200, 20_000_000)
    return Cluster(now, nodes, metrics, pm, offsets, a_node, a_pods, a_ts.astype(np.int64), pods)


def make_numa(c: Cluster, seed: int | None = None, numa_policy_pct: int = 30, cpuset_pod_pct: int = 20,
              mixed: bool = False) -> Cluster:
    """Adds the C3 NodeNUMAResource state to a cluster, in place:
    2 sockets, k in {2, 4} NUMA nodes, 32-128 physical cores (the cluster's cores draw) with SMT2, i.e. 64-256 logical
    CPUs: the node's CPU quantities (allocatable = the logical CPUs, as the kubelet reports them, requested,
    non-zero requested, raw allocatable, NodeMetric usage) are doubled so their utilisation is unchanged; NRT zones
    split cpu and memory evenly; `numa_policy_pct`% of nodes labelled numa-topology-policy in {SingleNUMANode, Restricted,
    BestEffort}; 3% node cpu-bind-policy FullPCPUsOnly, 2% SpreadByPCPUs; 4% cpu amplification 1.5; existing
    cpuset pods on 25% of nodes and NUMA allocations on labelled nodes; `cpuset_pod_pct`% of pending pods LSR/LSE
    Prod with integer CPUs (some with a required bind policy).
    mixed: also sibling-interleaved CPU numbering (cpu = thread * cores + core), SMT-4 and SMT-1 classes (256 SMT-1
    cores exceed the device cpuset scope), maxRefCount 2 on 3% of nodes, PCPU- and NUMANode-level
    exclusive existing allocations and pods."""
    from . import numa as nm
    s = Stream((BASE_SEED + 77) if seed is None else seed)
    N = c.num_nodes
    # SMT2: the logical CPUs are twice the physical cores
    zero_nz = c.nodes["nonzero_requested"][:, 0] - c.nodes["requested"][:, 0]
    c.nodes["allocatable"][:, 0] *= 2
    c.nodes["requested"][:, 0] *= 2
    c.nodes["nonzero_requested"][:, 0] = c.nodes["requested"][:, 0] + zero_nz
    c.nodes["raw_allocatable"][:, 0] *= 2
    c.metrics["node_usage"]["cpu_milli"] *= 2
    cores = c.nodes["allocatable"][:, 0] // 1000   # logical CPUs
    k = np.where(s.randint(300, N, 0, 1) == 0, 2, 4)
    # topology classes by (cores, k)
    classes, tid_of = {}, np.zeros(N, np.int32)
    for i in range(N):
        key = (int(cores[i]), int(k[i]))
        if key not in classes:
            classes[key] = len(classes)
        tid_of[i] = classes[key]
    topos = []
    for ci, ((nc, kk), _) in enumerate(sorted(classes.items(), key=lambda kv: kv[1])):
        per_socket = kk // 2
        smt, interleave = 2, False
        if mixed:
            # (256 logical CPUs as SMT-1 cores: outside the device cpuset scope, the host path)
            smt = 1 if (nc == 256 and kk == 2) else 4 if ci % 5 == 2 else (1 if ci % 7 == 3 else 2)
            interleave = ci % 3 == 1
        cores_per_numa = nc // smt // kk
        ncores = 2 * per_socket * cores_per_numa
        cpus = [None] * (ncores * smt)
        g = 0
        for sk in range(2):
            for nn in range(per_socket):
                for co in range(cores_per_numa):
                    for t in range(smt):
                        cpu = t * ncores + g if interleave else g * smt + t
                        cpus[cpu] = (sk, sk * per_socket + nn, nn * cores_per_numa + co)
                    g += 1
        topos.append(nm.topology(cpus))
    pol = s.randint(301, N, 0, 99)
    policy = np.where(pol < numa_policy_pct // 3, "SingleNUMANode",
                      np.where(pol < 2 * numa_policy_pct // 3, "Restricted",
                               np.where(pol < numa_policy_pct, "BestEffort", "")))
    bindk = s.randint(302, N, 0, 99)
    amp = s.randint(303, N, 0, 99) < 4
    recs = np.zeros(N, abi.NODE_NUMA_DTYPE)
    mem = c.nodes["allocatable"][:, 1]
    for i in range(N):
        kk = int(k[i])
        ratio = 1.5 if amp[i] else 0.0
        zc = int(cores[i]) * 1000 // kk
        if amp[i]:
            zc = int(np.ceil(zc * 1.5))
        zones = [(z, zc, int(mem[i]) // kk) for z in range(kk)]
        recs[i] = nm.node_numa(int(tid_of[i]), zones, numa_policy=str(policy[i]),
                               node_cpu_bind="FullPCPUsOnly" if bindk[i] < 3 else ("SpreadByPCPUs" if bindk[i] < 5 else ""),
                               cpu_ratio=ratio, node_cpu_ratio=1.5 if amp[i] else -1.0,
                               max_ref_count=2 if (mixed and bindk[i] >= 97) else 1)
    if amp.any():   # amplified allocatable (NodeResource controller), as makeNode does in plugin_test.go:114-120
        c.nodes["allocatable"][amp, 0] = np.ceil(c.nodes["allocatable"][amp, 0] * 1.5).astype(np.int64)
    # existing allocations: a cpuset pod (2-8 CPUs from CPU 0 up, full cores) on 25% of nodes; NUMA resources on
    # labelled nodes (zone 0)
    allocs, a_nodes = [], []
    has_cs = s.randint(304, N, 0, 99) < 25
    ncs = s.randint(305, N, 1, 4) * 2
    for i in np.nonzero(has_cs | (policy != ""))[0]:
        cpus = list(range(int(ncs[i]))) if has_cs[i] else []
        numa_res = [(0, int(ncs[i]) * 1000, 4 << 30)] if policy[i] != "" else []
        excl = ("PCPULevel", "NUMANodeLevel", "")[i % 3] if (mixed and cpus) else ""
        allocs.append(nm.pod_allocation(int(0x5EED0000 + i), cpus, numa_res, exclusive=excl))
        a_nodes.append(int(i))
    c.numa = {"topologies": topos, "node_numa": recs,
              "alloc_nodes": np.array(a_nodes, np.uint32),
              "allocs": np.array(allocs, abi.POD_ALLOCATION_DTYPE) if allocs else np.zeros(0, abi.POD_ALLOCATION_DTYPE)}
    # pending pods: cpuset_pod_pct% LSR/LSE Prod with integer cpus
    P = len(c.pods)
    cs = s.randint(306, P, 0, 99) < cpuset_pod_pct
    cpus = s.randint(307, P, 1, 8) * 1000
    c.pods["requests"][cs, 0] = cpus[cs]
    c.pods["nonzero_requests"][cs, 0] = cpus[cs]
    c.pods["limits"][cs, 0] = cpus[cs]
    c.pods["requests"][cs, 1] = np.maximum(c.pods["requests"][cs, 1], 256 << 20)
    c.pods["nonzero_requests"][cs, 1] = c.pods["requests"][cs, 1]
    c.pods["limits"][cs, 1] = c.pods["requests"][cs, 1]
    c.pods["request_mask"][cs] = (1 << abi.GS_RES_CPU) | (1 << abi.GS_RES_MEMORY)
    c.pods["priority_class"][cs] = abi.GS_PRIO_PROD
    c.pods["qos_class"] = np.where(cs, np.where(s.randint(308, P, 0, 1) == 0, abi.GS_QOS_LSR, abi.GS_QOS_LSE),
                                   abi.GS_QOS_LS)
    req = s.randint(309, P, 0, 99)
    c.pods["required_cpu_bind_policy"] = np.where(cs & (req < 10), abi.CPU_BIND["FullPCPUs"],
                                                  np.where(cs & (req < 15), abi.CPU_BIND["SpreadByPCPUs"], 0))
    c.pods["preferred_cpu_bind_policy"] = np.where(cs & (req >= 15) & (req < 30), abi.CPU_BIND["SpreadByPCPUs"], 0)
    c.pods["preferred_cpu_exclusive_policy"] = np.where(cs & (req >= 90), abi.CPU_EXCLUSIVE["PCPULevel"], 0)
    if mixed:
        c.pods["preferred_cpu_exclusive_policy"] = np.where(cs & (req >= 80) & (req < 90),
                                                            abi.CPU_EXCLUSIVE["NUMANodeLevel"],
                                                            c.pods["preferred_cpu_exclusive_policy"])
    return c


def load_into(engine, c: Cluster) -> None:
    """Push a cluster into an Engine / Oracle (same calls a scheduler's informers would make)."""
    engine.set_now(c.now_ns)
    engine.upsert_nodes(c.nodes)
    engine.upsert_metrics(c.metrics, c.pod_metrics, c.pm_offsets)
    if len(c.assigned_pods):
        engine.assign(c.assigned_node, c.assigned_pods, c.assigned_ts)
    if c.numa is not None:
        ids = [engine.register_topology(t) for t in c.numa["topologies"]]
        recs = c.numa["node_numa"].copy()
        recs["topology"] = np.array(ids, np.int32)[recs["topology"]]
        engine.upsert_numa(recs)
        if len(c.numa["allocs"]):
            engine.update_allocations(c.numa["alloc_nodes"], c.numa["allocs"])


def make_ext(c: Cluster, seed: int | None = None, gpu_node_pct: int = 20, gpus_per_node: int = 8,
             rsv_node_pct: int = 5, owners: int = 40, owner_pod_pct: int = 10, required_pct: int = 2,
             gpu_pod_pct: int = 10, xres_node_pct: int = 0, xres_pod_pct: int = 0, owner_gpu_pct: int = 0) -> Cluster:
    """Reservation + DeviceShare state for config C5: GPU Device objects on gpu_node_pct% of the nodes
    (8 GPUs of 80 GiB, partly used), 1-2 reservations on rsv_node_pct% of the nodes (owner groups, Default /
    Restricted policies, some allocate-once, some already used by assigned pods, 10% with a reservation-order label),
    and per-pod plugin inputs: owner-group pods (owner_pod_pct%, required_pct% with reservation affinity) and GPU
    pods (gpu_pod_pct%: gpu-core + gpu-memory-ratio, nvidia.com/gpu, gpu-memory-ratio alone or gpu-memory, 1% with an
    invalid gpu-core). NodeInfo (c.nodes) already holds the reserve pods and the pods assigned to them.
    xres_node_pct / xres_pod_pct: two registered extended resources (x0 "example.com/fpga": 1-4 per node, pods ask 1;
    x1 "example.com/shared-nic": 1000 per node, pods ask 100-400) on that share of nodes / pods, 1% of the pods asking
    for both (Fit's scalar check over names outside the fixed slots).
    owner_gpu_pct: that share of the owner-group pods also requests GPUs (GPU pods that match reservations)."""
    s = Stream((BASE_SEED + 0x5C5) if seed is None else seed)
    N = c.num_nodes
    P = len(c.pods)
    # ---- GPU devices
    devs = np.zeros(N, abi.NODE_DEVICES_DTYPE)
    gpu_node = s.randint(1, N, 0, 99) < gpu_node_pct
    G = gpus_per_node
    mem = 80 * GiB
    used_steps = s.randint(2, N * G, 0, 7).reshape(N, G)            # used ratio in 0, 25, 50, 75, 100 (more idle)
    used_ratio = np.array([0, 0, 0, 25, 50, 75, 100, 100], np.int64)[used_steps]
    unhealthy = s.randint(3, N * G, 0, 99).reshape(N, G) == 0        # 1% of devices report zero resources
    nn = c.numa["node_numa"] if c.numa is not None else None
    for i in np.nonzero(gpu_node)[0]:
        d = devs[i]
        d["has_device"] = 1
        d["num_gpus"] = G
        tot_core = tot_ratio = tot_mem = 0
        u_core = u_ratio = u_mem = 0
        # Topology.NodeID: the GPUs spread evenly over the node's NUMA zones in minor order (two NUMA nodes without
        # NRT zones), as fakeDeviceCR (deviceshare/device_allocator_test.go:49-57) places 8 GPUs on 2 nodes
        nz = int(nn["num_zones"][i]) if nn is not None else 0
        for g in range(G):
            gg = d["gpus"][g]
            gg["minor"] = g
            gg["has_info"] = 1
            gg["numa_node"] = int(nn["zones"][i][g * nz // G]["node_id"]) if nz else g * 2 // G
            if unhealthy[i, g]:
                continue
            gg["total"] = (100, 100, mem)
            ur = int(used_ratio[i, g])
            gg["used"] = (ur, ur, ur * mem // 100)
            tot_core += 100; tot_ratio += 100; tot_mem += mem
            u_core += ur; u_ratio += ur; u_mem += ur * mem // 100
        d["allocatable"] = (G, tot_core, tot_core, tot_mem, tot_ratio)
        d["requested"] = (int((used_ratio[i] == 100).sum()), u_core, u_core, u_mem, u_ratio)
    # ---- reservations
    has_r = s.randint(4, N, 0, 99) < rsv_node_pct
    nr = np.where(has_r, s.randint(5, N, 1, 2), 0)
    R = int(nr.sum())
    rnode = np.repeat(np.arange(N, dtype=np.uint32), nr)
    rsv = np.zeros(R, abi.RESERVATION_DTYPE)
    rsv["uid"] = s.u64(6, R) | np.uint64(1)
    rsv["owner_key"] = (s.randint(7, R, 1, owners)).astype(np.uint64)
    rsv["node"] = rnode
    pol = s.randint(8, R, 0, 9)
    rsv["allocate_policy"] = np.where(pol < 7, abi.RSV_POLICY["Default"], abi.RSV_POLICY["Restricted"])
    rsv["order"] = np.where(s.randint(9, R, 0, 9) == 0, s.randint(10, R, 1, 1000), 0)
    rsv["available"] = 1
    rsv["unschedulable"] = (s.randint(11, R, 0, 49) == 0).astype(np.int32)
    rsv["allocate_once"] = (s.randint(12, R, 0, 4) == 0).astype(np.int32)
    rcpu = np.array([2000, 4000, 8000, 16000], np.int64)[s.randint(13, R, 0, 3)]
    rmem = np.array([4, 8, 16, 32], np.int64)[s.randint(14, R, 0, 3)] * GiB
    alloc = np.zeros((R, abi.GS_NUM_RES), np.int64)
    alloc[:, 0], alloc[:, 1] = rcpu, rmem
    rsv["allocatable"] = alloc
    rsv["allocatable_mask"] = 3
    rsv["resource_names_mask"] = 3
    used = s.randint(15, R, 0, 9) < 3                                  # 30% already used by 1-2 assigned pods
    npods = np.where(used, s.randint(16, R, 1, 2), 0)
    allocated = np.zeros((R, abi.GS_NUM_RES), np.int64)
    allocated[:, 0] = np.where(used, s.randint(17, R, 1, 10) * rcpu // 10 // 100 * 100, 0)
    allocated[:, 1] = np.where(used, s.randint(18, R, 1, 10) * rmem // 10 // MiB * MiB, 0)
    rsv["allocated"] = allocated
    rsv["allocated_mask"] = np.where(used, 3, 0).astype(np.uint32)
    rsv["assigned_pods"] = npods
    # NodeInfo holds the reserve pod (its requests = Allocatable) and the pods assigned to the reservation
    nodes = c.nodes
    for k in range(R):
        i = int(rnode[k])
        for sl in (0, 1):
            nodes["requested"][i, sl] += alloc[k, sl] + allocated[k, sl]
            nodes["nonzero_requested"][i, sl] += alloc[k, sl] + allocated[k, sl]
        nodes["pod_count"][i] += 1 + int(npods[k])
    # ---- per-pod plugin inputs
    ext = np.zeros(P, abi.POD_EXT_DTYPE)
    kind = s.randint(20, P, 0, 99)
    own = kind < owner_pod_pct
    ext["reservation_owner"] = np.where(own, s.randint(21, P, 1, owners), 0).astype(np.uint64)
    ext["reservation_required"] = (own & (s.randint(22, P, 0, 99) < required_pct * 100 // max(1, owner_pod_pct))).astype(np.int32)
    gp = (kind >= owner_pod_pct) & (kind < owner_pod_pct + gpu_pod_pct)
    if owner_gpu_pct:
        gp |= own & (s.randint(40, P, 0, 99) < owner_gpu_pct)
    gk = s.randint(23, P, 0, 99)
    amount = np.array([25, 50, 100, 100, 200, 400], np.int64)[s.randint(24, P, 0, 5)]
    nv = s.randint(25, P, 1, 2)
    masks = np.zeros(P, np.uint32)
    reqs = np.zeros((P, abi.GS_NUM_GPU_NAMES), np.int64)
    CO, RA, ME, NV = (abi.GPU_NAMES["koordinator.sh/gpu-core"], abi.GPU_NAMES["koordinator.sh/gpu-memory-ratio"],
                      abi.GPU_NAMES["koordinator.sh/gpu-memory"], abi.GPU_NAMES["nvidia.com/gpu"])
    for p in np.nonzero(gp)[0]:
        if gk[p] < 50:
            reqs[p, CO] = reqs[p, RA] = amount[p]
            masks[p] = (1 << CO) | (1 << RA)
        elif gk[p] < 80:
            reqs[p, NV] = nv[p]
            masks[p] = 1 << NV
        elif gk[p] < 90:
            reqs[p, RA] = min(amount[p], 100)
            masks[p] = 1 << RA
        elif gk[p] < 99:
            reqs[p, CO] = 50
            reqs[p, ME] = 40 * GiB
            masks[p] = (1 << CO) | (1 << ME)
        else:
            reqs[p, CO] = reqs[p, RA] = 150                          # invalid percentage: PreFilter fails
            masks[p] = (1 << CO) | (1 << RA)
    ext["gpu_request_mask"] = masks
    ext["gpu_requests"] = reqs
    if xres_node_pct:
        xn = s.randint(30, N, 0, 99) < xres_node_pct
        fp = s.randint(31, N, 1, 4)
        devs["xres_allocatable"][:, 0] = np.where(xn, fp, 0)
        devs["xres_requested"][:, 0] = np.where(xn, np.minimum(s.randint(32, N, 0, 2), fp), 0)
        devs["xres_allocatable"][:, 1] = np.where(xn, 1000, 0)
        devs["xres_requested"][:, 1] = np.where(xn, s.randint(33, N, 0, 9) * 100, 0)
    if xres_pod_pct:
        xk = s.randint(34, P, 0, 999)
        xp0 = xk < xres_pod_pct * 5
        xp1 = (xk >= xres_pod_pct * 5) & (xk < xres_pod_pct * 10)
        both = xk >= 990
        ext["xres_requests"][:, 0] = np.where(xp0 | both, 1, 0)
        ext["xres_requests"][:, 1] = np.where(xp1 | both, s.randint(35, P, 1, 4) * 100, 0)
        ext["xres_request_mask"] = (np.where(xp0 | both, 1, 0) | np.where(xp1 | both, 2, 0)).astype(np.uint32)
    c.ext = {"devices": devs, "reservations": rsv, "pod_ext": ext}
    return c


def load_ext_into(engine, c: Cluster, args) -> None:
    """Push the Reservation / DeviceShare state of make_ext into an Engine / Oracle."""
    engine.ext_configure(args)
    engine.upsert_devices(c.ext["devices"])
    if len(c.ext["reservations"]):
        engine.upsert_reservations(c.ext["reservations"])
