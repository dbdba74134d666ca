"""Builds a NodeNUMAResource golden scenario (tests/golden/numa_score.json) into an Engine or an Oracle."""
import json
import os

import numpy as np

from koordinator_amd import abi, config, numa

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name="numa_score.json"):
    return json.load(open(os.path.join(HERE, "golden", name)))


def build(case, cls, device=0):
    nodes_spec = case["nodes"]
    N = len(nodes_spec)
    a = case["args"]
    extra = {"numaScoringStrategy": a["numa_scoring"]} if "numa_scoring" in a else {}
    nargs = config.numa_args(scoringStrategy={"type": a["scoring"], "resources": a["weights"]}, **extra)
    enabled = abi.GS_ENABLE_NUMA_SCORE | (abi.GS_ENABLE_NUMA_FILTER if case["filter"] else 0)
    cfg = config.make_config(N, enabled=enabled, numa=nargs, device=device)
    e = cls(cfg)
    nodes = np.zeros(N, abi.NODE_DTYPE)
    for i, n in enumerate(nodes_spec):
        nodes[i]["allocatable"][abi.GS_RES_CPU] = n["cpu_milli"]
        nodes[i]["allocatable"][abi.GS_RES_MEMORY] = n["memory"]
        nodes[i]["allowed_pod_number"] = 110
        nodes[i]["requested"][abi.GS_RES_CPU] = n.get("requested_cpu", 0)
    e.set_now(0)
    e.upsert_nodes(nodes)
    metrics = np.zeros(N, abi.METRIC_DTYPE)
    e.upsert_metrics(metrics)
    recs = []
    for n in nodes_spec:
        tid = e.register_topology(numa.test_topology(*n["topology"])) if n["topology"] else None
        recs.append(numa.node_numa(tid, zones=[tuple(z) for z in n["zones"]], numa_policy=n["numa_policy"],
                                   node_cpu_bind=n.get("node_cpu_bind", ""),
                                   numa_allocate_strategy=n.get("numa_allocate_strategy", ""),
                                   node_cpu_ratio=n.get("node_cpu_ratio", -1.0),
                                   has_options=n.get("has_options", True)))
    e.upsert_numa(np.array(recs, abi.NODE_NUMA_DTYPE))
    if case["allocations"]:
        allocs = [numa.pod_allocation(x["uid"], x["cpus"], [tuple(z) for z in x["numa"]]) for x in case["allocations"]]
        e.update_allocations([x["node"] for x in case["allocations"]], np.array(allocs, abi.POD_ALLOCATION_DTYPE))
    p = case["pod"]
    pod = np.zeros(1, abi.POD_DTYPE)[0]
    mask = 0
    if "cpu" in p:
        pod["requests"][abi.GS_RES_CPU] = p["cpu"]
        pod["nonzero_requests"][0] = p["cpu"]
        mask |= 1 << abi.GS_RES_CPU
    if "batch_cpu" in p:
        pod["requests"][abi.GS_RES_BATCH_CPU] = p["batch_cpu"]
        mask |= 1 << abi.GS_RES_BATCH_CPU
    if "memory" in p:
        pod["requests"][abi.GS_RES_MEMORY] = p["memory"]
        pod["nonzero_requests"][1] = p["memory"]
        mask |= 1 << abi.GS_RES_MEMORY
    pod["request_mask"] = mask
    pod["priority_class"] = abi.GS_PRIO_PROD if p.get("prod") else abi.GS_PRIO_NONE
    pod["qos_class"] = {"": 0, "LSE": abi.GS_QOS_LSE, "LSR": abi.GS_QOS_LSR}[p.get("qos", "")]
    pod["preferred_cpu_bind_policy"] = abi.CPU_BIND[p.get("preferred", "")]
    pod["required_cpu_bind_policy"] = abi.CPU_BIND[p.get("required", "")]
    pod["uid"] = 0xABCDEF
    return e, pod
