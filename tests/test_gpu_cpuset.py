"""The device cpuset Reserve past 64 cores and with maxRefCount 2 (koordinator_amd/csrc/gs_cpuset_dev.h).

* cpu_accumulator_test.go TestTakeCPUsWithMaxRefCount (:560-599) and TestTakeCPUsSortByRefCount (:601-648): each
  sequence's pods scheduled in ONE gs_schedule call on a one-node cluster (maxRefCount 2, MostAllocated), so every
  step after the first is the commit kernel's Reserve on a row an earlier pod of the batch landed on; each pod's cpuset
  must be the test's, the batch must not be cut (the device selected every cpuset), and the host's takeCPUs must agree
  (verify_cpusets). The same harness runs on the oracle engine (CPU).
* The C3 topology (32-128 cores SMT2, 2 sockets, 2 / 4 NUMA nodes; synth.make_numa): a cluster of it
  schedules with no cut and no host-resolved pod, bit-exact against the oracle's sequential scheduleOne.
"""
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi, config, numa, synth
from oracle import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
SEQS = json.load(open(os.path.join(HERE, "golden", "numa_takecpus.json")))["sequences"]


def _engine(gpu: bool):
    if gpu:
        from koordinator_amd.engine import Engine
        return Engine
    return orc.Oracle


def run_sequence(seq, cls):
    s, n, c, p = seq["topology"]
    total = s * n * c * p
    cfg = config.make_config(1, enabled=abi.GS_ENABLE_ALL)
    e = cls(cfg)
    nodes = np.zeros(1, abi.NODE_DTYPE)
    nodes[0]["allocatable"][abi.GS_RES_CPU] = 1000 * 1000   # Fit never binds: the sequences share CPUs (RefCount 2)
    nodes[0]["allocatable"][abi.GS_RES_MEMORY] = 1 << 40
    nodes[0]["allowed_pod_number"] = 110
    e.set_now(0)
    e.upsert_nodes(nodes)
    e.upsert_metrics(np.zeros(1, abi.METRIC_DTYPE))
    tid = e.register_topology(numa.test_topology(s, n, c, p))
    zones = [(z, total * 1000 // (s * n), 1 << 36) for z in range(s * n)]
    e.upsert_numa(np.array([numa.node_numa(tid, zones=zones, numa_allocate_strategy="MostAllocated",
                                           max_ref_count=seq["max_ref"])], abi.NODE_NUMA_DTYPE))
    steps = seq["steps"]
    pods = np.zeros(len(steps), abi.POD_DTYPE)
    for k, st in enumerate(steps):
        pods[k]["requests"][abi.GS_RES_CPU] = st["needed"] * 1000
        pods[k]["limits"][abi.GS_RES_CPU] = st["needed"] * 1000
        pods[k]["nonzero_requests"][0] = st["needed"] * 1000
        pods[k]["requests"][abi.GS_RES_MEMORY] = 1 << 20
        pods[k]["limits"][abi.GS_RES_MEMORY] = 1 << 20
        pods[k]["nonzero_requests"][1] = 1 << 20
        pods[k]["request_mask"] = (1 << abi.GS_RES_CPU) | (1 << abi.GS_RES_MEMORY)
        pods[k]["priority_class"] = abi.GS_PRIO_PROD
        pods[k]["qos_class"] = abi.GS_QOS_LSR
        # takeCPUs(bind) as the test calls it: the pod's preferred policy (a required one would first filter the
        # available CPUs, filterCPUsByRequiredCPUBindPolicy)
        pods[k]["preferred_cpu_bind_policy"] = abi.CPU_BIND[st["bind"]]
        pods[k]["uid"] = 0x51000 + k
    if hasattr(e, "verify_cpusets"):
        e.verify_cpusets(True)
        e.reset_stats()
    out = e.schedule(pods, np.arange(len(steps), dtype=np.uint64))
    got = []
    for k in range(len(steps)):
        assert out["node"][k] == 0, f"{seq['src']}: step {k} not placed"
        a = e.allocation(0, int(pods[k]["uid"]))
        got.append(numa.cpus_of(a["cpuset"]))
    return e, got


@pytest.mark.parametrize("seq", SEQS, ids=lambda s: s["src"].split()[-1])
def test_maxrefcount_sequences_oracle_engine(seq):
    _, got = run_sequence(seq, orc.Oracle)
    assert got == [st["want"] for st in seq["steps"]], seq["src"]


@pytest.mark.gpu
@pytest.mark.parametrize("seq", SEQS, ids=lambda s: s["src"].split()[-1])
def test_maxrefcount_sequences_gpu(seq):
    e, got = run_sequence(seq, _engine(True))
    assert got == [st["want"] for st in seq["steps"]], seq["src"]
    st = e.stats()
    assert st["cuts"] == 0, f"{seq['src']}: the batch was cut ({st['cuts']}): a cpuset left the device"


def c3_cluster(n_nodes, n_pods, **kw):
    c = synth.make_cluster(n_nodes, n_pods, config_id=2)
    synth.make_numa(c, **kw)
    return c


def test_c3_topology_is_the_survey_shape():
    """2 sockets, 2 or 4 NUMA nodes, 32-128 physical cores, SMT2 (64-256 logical CPUs), and the
    node's allocatable CPUs = its logical CPUs."""
    c = c3_cluster(400, 10)
    seen = set()
    for t in c.numa["topologies"]:
        nc = int(t["num_cpus"])
        cores = {(int(t["socket_id"][i]), int(t["core_id"][i])) for i in range(nc)}
        assert len({int(t["socket_id"][i]) for i in range(nc)}) == 2
        assert len({int(t["node_id"][i]) for i in range(nc)}) in (2, 4)
        assert nc == 2 * len(cores) and 32 <= len(cores) <= 128
        seen.add(len(cores))
    assert max(seen) == 128 and min(seen) == 32
    rec = c.numa["node_numa"]
    for i in range(len(c.nodes)):
        t = c.numa["topologies"][int(rec[i]["topology"])]
        alloc = int(c.nodes["allocatable"][i][abi.GS_RES_CPU])
        amp = float(rec[i]["node_cpu_amplification_ratio"])
        assert alloc == (int(np.ceil(int(t["num_cpus"]) * 1000 * amp)) if amp > 1 else int(t["num_cpus"]) * 1000)


@pytest.mark.gpu
@pytest.mark.parametrize("kw", [dict(), dict(numa_policy_pct=60, cpuset_pod_pct=60),
                                dict(numa_policy_pct=40, cpuset_pod_pct=50, mixed=True)],
                         ids=["c3", "dense-cpuset", "mixed-maxref2"])
def test_c3_wide_topology_bit_exact_no_cuts(kw):
    from koordinator_amd.engine import Engine
    c = c3_cluster(3000, 2048, **kw)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL)
    e = Engine(cfg)
    synth.load_into(e, c)
    e.verify_cpusets(True)
    e.reset_stats()
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    got = e.schedule(c.pods, seq)
    want = o.schedule(c.pods, seq, nthreads=8)
    for f in ("node", "score", "ties", "feasible"):
        bad = np.nonzero(got[f] != want[f])[0]
        assert not len(bad), f"{f} differs at pods {bad[:8]}"
    placed = got["node"] >= 0
    for k in np.nonzero(placed & (c.pods["qos_class"] != abi.GS_QOS_LS))[0][:400]:
        a, b = e.allocation(int(got["node"][k]), int(c.pods["uid"][k])), o.allocation(int(got["node"][k]),
                                                                                   int(c.pods["uid"][k]))
        assert (a is None) == (b is None)
        if a is not None:
            assert numa.cpus_of(a["cpuset"]) == numa.cpus_of(b["cpuset"]), f"pod {k} cpuset"
    st = e.stats()
    if not kw.get("mixed"):   # (mixed: SMT-1 classes of more than 128 cores stay on the host path by design)
        assert st["cuts"] == 0 and st["slowpath_pods"] == 0, st
