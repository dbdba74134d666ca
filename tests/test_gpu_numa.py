"""NodeNUMAResource on the HIP path vs the CPU oracle (bit-exact): reference golden vectors, per-pair Filter codes
and per-plugin scores on synthetic C3 clusters, and sequential scheduling incl. Reserve (NUMA splits and the
cpusets chosen for LSE/LSR pods), with the HBM mirror re-derived on the host after every run."""
import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from oracle import oracle as orc
from tests import numa_util as nu

pytestmark = pytest.mark.gpu


def engine_cls():
    from koordinator_amd.engine import Engine
    return Engine


S = nu.load()


@pytest.mark.parametrize("case", S["cases"], ids=lambda c: c["name"].replace(" ", "_"))
def test_numa_score_golden_gpu(case):
    e, pod = nu.build(case, engine_cls())
    _, codes, plugin = e.evaluate(np.array([pod], abi.POD_DTYPE))
    assert (codes[0] == 0).all(), f"{case['src']}: filter rejected {codes[0]}"
    assert list(plugin[0, :, abi.GS_PLUGIN_NUMA]) == case["want"], case["src"]


def numa_pair(c, **kw):
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL, **kw)
    e = engine_cls()(cfg)
    e.verify_cpusets(True)   # every device-chosen cpuset is re-checked against the host takeCPUs
    o = orc.Oracle(cfg)
    synth.load_into(e, c)
    synth.load_into(o, c)
    return e, o


@pytest.mark.parametrize("nodes,pods,pol,cs", [(1000, 96, 30, 20), (700, 64, 90, 50), (300, 128, 100, 100)])
def test_numa_evaluate_matches_oracle(nodes, pods, pol, cs):
    c = synth.make_cluster(nodes, pods, 1)
    synth.make_numa(c, numa_policy_pct=pol, cpuset_pod_pct=cs)
    e, o = numa_pair(c)
    gs, gc, gp = e.evaluate(c.pods)
    os_, oc, op = o.evaluate(c.pods)
    assert np.array_equal(gc, oc), f"filter codes differ at {np.argwhere(gc != oc)[:5]}"
    assert np.array_equal(gp, op), f"plugin scores differ at {np.argwhere(gp != op)[:5]}"
    assert np.array_equal(gs, os_)


@pytest.mark.parametrize("variant", ["most_allocated", "score_only", "default_spread"])
def test_numa_evaluate_variants(variant):
    c = synth.make_cluster(500, 64, 3)
    synth.make_numa(c, numa_policy_pct=60, cpuset_pod_pct=40)
    kw = {}
    if variant == "most_allocated":
        kw["numa"] = config.numa_args(scoringStrategy={"type": "MostAllocated", "resources": {"cpu": 2, "memory": 1}},
                                      numaScoringStrategy={"type": "MostAllocated"})
    elif variant == "default_spread":
        kw["numa"] = config.numa_args(defaultCPUBindPolicy="SpreadByPCPUs")
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL, **kw)
    if variant == "score_only":
        cfg.enabled = abi.GS_ENABLE_ALL & ~abi.GS_ENABLE_NUMA_FILTER
    e, o = engine_cls()(cfg), orc.Oracle(cfg)
    synth.load_into(e, c)
    synth.load_into(o, c)
    gs, gc, gp = e.evaluate(c.pods)
    os_, oc, op = o.evaluate(c.pods)
    assert np.array_equal(gc, oc)
    assert np.array_equal(gp, op), f"plugin scores differ at {np.argwhere(gp != op)[:5]}"


def _check_schedule(e, o, c, chunks):
    i = 0
    for n in chunks:
        got = e.schedule(c.pods[i:i + n], np.arange(i, i + n, dtype=np.uint64))
        want = o.schedule(c.pods[i:i + n], np.arange(i, i + n, dtype=np.uint64))
        for f in ("node", "score", "ties", "feasible"):
            bad = np.nonzero(got[f] != want[f])[0]
            assert not len(bad), f"{f} differs at pod {i + bad[0]}: gpu {got[bad[0]]} oracle {want[bad[0]]}"
        mask = abi.GS_PLACED_NUMA | abi.GS_PLACED_CPUSET | (0xF << abi.GS_PLACED_AFFINITY_SHIFT)
        assert np.array_equal(got["flags"] & mask, want["flags"] & mask), "Reserve flags differ"
        for j in np.nonzero(got["flags"] & (abi.GS_PLACED_CPUSET | abi.GS_PLACED_NUMA))[0]:
            node, uid = int(got["node"][j]), int(c.pods["uid"][i + j])
            ga, oa = e.allocation(node, uid), o.allocation(node, uid)
            assert (ga is None) == (oa is None), f"pod {i + j}: allocation presence differs"
            if ga is not None:
                assert ga.tobytes() == oa.tobytes(), f"pod {i + j}: allocation differs (cpuset / NUMA split)"
        i += n
    assert e.mirror_check() == 0, "HBM mirror diverged from the host mirror"


@pytest.mark.parametrize("batch", [1, 16, 128])
def test_numa_schedule_matches_oracle(batch):
    c = synth.make_cluster(2000, 300, 1)
    synth.make_numa(c)
    e, o = numa_pair(c, batch_size=batch)
    _check_schedule(e, o, c, [300])


def test_numa_schedule_dense_policies_and_cpusets():
    c = synth.make_cluster(400, 400, 5)
    synth.make_numa(c, numa_policy_pct=90, cpuset_pod_pct=60)
    e, o = numa_pair(c)
    _check_schedule(e, o, c, [150, 1, 249])


@pytest.mark.parametrize("batch", [16, 128])
def test_numa_schedule_mixed_topologies(batch):
    """Sibling-interleaved CPU numbering, SMT 4, 256-core SMT-1 nodes (outside the device cpuset scope: host
    takeCPUs and a batch cut), maxRefCount 2 nodes (device RefCount ordering), PCPU- and NUMANode-level exclusivity."""
    c = synth.make_cluster(1500, 300, 7)
    synth.make_numa(c, numa_policy_pct=40, cpuset_pod_pct=60, mixed=True)
    e, o = numa_pair(c, batch_size=batch)
    _check_schedule(e, o, c, [200, 100])
    st = e.stats()
    assert st["cuts"] > 0, "the host cpuset path was not exercised"


def test_numa_schedule_after_release():
    c = synth.make_cluster(600, 200, 6)
    synth.make_numa(c, numa_policy_pct=50, cpuset_pod_pct=40)
    e, o = numa_pair(c)
    _check_schedule(e, o, c, [100])
    # release the existing allocations of the first 40 nodes, then keep scheduling
    nodes = c.numa["alloc_nodes"][:40]
    uids = c.numa["allocs"]["uid"][:40]
    e.release_allocations(nodes, uids)
    o.release_allocations(nodes, uids)
    _check_schedule(e, o, c.__class__(**{**c.__dict__, "pods": c.pods[100:]}), [100])


def test_numa_two_ranks_on_one_gpu_callback_transport():
    """Node-sharded NodeNUMAResource path (2 ranks, host all-gather) on one GPU: every rank replays the same Reserve
    (NUMA splits and device-chosen cpusets; a rank reuses the batch-start affinity only for its own shard) and both
    match the oracle."""
    import threading
    c = synth.make_cluster(1201, 200, 17)
    synth.make_numa(c, numa_policy_pct=50, cpuset_pod_pct=50, mixed=True)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL)
    E = engine_cls()
    engines = [E(cfg), E(cfg)]
    for x in engines:
        synth.load_into(x, c)
        x.verify_cpusets(True)
    barrier = threading.Barrier(2)
    slots = [None, None]

    def make_ag(r):
        def ag(data):
            slots[r] = data
            barrier.wait()
            out = list(slots)
            barrier.wait()
            return out
        return ag

    for r, x in enumerate(engines):
        x.comm_init_callback(2, r, make_ag(r))
    res = [None, None]

    def run(r):
        res[r] = engines[r].schedule(c.pods, np.arange(len(c.pods), dtype=np.uint64))

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods, np.arange(len(c.pods), dtype=np.uint64))
    mask = abi.GS_PLACED_NUMA | abi.GS_PLACED_CPUSET | (0xF << abi.GS_PLACED_AFFINITY_SHIFT)
    for r in range(2):
        assert res[r] is not None, f"rank {r} did not finish"
        for f in ("node", "score", "ties", "feasible"):
            bad = np.nonzero(res[r][f] != want[f])[0]
            assert not len(bad), f"rank {r}: {f} differs at pod {bad[0]}"
        assert np.array_equal(res[r]["flags"] & mask, want["flags"] & mask), f"rank {r}: Reserve flags differ"
        for j in np.nonzero(want["flags"] & abi.GS_PLACED_CPUSET)[0]:
            node, uid = int(want["node"][j]), int(c.pods["uid"][j])
            assert engines[r].allocation(node, uid).tobytes() == o.allocation(node, uid).tobytes(), (r, j)
        assert engines[r].mirror_check() == 0
