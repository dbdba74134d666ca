"""Node sampling on the HIP path ([upstream] findNodesThatPassFilters with percentageOfNodesToScore < 100,
parallelism-1 rotation order from nextStartNodeIndex; gs_config.sample_nodes): the commit kernel's window
selection against the oracle, bit-exact — node, max score, ties and feasible count (= the window size) of
every pod, and nextStartNodeIndex after every call. Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from oracle import oracle as orc
from tests.test_gpu_parity import homogeneous_cluster

pytestmark = pytest.mark.gpu


def sampling_pair(c, pct, **kw):
    from koordinator_amd.engine import Engine
    cfg = config.make_config(c.num_nodes, percentage_of_nodes_to_score=pct, **kw)
    e, o = Engine(cfg), orc.Oracle(cfg)
    if kw.get("enabled", 0) & abi.GS_ENABLE_NUMA_FILTER:
        e.verify_cpusets(True)
    synth.load_into(e, c)
    synth.load_into(o, c)
    return e, o


def check(e, o, pods, lo=0):
    seq = np.arange(lo, lo + len(pods), dtype=np.uint64)
    got, want = e.schedule(pods, seq), o.schedule(pods, seq)
    for f in ("node", "score", "ties", "feasible"):
        bad = np.nonzero(got[f] != want[f])[0]
        assert not len(bad), f"{f} differs at pod {lo + bad[0]}: gpu {got[bad[0]]} oracle {want[bad[0]]}"
    assert e.stats()["next_start_node_index"] == o.next_start_node_index
    return got


def loaded_cluster(nodes, pods, cid):
    c = synth.make_cluster(nodes, pods, cid)
    c.pods["requests"][::3, 0] = 60_000     # many infeasible nodes per pod
    c.pods["requests"][5::17, 0] = 400_000  # FitError: the whole ring is processed
    c.pods["request_mask"][:] |= 0x1
    return c


@pytest.mark.parametrize("batch", [1, 16, 128])
def test_sampling_adaptive_matches_oracle(batch):
    c = loaded_cluster(3000, 600, 11)
    e, o = sampling_pair(c, 0, batch_size=batch)
    got = check(e, o, c.pods)
    k = orc.num_feasible_nodes_to_find(3000, 0)
    assert got["feasible"].max() == k and (got["node"] < 0).any()
    assert e.mirror_check() == 0


def test_sampling_percentage_across_calls():
    """pct = 10 over several gs_schedule calls: nextStartNodeIndex carries over, pipelined batches read it on the
    device from the batch before."""
    c = loaded_cluster(5000, 900, 12)
    e, o = sampling_pair(c, 10)
    for lo in range(0, 900, 300):
        check(e, o, c.pods[lo:lo + 300], lo)
    assert e.mirror_check() == 0


def test_sampling_numa_profile():
    c = synth.make_cluster(2000, 300, 13)
    synth.make_numa(c, numa_policy_pct=60, cpuset_pod_pct=30)
    e, o = sampling_pair(c, 0, enabled=abi.GS_ENABLE_ALL)
    got = check(e, o, c.pods)
    assert (got["flags"] & abi.GS_PLACED_CPUSET).any()
    assert e.mirror_check() == 0


def test_sampling_homogeneous_ties():
    """Identical nodes: every window node ties; the jp-th tie is located in window (rotation) order."""
    c = homogeneous_cluster(4000, 200, 14)
    e, o = sampling_pair(c, 5)
    got = check(e, o, c.pods)
    assert got["ties"].max() >= 100


def test_sampling_refuses_several_ranks_under_levels(monkeypatch):
    """The level exchange holds a shard's rows only: node sampling's rotation window needs every node's verdict."""
    monkeypatch.setenv("GS_XCHG", "levels")
    c = synth.make_cluster(500, 8, 15)
    e, _ = sampling_pair(c, 0)
    from koordinator_amd.engine import GpuScoreError
    with pytest.raises(GpuScoreError, match="score-row exchange"):
        e.comm_init_callback(2, 0, lambda send: [send, send])


@pytest.mark.parametrize("n,pct", [(2, 0), (3, 10)])
def test_sampling_on_several_ranks_score_rows(n, pct):
    """Node sampling on several ranks (threads over the in-process device transport, score-row exchange): every rank
    holds every node's scores after the all-gather and resolves the rotation window itself; placements and
    nextStartNodeIndex of every rank equal the oracle's."""
    import threading
    from koordinator_amd.engine import Engine, LocalGroup
    c = loaded_cluster(4000, 500, 18 + n)
    cfg = config.make_config(c.num_nodes, percentage_of_nodes_to_score=pct)
    g = LocalGroup(n)
    engines = [Engine(cfg) for _ in range(n)]
    for r, x in enumerate(engines):
        synth.load_into(x, c)
        x.comm_init_local(g, r)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    res = [None] * n

    def run(r):
        try:
            res[r] = np.concatenate([engines[r].schedule(c.pods[k:k + 250], seq[k:k + 250]) for k in (0, 250)])
        except Exception as ex:   # noqa: BLE001 (reported per rank)
            res[r] = ex
    th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=200)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods, seq)
    for r in range(n):
        assert not isinstance(res[r], Exception) and res[r] is not None, (r, res[r])
        for f in ("node", "score", "ties", "feasible"):
            assert np.array_equal(res[r][f], want[f]), (r, f)
        assert engines[r].stats()["next_start_node_index"] == o.next_start_node_index
    assert want["feasible"].max() == orc.num_feasible_nodes_to_find(4000, pct)


@pytest.mark.parametrize("kind", ["homogeneous", "loaded"])
def test_sampling_window_spans_several_passes(kind):
    """Windows longer than one 4096-position pass of the commit kernel: the scan continues across passes and the
    tie location re-reads them."""
    if kind == "homogeneous":
        c = homogeneous_cluster(10_000, 120, 16)
        e, o = sampling_pair(c, 50)   # K = 5000 feasible of 10000: every window spans two passes
    else:
        c = loaded_cluster(12_000, 240, 17)
        e, o = sampling_pair(c, 30)   # K = 3600, sparse feasibility for the 60-core pods
    got = check(e, o, c.pods)
    assert got["feasible"].max() > 4096 or (got["feasible"] < 3600).any()
    assert e.mirror_check() == 0


def test_sampling_special_pods_and_host_cuts():
    """Node sampling with pods that run in a batch of their own (UID in an assign cache, a PodMetric carrying the
    pod's name, DaemonSet / terminated pods) and with batches cut for a host-side cpuset Reserve (topologies
    outside the device scope): the start index survives every kind of batch boundary."""
    c = synth.make_cluster(1500, 300, 18)
    synth.make_numa(c, numa_policy_pct=40, cpuset_pod_pct=60, mixed=True)
    pods = c.pods.copy()
    pods["flags"][5] |= abi.GS_POD_DAEMONSET
    pods["flags"][6] |= abi.GS_POD_TERMINATED
    pods["uid"][7] = c.assigned_pods["uid"][0]
    pods["name_key"][8] = c.pod_metrics["name_key"][0]
    e, o = sampling_pair(c, 0, enabled=abi.GS_ENABLE_ALL, batch_size=64)
    check(e, o, pods[:180])
    check(e, o, pods[180:], 180)
    assert e.stats()["cuts"] > 0, "no host-side cut exercised"
    assert e.mirror_check() == 0
