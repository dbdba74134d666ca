"""Parity of the HIP path (through the C-ABI) with the CPU oracle. Needs an MI355X: -m gpu.

Bit-exact is the bar everywhere: feasibility codes, per-plugin int64 scores, weighted totals, and the
selected node / max score / tie count of every sequentially scheduled pod.
"""
import threading

import numpy as np
import pytest

from koordinator_amd import abi, config, objects, synth
from oracle import oracle as orc
from tests import golden_util as gu

pytestmark = pytest.mark.gpu


def engine_cls():
    from koordinator_amd.engine import Engine
    return Engine


def pair(cluster, **cfg_kw):
    cfg = config.make_config(cluster.num_nodes, **cfg_kw)
    e = engine_cls()(cfg)
    o = orc.Oracle(cfg)
    synth.load_into(e, cluster)
    synth.load_into(o, cluster)
    return e, o


G = gu.load()


@pytest.mark.parametrize("case", G["filter_expired"] + G["filter_usage"], ids=lambda c: c["name"])
def test_golden_loadaware_filter(case):
    eng, pod = gu.build(case, engine_cls())
    _, codes, _ = eng.evaluate(np.array([pod], abi.POD_DTYPE))
    assert bool(codes[0, 0] & abi.GS_FAIL_LOADAWARE) == case["want_fail"], case["src"]


@pytest.mark.parametrize("case", G["score"], ids=lambda c: c["name"])
def test_golden_loadaware_score(case):
    eng, pod = gu.build(case, engine_cls())
    _, _, plugin = eng.evaluate(np.array([pod], abi.POD_DTYPE))
    assert plugin[0, 0, abi.GS_PLUGIN_LOADAWARE] == case["want"], case["src"]


@pytest.mark.parametrize("cid,nodes,pods", [(0, 1000, 300), (1, 5000, 64)])
def test_evaluate_matches_oracle(cid, nodes, pods):
    c = synth.make_cluster(nodes, pods, cid)
    c.pods["requests"][::5, 0] = 40_000          # 40-core pods: exercise Fit "Insufficient cpu"
    c.pods["requests"][1::7, 2] = 480 << 30      # and "Insufficient ephemeral-storage"
    c.pods["request_mask"][:] |= 0x7
    e, o = pair(c)
    gs, gc, gp = e.evaluate(c.pods)
    os_, oc, op = o.evaluate(c.pods)
    assert np.array_equal(gc, oc), "filter codes differ"
    assert np.array_equal(gp, op), "per-plugin scores differ"
    assert np.array_equal(gs, os_), "weighted totals differ"
    # the synthetic cluster exercises every verdict
    for bit in (abi.GS_FAIL_LOADAWARE, abi.GS_FAIL_FIT_CPU, abi.GS_FAIL_FIT_EPHEMERAL):
        assert (gc & bit).any(), bit
    assert (gc == 0).any()


def _check_schedule(e, o, pods, seq=None):
    got = e.schedule(pods, seq)
    want = o.schedule(pods, seq)
    for f in ("node", "score", "ties", "feasible"):
        bad = np.nonzero(got[f] != want[f])[0]
        assert len(bad) == 0, f"{f} differs first at pod {bad[0]}: gpu {got[bad[0]]} oracle {want[bad[0]]}"
    assert e.mirror_check() == 0
    return got


@pytest.mark.parametrize("batch", [1, 7, 128])
def test_schedule_c1_matches_oracle(batch):
    c = synth.make_cluster(1000, 1000, 0)
    e, o = pair(c, batch_size=batch)
    got = _check_schedule(e, o, c.pods)
    assert (got["node"] >= 0).all()


def test_schedule_c2_slice_matches_oracle():
    c = synth.make_cluster(5000, 1500, 1)
    e, o = pair(c)
    _check_schedule(e, o, c.pods)
    st = e.stats()
    assert st["pods"] == 1500 and st["batches"] >= 12


def test_schedule_in_chunks_and_custom_seq():
    c = synth.make_cluster(2000, 600, 7)
    e, o = pair(c)
    seq = np.arange(10_000, 10_600, dtype=np.uint64)
    for lo in range(0, 600, 150):
        _check_schedule(e, o, c.pods[lo:lo + 150], seq[lo:lo + 150])


@pytest.mark.parametrize("chunk,numa,homog", [(1, False, False), (5, False, False), (32, True, False),
                                              (7, False, True)], ids=["1", "5", "32-numa", "7-ties"])
def test_short_batches_over_long_rows_match_oracle(chunk, numa, homog):
    """A gs_schedule call's first batch of <= 32 pods over rows of >= 4096 entries builds its levels over row slices
    spread across the chip (launch_cand's cs_hist / cs_pick / cs_list kernels, the plain runs between C5's extension
    pods): calls of `chunk` pods on a 20k-node cluster, every placement the oracle's. 7-ties: one level of 20k nodes, too
    large to list (no listed level: the exact full-row path)."""
    c = homogeneous_cluster(20_000, 224, 4) if homog else synth.make_cluster(20_000, 224, 3)
    if numa:
        synth.make_numa(c)
    kw = dict(enabled=abi.GS_ENABLE_ALL) if numa else {}
    e, o = pair(c, **kw)
    for lo in range(0, 224, chunk):
        _check_schedule(e, o, c.pods[lo:lo + chunk], np.arange(lo, min(224, lo + chunk), dtype=np.uint64))
    assert e.stats()["batches"] >= 224 // chunk


@pytest.mark.parametrize("numa", [False, True])
def test_overlapped_levels_match_serial_levels(numa, monkeypatch):
    """Candidate levels built beside the previous batch's commit and fixed up after it (fix_levels_kernel, the
    default) against levels built after the commit (GS_CAND_OVERLAP=0): identical placements, both the oracle's."""
    c = synth.make_cluster(4000, 800, 5)
    if numa:
        synth.make_numa(c)
    kw = dict(enabled=abi.GS_ENABLE_ALL) if numa else {}
    got = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("GS_CAND_OVERLAP", mode)
        e, o = pair(c, **kw)
        got[mode] = _check_schedule(e, o, c.pods)
        assert e.stats()["batches"] >= 6
    for f in ("node", "score", "ties", "feasible"):
        assert (got["1"][f] == got["0"][f]).all()


def homogeneous_cluster(nodes, pods, seed):
    c = synth.make_cluster(nodes, pods, seed)
    c.nodes["requested"] = 0
    c.nodes["nonzero_requested"] = 0
    c.nodes["allocatable"][:, 0] = 64000
    c.nodes["allocatable"][:, 1] = 256 << 30
    c.nodes["raw_allocatable_mask"] = 0
    c.nodes["custom_flags"] = 0
    c.metrics["exists"] = 0
    c.assigned_pods = c.assigned_pods[:0]
    c.assigned_node = c.assigned_node[:0]
    c.assigned_ts = c.assigned_ts[:0]
    c.pod_metrics = c.pod_metrics[:0]
    c.pm_offsets[:] = 0
    return c


@pytest.mark.parametrize("nodes,pods,numa,batch", [(60, 1024, False, 128), (200, 1024, False, 32), (90, 640, True, 128)],
                         ids=["60n", "200n-b32", "90n-numa"])
def test_contention_few_nodes_many_pods(nodes, pods, numa, batch):
    """Many pods on few nodes: most decisions land on rows earlier pods of the batch landed on (re-landings, dirty
    slots past 64, rollbacks, the split selector's exclusions, exact re-records and full decisions), bit-exact."""
    c = synth.make_cluster(nodes, pods, 21)
    if numa:
        synth.make_numa(c)
    kw = dict(enabled=abi.GS_ENABLE_ALL) if numa else {}
    e, o = pair(c, batch_size=batch, **kw)
    got = _check_schedule(e, o, c.pods)
    assert (got["node"] >= 0).sum() > pods // 4


def test_homogeneous_cluster_massive_ties_many_pods():
    """Identical empty nodes, 1,024 pods: every decision a large tie whose winner moves as rows fill up."""
    c = homogeneous_cluster(400, 1024, 5)
    e, o = pair(c)
    got = _check_schedule(e, o, c.pods)
    assert got["ties"].max() > 100


def test_homogeneous_cluster_massive_ties():
    """Identical empty nodes: every node ties, candidate lists overflow -> exact full-row path (in the commit
    kernel on a single shard)."""
    c = homogeneous_cluster(3000, 200, 3)
    e, o = pair(c)
    got = _check_schedule(e, o, c.pods)
    assert got["ties"].max() > 1000
    assert e.stats()["slowpath_pods"] > 0


def test_homogeneous_cluster_two_ranks_host_slow_path():
    """The same on 2 shards: the batch is cut and the host resolves the pod (row_stats / row_select / exchange)."""
    c = homogeneous_cluster(6001, 120, 4)   # 3000 nodes per shard: a top level beyond the list capacity (2048)
    cfg = config.make_config(c.num_nodes)
    res, engines = run_two_ranks(c, cfg)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods)
    for r in range(2):
        for f in ("node", "score", "ties", "feasible"):
            assert np.array_equal(res[r][f], want[f]), (r, f)
        assert engines[r].stats()["slowpath_pods"] > 0


def test_unschedulable_and_special_pods():
    c = synth.make_cluster(800, 100, 11)
    pods = c.pods.copy()
    pods["requests"][::10, 0] = 10**9         # never fits: FitError, nothing assumed
    pods["request_mask"][::10] |= 1
    pods["flags"][5] |= abi.GS_POD_DAEMONSET
    pods["flags"][6] |= abi.GS_POD_TERMINATED
    pods["uid"][7] = c.assigned_pods["uid"][0]      # UID already in an assign cache
    pods["name_key"][8] = c.pod_metrics["name_key"][0]  # a PodMetric carries its name
    e, o = pair(c)
    got = _check_schedule(e, o, pods)
    assert (got["node"][::10] == -1).all()


def test_score_according_prod_usage_and_weights():
    c = synth.make_cluster(1500, 400, 5)
    la = config.loadaware_args(scoreAccordingProdUsage=True, resourceWeights={"cpu": 3, "memory": 1},
                               prodUsageThresholds={"cpu": 55})
    fit = config.fit_args({"cpu": 2, "memory": 1, "ephemeral-storage": 1})
    e, o = pair(c, la=la, fit=fit, weights=(2, 3))
    _check_schedule(e, o, c.pods)


def test_metric_and_node_updates_between_batches():
    c = synth.make_cluster(1200, 600, 9)
    e, o = pair(c)
    _check_schedule(e, o, c.pods[:200])
    # informer events: new metrics for some nodes, a node resize, pods unassigned, clock moves
    idx = np.arange(0, 1200, 7, dtype=np.uint32)
    m = c.metrics[idx].copy()
    m["node_usage"]["cpu_milli"] //= 2
    m["update_time_ns"] = c.now_ns + 30 * synth.SEC
    for x in (e, o):
        x.set_now(c.now_ns + 200 * synth.SEC)
        x.upsert_metrics(m, idx=idx)
        n = c.nodes[:50].copy()
        n["allocatable"][:, 0] += 8000
        x.upsert_nodes(n, idx=np.arange(50, dtype=np.uint32))
        x.unassign(c.assigned_node[:40], c.assigned_pods[:40])
    _check_schedule(e, o, c.pods[200:])


def run_two_ranks(c, cfg):
    E = engine_cls()
    engines = [E(cfg), E(cfg)]
    for x in engines:
        synth.load_into(x, c)
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
        res[r] = engines[r].schedule(c.pods)

    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert res[0] is not None and res[1] is not None
    return res, engines


def test_two_ranks_on_one_gpu_callback_transport():
    """The sharded path (2 ranks, host all-gather) on one GPU: same placements as one rank / the oracle."""
    c = synth.make_cluster(3001, 500, 13)
    cfg = config.make_config(c.num_nodes)
    res, engines = run_two_ranks(c, cfg)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods)
    for r in range(2):
        for f in ("node", "score", "ties", "feasible"):
            assert np.array_equal(res[r][f], want[f]), (r, f)
    assert engines[0].stats()["shard_end"] == engines[1].stats()["shard_begin"]


def run_ranks_local(c, cfg, n, pods=None, enabled=None):
    """n ranks as threads of this process on the box's GPU, over the in-process device transport
    (gs_comm_init_local): the level all-gathers run stream-ordered, as ncclAllGather does, instead of through a host
    callback; returns every rank's placements (or its exception)."""
    from koordinator_amd.engine import Engine, LocalGroup
    g = LocalGroup(n)
    engines = [Engine(cfg) for _ in range(n)]
    for r, x in enumerate(engines):
        synth.load_into(x, c)
        x.comm_init_local(g, r)
    pods = c.pods if pods is None else pods
    res = [None] * n

    def run(r):
        try:
            res[r] = engines[r].schedule(pods)
        except Exception as ex:   # noqa: BLE001 (reported per rank)
            res[r] = ex
    th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    return res, engines, g


@pytest.mark.parametrize("n,numa,xchg", [(2, False, "scores"), (4, True, "scores"), (2, True, "levels"), (4, True, "levels")],
                         ids=["2ranks", "4ranks-numa", "2ranks-numa-levels", "4ranks-numa-levels"])
def test_ranks_on_one_gpu_device_transport(n, numa, xchg, monkeypatch):
    """The sharded path over the stream-ordered device transport (RCCL's ordering: tags written on the stream, the
    blocks copied device-to-device behind the senders' events, the next batch's kernels behind every rank's copies,
    batches in flight across exchanges): every rank's placements equal the oracle's. Both exchanges: the score rows of
    every shard (the default; every rank then runs the one-shard pipeline over all nodes) and the candidate levels
    (GS_XCHG=levels: merged level lists, the multi-shard commit)."""
    monkeypatch.setenv("GS_XCHG", xchg)
    c = synth.make_cluster(3001, 400, 13)
    en = abi.GS_ENABLE_ALL if numa else abi.GS_ENABLE_LA_FIT
    if numa:
        synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, enabled=en)
    res, engines, _ = run_ranks_local(c, cfg, n)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods)
    for r in range(n):
        assert not isinstance(res[r], Exception) and res[r] is not None, (r, res[r])
        for f in ("node", "score", "ties", "feasible"):
            assert np.array_equal(res[r][f], want[f]), (r, f)
    for r in range(n - 1):
        assert engines[r].stats()["shard_end"] == engines[r + 1].stats()["shard_begin"]


@pytest.mark.parametrize("xchg", ["scores", "levels"])
def test_ranks_with_an_empty_shard(xchg, monkeypatch):
    """5 nodes over 4 ranks: shards of 2, 2, 1 and 0 nodes (the last rank evaluates nothing and all-gathers an empty
    block). Every rank's placements equal the oracle's, contention included."""
    monkeypatch.setenv("GS_XCHG", xchg)
    c = synth.make_cluster(5, 90, 31)
    synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL)
    res, engines, _ = run_ranks_local(c, cfg, 4)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods)
    for r in range(4):
        assert not isinstance(res[r], Exception) and res[r] is not None, (r, res[r])
        for f in ("node", "score", "ties", "feasible"):
            assert np.array_equal(res[r][f], want[f]), (r, f)
    assert engines[3].stats()["shard_begin"] == engines[3].stats()["shard_end"] == 5
    assert (want["node"] >= 0).sum() > 5


@pytest.mark.parametrize("n,xchg", [(2, "scores"), (3, "scores"), (2, "levels")])
def test_ranks_submit_across_runs(n, xchg, monkeypatch):
    """gs_schedule_submit on several ranks: each rank submits the same runs at its own pace (rank-dependent sleeps,
    so at a run boundary one rank may hold the next run while another does not). The ranks agree at every run-ending
    batch whether to speculate into the next run (XSITE_RUNS), so their exchanges pair up and the placements of every
    rank equal the oracle's over the whole stream."""
    import time
    from koordinator_amd.engine import Engine, LocalGroup
    monkeypatch.setenv("GS_XCHG", xchg)
    c = synth.make_cluster(3001, 700, 13)
    synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL)
    cuts = [0, 150, 240, 300, 470, 600, 700]
    seq = np.arange(700, dtype=np.uint64)
    g = LocalGroup(n)
    engines = [Engine(cfg) for _ in range(n)]
    for r, x in enumerate(engines):
        synth.load_into(x, c)
        x.comm_init_local(g, r)
    rng = np.random.default_rng(5)
    delays = rng.uniform(0, 0.004, size=(n, len(cuts) - 1))
    res = [None] * n

    def run(r):
        try:
            hs = []
            for k in range(len(cuts) - 1):
                time.sleep(delays[r, k])
                hs.append(engines[r].schedule_submit(c.pods[cuts[k]:cuts[k + 1]], seq[cuts[k]:cuts[k + 1]]))
            res[r] = np.concatenate([engines[r].schedule_wait(h) for h in hs])
        except Exception as ex:   # noqa: BLE001 (reported per rank)
            res[r] = ex
    th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods)
    for r in range(n):
        assert not isinstance(res[r], Exception) and res[r] is not None, (r, res[r])
        for f in ("node", "score", "ties", "feasible"):
            assert np.array_equal(res[r][f], want[f]), (r, f)


@pytest.mark.parametrize("xchg", ["scores", "levels"])
def test_device_transport_divergence_fails_on_every_rank(xchg, monkeypatch):
    """A rank whose exchange sequence diverges over the device transport: every rank fails with GS_ECOMM naming the
    batch (the tags travel with the blocks and unpack_scores_kernel / merge_levels_kernel checks them on each rank's
    stream)."""
    c = synth.make_cluster(3001, 300, 13)
    cfg = config.make_config(c.num_nodes)
    monkeypatch.setenv("GS_XCHG", xchg)
    monkeypatch.setenv("GS_DEBUG_XCHG_SKEW", "1:1")
    res, _, _ = run_ranks_local(c, cfg, 2)
    for r in range(2):
        assert isinstance(res[r], Exception), (r, res[r])
        msg = str(res[r])
        assert "exchange sequence diverged" in msg and "batch 1" in msg, (r, msg)


def test_reset_rebuilds_mirror():
    """gs_reset (device-error recovery) rebuilds the HBM mirror from the host state: scheduling continues
    bit-exact with the oracle."""
    c = synth.make_cluster(1500, 256, 1)
    synth.make_numa(c)
    e, o = pair(c, enabled=abi.GS_ENABLE_ALL)
    seq = np.arange(256, dtype=np.uint64)
    got1, want1 = e.schedule(c.pods[:128], seq[:128]), o.schedule(c.pods[:128], seq[:128])
    e.reset()
    assert e.mirror_check() == 0
    got2, want2 = e.schedule(c.pods[128:], seq[128:]), o.schedule(c.pods[128:], seq[128:])
    for f in ("node", "score", "ties", "feasible"):
        assert np.array_equal(np.concatenate([got1[f], got2[f]]), np.concatenate([want1[f], want2[f]])), f
