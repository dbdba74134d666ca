"""Full-size parity (BASELINE.json north star): the HIP path schedules the 100k-node x 50k-pod synthetic C3
cluster (NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource, Reserve incl. NUMA splits and cpusets) and
its decisions are checked against the CPU oracle by replay: the oracle places every pod on the node the GPU
chose (Filter on that node for the affinity, Reserve, assume — a GPU placement the oracle's Filter rejects
fails the run) and re-runs the full scheduleOne over all 100k nodes for a sample of pods on the replayed state;
node, max score, tie count and feasible count must be identical. About 32 FitError pods are re-checked in full
(the others are replayed as FitErrors: a wrong one would shift the state every later sampled pod sees)."""
import os
import time

import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


def _save(name: str, got, extra: dict):
    """The GPU placements for the offline every-pod check (scripts/full_parity.py; committed under
    tests/golden/fullsize/)."""
    import json
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(os.path.join("gpurun_out", f"placements_{name}.npz"),
                        placements=np.ascontiguousarray(got).view(np.uint8), meta=json.dumps(extra))


GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize")


def _golden_equal(name: str, got):
    """Every decision of the run equals the committed placements, which were checked pod by pod against the oracle's
    sequential scheduleOne (all 50,000 north-star pods and all 20,480 bench pods, 0 mismatches:
    profiles/r04_full_parity_{northstar,bench}.json, scripts/full_parity.py). Every field of every placement record
    (node, max score, ties, feasible count, flags, NUMA zone split, cpuset) must match, so any later change that moves
    a single decision fails here, on the driver's box, not only in an offline check."""
    want = np.load(os.path.join(GOLDEN, f"placements_{name}.npz"))["placements"].view(abi.PLACEMENT_DTYPE)
    assert len(want) == len(got), f"{name}: {len(got)} placements, golden holds {len(want)}"
    for f in abi.PLACEMENT_DTYPE.names:
        bad = np.nonzero(np.any((got[f] != want[f]).reshape(len(got), -1), axis=1))[0]
        assert len(bad) == 0, f"{name}: {f} differs from the verified placements at pods {bad[:5]} ({len(bad)} pods)"
    return len(got)


def _replay_check(c, cfg, got, sample):
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    given = got["node"].astype(np.int32).copy()
    fit_err = np.nonzero(got["node"] < 0)[0]
    given[fit_err] = -2                   # replayed FitError (nothing assumed) ...
    given[fit_err[:: max(1, len(fit_err) // 32)]] = -1   # ... and ~32 of them re-checked in full
    given[sample] = -1
    want = o.schedule_replay(c.pods, given, nthreads=THREADS)
    chk = given == -1
    for f in ("node", "score", "ties", "feasible"):
        bad = np.nonzero(got[f][chk] != want[f][chk])[0]
        assert len(bad) == 0, f"{f} differs at pod {np.nonzero(chk)[0][bad[:5]]}"
    _replay_check.oracle = o
    return int(chk.sum())


def _allocations_equal(e, o, c, got):
    """Every placed pod's NodeNUMAResource allocation — NUMA zone split and cpuset, which the GPU chose and the engine
    recorded — equals the one the oracle's Reserve made on the same node during the replay (resourceManager.Allocate
    -> takeCPUs, nodenumaresource/plugin.go:375-419): the placement records' zone and cpuset fields pinned pod by pod
    against the oracle, not only through the golden files."""
    n = 0
    for j in np.nonzero(got["node"] >= 0)[0]:
        node, uid = int(got["node"][j]), int(c.pods["uid"][j])
        a, b = e.allocation(node, uid), o.allocation(node, uid)
        assert (a is None) == (b is None), f"pod {j}: allocation on one side only ({a is None}, {b is None})"
        if a is not None:
            assert a.tobytes() == b.tobytes(), f"pod {j} on node {node}: GPU allocation {a} oracle {b}"
            n += 1
    return n


def test_c3_100k_nodes_50k_pods_replay_parity():
    from koordinator_amd.engine import Engine
    t0 = time.perf_counter()
    c = synth.make_cluster(100_000, 50_000, 3)
    synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL)
    e = Engine(cfg)
    synth.load_into(e, c)
    got = e.schedule(c.pods)
    assert e.mirror_check() == 0
    _save("northstar", got, {"stats": {k: (float(v) if isinstance(v, float) else int(v)) for k, v in e.stats().items()}})
    ng = _golden_equal("northstar", got)
    P = len(c.pods)
    sample = np.unique(np.concatenate([np.arange(48), np.arange(48, P, 64)]))   # every 64th pod
    n = _replay_check(c, cfg, got, sample)
    na = _allocations_equal(e, _replay_check.oracle, c, got)
    placed = int((got["node"] >= 0).sum())
    print(f"100k x 50k: {placed} placed, all {ng} placements equal the oracle-verified golden ones, {n} pods "
          f"re-scheduled by the oracle and identical, {na} NUMA / cpuset allocations equal the oracle's; "
          f"wall {time.perf_counter() - t0:.1f} s; stats {e.stats()}")


def test_c3_bench_config_50k_nodes_replay_parity():
    """Exactly the bench's workload (bench.py defaults: C3 cluster of config id 2, 50,000 nodes, 2048-pod calls,
    batch 128): 10 calls (20,480 pods), every 64th pod re-scheduled by the oracle over all 50k nodes."""
    from koordinator_amd.engine import Engine
    t0 = time.perf_counter()
    P, step = 20_480, 2048
    c = synth.make_cluster(50_000, P, config_id=2)
    synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, batch_size=128, enabled=abi.GS_ENABLE_ALL)
    e = Engine(cfg)
    synth.load_into(e, c)
    seq = np.arange(P, dtype=np.uint64)
    got = np.concatenate([e.schedule(c.pods[k:k + step], seq[k:k + step]) for k in range(0, P, step)])
    assert e.mirror_check() == 0
    _save("bench", got, {"stats": {k: (float(v) if isinstance(v, float) else int(v)) for k, v in e.stats().items()}})
    ng = _golden_equal("bench", got)
    n = _replay_check(c, cfg, got, np.arange(0, P, 64))
    na = _allocations_equal(e, _replay_check.oracle, c, got)
    assert na > 1000
    print(f"C3 bench config 50k x {P}: {int((got['node'] >= 0).sum())} placed, all {ng} placements equal the "
          f"oracle-verified golden ones, {n} pods re-checked in full, {na} NUMA / cpuset allocations equal the "
          f"oracle's; "
          f"wall {time.perf_counter() - t0:.1f} s")


def test_c2_5k_nodes_10k_pods_full_parity():
    """C2: 5,000 nodes x 10,000 pods, NodeResourcesFit + LoadAwareScheduling; every pod's node, max
    score, tie count and feasible count compared with the oracle's full sequential scheduleOne."""
    from koordinator_amd.engine import Engine
    t0 = time.perf_counter()
    c = synth.make_cluster(5_000, 10_000, config_id=1)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_LA_FIT)
    e = Engine(cfg)
    synth.load_into(e, c)
    got = e.schedule(c.pods)
    assert e.mirror_check() == 0
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods, nthreads=THREADS)
    for f in ("node", "score", "ties", "feasible"):
        bad = np.nonzero(got[f] != want[f])[0]
        assert len(bad) == 0, f"{f} differs at pods {bad[:5]}"
    print(f"C2 5k x 10k: {int((got['node'] >= 0).sum())} placed, all 10,000 decisions identical; "
          f"wall {time.perf_counter() - t0:.1f} s")


@pytest.mark.parametrize("n,xchg", [(2, "scores"), (4, "scores"), (2, "levels")])
def test_c3_bench_config_ranks_equal_golden(n, xchg, monkeypatch):
    """The bench workload sharded over n ranks (threads of this process on the box's GPU, the stream-ordered device
    transport that has RCCL's ordering), submitted one 2048-pod call ahead as bench.py does at every N: every rank's
    20,480 placements — every field, NUMA zone split and cpuset included — equal the oracle-verified golden ones of
    the one-GPU run, for the score-row exchange (the default) and the level exchange."""
    import threading
    from koordinator_amd.engine import Engine, LocalGroup
    monkeypatch.setenv("GS_XCHG", xchg)
    P, step = 20_480, 2048
    c = synth.make_cluster(50_000, P, config_id=2)
    synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, batch_size=128, enabled=abi.GS_ENABLE_ALL)
    g = LocalGroup(n)
    engines = [Engine(cfg) for _ in range(n)]
    for r, e in enumerate(engines):
        synth.load_into(e, c)
        e.comm_init_local(g, r)
    seq = np.arange(P, dtype=np.uint64)
    res = [None] * n

    def run(r):
        try:
            e = engines[r]
            hs = [e.schedule_submit(c.pods[k:k + step], seq[k:k + step]) for k in range(0, P, step)]
            res[r] = np.concatenate([e.schedule_wait(h) for h in hs])
        except Exception as ex:   # noqa: BLE001 (reported per rank)
            res[r] = ex
    th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=200)
    for r in range(n):
        assert not isinstance(res[r], Exception) and res[r] is not None, (r, res[r])
        _golden_equal("bench", res[r])
        assert engines[r].mirror_check() == 0
