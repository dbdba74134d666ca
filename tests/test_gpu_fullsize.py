"""Full-size parity (BASELINE.json north star): the HIP path schedules the 100k-node x 50k-pod synthetic C3
cluster (NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource, Reserve incl. NUMA splits and cpusets) and
its decisions are checked against the CPU oracle by replay: the oracle places every pod on the node the GPU
chose (Filter on that node for the affinity, Reserve, assume — a GPU placement the oracle's Filter rejects
fails the run) and re-runs the full scheduleOne over all 100k nodes for a sample of pods on the replayed state;
node, max score, tie count and feasible count must be identical. About 32 FitError pods are re-checked in full
(the others are replayed as FitErrors: a wrong one would shift the state every later sampled pod sees)."""
import os

import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


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
    return int(chk.sum())


def test_c3_100k_nodes_50k_pods_replay_parity():
    from koordinator_amd.engine import Engine
    c = synth.make_cluster(100_000, 50_000, 3)
    synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL)
    e = Engine(cfg)
    synth.load_into(e, c)
    got = e.schedule(c.pods)
    assert e.mirror_check() == 0
    P = len(c.pods)
    sample = np.unique(np.concatenate([np.arange(48), np.linspace(48, P - 1, 48).astype(np.int64)]))
    n = _replay_check(c, cfg, got, sample)
    placed = int((got["node"] >= 0).sum())
    print(f"100k x 50k: {placed} placed, {n} pods re-scheduled by the oracle and identical; stats {e.stats()}")
