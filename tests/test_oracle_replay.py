"""The oracle's replay mode (test infrastructure for the full-size GPU parity test): placing pods on the
nodes the oracle itself chose and re-scheduling sampled pods on the replayed state reproduces scheduleOne's
decisions exactly, with and without NodeNUMAResource (Reserve incl. NUMA splits and cpusets)."""
import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from oracle import oracle as orc


def _pair(c, numa):
    kw = {"enabled": abi.GS_ENABLE_ALL} if numa else {}
    cfg = config.make_config(c.num_nodes, **kw)
    a, b = orc.Oracle(cfg), orc.Oracle(cfg)
    synth.load_into(a, c)
    synth.load_into(b, c)
    return a, b


@pytest.mark.parametrize("numa", [False, True])
def test_replay_reproduces_schedule(numa):
    c = synth.make_cluster(600, 400, 21)
    if numa:
        synth.make_numa(c, numa_policy_pct=60, cpuset_pod_pct=40)
    a, b = _pair(c, numa)
    want = a.schedule(c.pods)
    given = want["node"].astype(np.int32).copy()
    sample = np.arange(7, len(given), 37)
    given[sample] = -1
    fe = np.nonzero(want["node"] < 0)[0]
    given[fe] = -2                        # FitError pods: replayed as such ...
    given[fe[::2]] = -1                   # ... or re-scheduled
    got = b.schedule_replay(c.pods, given)
    for f in ("node", "score", "ties", "feasible"):
        assert np.array_equal(got[f][given < 0], want[f][given < 0]), f
    assert np.array_equal(got["node"], want["node"])
    assert numa is False or len(fe) > 0
    assert np.array_equal(got["flags"][given < 0], want["flags"][given < 0])


def test_replay_rejects_infeasible_node():
    c = synth.make_cluster(50, 4, 22)
    a, _ = _pair(c, False)
    p = c.pods[:1].copy()
    p["requests"][0, 0] = 10 ** 9          # cannot fit anywhere
    with pytest.raises(Exception):
        a.schedule_replay(p, np.array([0], np.int32))


def test_hint_provider_order_sensitivity():
    """policy.go:108 merges the providers' hints in Go map order; the restatement fixes (cpu, memory).
    Reported, not asserted: how many decisions the reverse order changes on a NUMA-dense synthetic cluster."""
    c = synth.make_cluster(400, 300, 23)
    synth.make_numa(c, numa_policy_pct=90, cpuset_pod_pct=40)
    a, b = _pair(c, True)
    b.set_hint_order(True)
    x, y = a.schedule(c.pods), b.schedule(c.pods)
    diff = int((x["node"] != y["node"]).sum() + (x["score"] != y["score"]).sum())
    print(f"hint-order sensitivity: {diff} of {len(c.pods)} decisions differ under the reverse provider order")
    assert (x["node"] >= 0).sum() > 0
