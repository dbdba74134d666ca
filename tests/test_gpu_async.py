"""gs_schedule_submit / gs_schedule_wait: submissions form one scheduling stream (the batch pipeline continues across
them), so the placements equal one gs_schedule over the concatenated queue and the oracle's sequential scheduleOne
(node, score, ties, feasible, NUMA flags), with chunk sizes that end mid-batch, empty submissions, several outstanding
submissions, and other calls in between (they wait for the submissions). Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from koordinator_amd.engine import Engine, GpuScoreError
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
FIELDS = ("node", "score", "ties", "feasible", "flags")


def _cluster(n=4000, p=1400):
    c = synth.make_cluster(n, p, 2)
    synth.make_numa(c)
    return c


def _engine(c):
    e = Engine(config.make_config(c.num_nodes, device=0, enabled=abi.GS_ENABLE_ALL))
    synth.load_into(e, c)
    return e


def test_submissions_equal_one_stream_and_oracle():
    c = _cluster()
    seq = np.arange(len(c.pods), dtype=np.uint64)
    cuts = [0, 300, 300, 437, 700, 1024, 1025, 1400]   # an empty chunk, chunks ending mid-batch
    e = _engine(c)
    hs = [e.schedule_submit(c.pods[a:b], seq[a:b]) for a, b in zip(cuts, cuts[1:])]
    got = np.concatenate([e.schedule_wait(h) for h in hs])
    ref = _engine(c).schedule(c.pods, seq)
    o = orc.Oracle(config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL))
    synth.load_into(o, c)
    want = o.schedule(c.pods, seq)
    for f in FIELDS:
        assert np.array_equal(got[f], ref[f]), f
        assert np.array_equal(got[f], want[f]), f
    assert e.mirror_check() == 0


def test_one_ahead_with_calls_between():
    c = _cluster(3000, 1024)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    e = _engine(c)
    P = 256
    h = e.schedule_submit(c.pods[:P], seq[:P])
    outs = []
    for s in range(1, 5):
        h2 = e.schedule_submit(c.pods[s * P:(s + 1) * P], seq[s * P:(s + 1) * P]) if s < 4 else None
        outs.append(e.schedule_wait(h))
        e.stats()   # waits for the outstanding submission
        h = h2
    got = np.concatenate(outs)
    want = _engine(c).schedule(c.pods, seq)
    for f in FIELDS:
        assert np.array_equal(got[f], want[f]), f


def test_invalid_submission_is_refused():
    c = _cluster(2000, 200)
    e = _engine(c)
    bad = c.pods[:10].copy()
    bad["requests"][3, 0] = -1
    with pytest.raises(GpuScoreError):
        e.schedule_submit(bad)
    out = e.schedule_wait(e.schedule_submit(c.pods[:100]))
    assert (out["node"] >= 0).sum() > 50


@pytest.mark.parametrize("pct", [0, 10])
def test_submissions_with_node_sampling(pct):
    """Node sampling under gs_schedule_submit: nextStartNodeIndex carries across submissions as across batches (the
    speculative pass reads it on the device from the batch before); placements and the final index equal the
    oracle's sequential scheduleOne."""
    c = synth.make_cluster(4000, 1100, 9)
    c.pods["requests"][::3, 0] = 60_000
    c.pods["request_mask"][:] |= 0x1
    cfg = config.make_config(c.num_nodes, device=0, percentage_of_nodes_to_score=pct)
    e = Engine(cfg)
    synth.load_into(e, c)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    cuts = [0, 200, 437, 700, 701, 1100]
    hs = [e.schedule_submit(c.pods[a:b], seq[a:b]) for a, b in zip(cuts, cuts[1:])]
    got = np.concatenate([e.schedule_wait(h) for h in hs])
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = o.schedule(c.pods, seq)
    for f in ("node", "score", "ties", "feasible"):
        assert np.array_equal(got[f], want[f]), f
    assert e.stats()["next_start_node_index"] == o.next_start_node_index
    assert want["feasible"].max() == orc.num_feasible_nodes_to_find(4000, pct)
