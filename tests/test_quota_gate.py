"""Quota-gated batched scheduling (koordinator_amd.quota.schedule_with_quota): speculative admission + batch
cuts before rejections give the same PreFilter verdicts and placements as the reference's one-pod-at-a-time
order. CPU: the oracle stands in for the engine (the gate logic is what is tested here); the GPU test in
test_gpu_quota_gate.py runs libgpuscore's gs_schedule under the same gate."""
import numpy as np

from koordinator_amd.quota import schedule_with_quota
from oracle import oracle as orc
from koordinator_amd import synth
from tests import quota_util as qu


import pytest


@pytest.mark.parametrize("seed,check_parent", [(3, True), (4, False), (9, True)])
def test_gate_matches_sequential_order(seed, check_parent):
    c, cfg = qu.setup(800, 240, seed)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    o1, o2 = orc.Oracle(cfg), orc.Oracle(cfg)
    synth.load_into(o1, c)
    synth.load_into(o2, c)
    p1, p2 = qu.plugin(check_parent=check_parent), qu.plugin(check_parent=check_parent)
    pq1, pq2 = qu.pod_quotas(c, p1), qu.pod_quotas(c, p2)
    got, st = schedule_with_quota(o1, p1, c.pods, pq1, seq)
    want_nodes, want_codes = qu.sequential(o2, p2, c.pods, pq2, seq)
    assert [(s.code, s.message) for s in st] == want_codes   # verdicts and the reference's status text
    assert np.array_equal(got["node"], want_nodes)
    rejected = sum(s.code != "Success" for s in st)
    unplaced = int(((got["node"] < 0) & np.array([s.code == "Success" for s in st])).sum())
    assert rejected > 0 and unplaced > 0            # both the cut and the unreserve repair ran
    for name in ("team-a", "team-a-1", "team-a-2", "team-b"):
        assert p1.get(name, "used") == p2.get(name, "used")


@pytest.mark.parametrize("seed,check_parent", [(3, True), (4, False)])
def test_gate_matches_quota_oracle(seed, check_parent):
    """Against the independent Python restatement of the quota gate (oracle/quota.py)."""
    c, cfg = qu.setup(800, 240, seed)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    o1, o2 = orc.Oracle(cfg), orc.Oracle(cfg)
    synth.load_into(o1, c)
    synth.load_into(o2, c)
    p1 = qu.plugin(check_parent=check_parent)
    pq = qu.pod_quotas(c, p1)
    got, st = schedule_with_quota(o1, p1, c.pods, pq, seq)
    want_nodes, want_codes = qu.sequential_oracle(o2, c.pods, pq, seq, check_parent)
    assert [s.code for s in st] == want_codes
    assert np.array_equal(got["node"], want_nodes)
