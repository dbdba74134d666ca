"""Quota-gated batched scheduling on the HIP path: schedule_with_quota over libgpuscore's gs_schedule gives the
reference's one-pod-at-a-time PreFilter verdicts and placements (oracle, sequential). Needs an MI355X."""
import numpy as np
import pytest

from koordinator_amd import synth
from koordinator_amd.quota import schedule_with_quota
from oracle import oracle as orc
from tests import quota_util as qu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch", [16, 128])
def test_gpu_gate_matches_sequential_oracle(batch):
    from koordinator_amd import config
    from koordinator_amd.engine import Engine
    c, _ = qu.setup(2000, 400, 5)
    cfg = config.make_config(c.num_nodes, batch_size=batch)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    e, o = Engine(cfg), orc.Oracle(cfg)
    synth.load_into(e, c)
    synth.load_into(o, c)
    p1, p2 = qu.plugin(), qu.plugin()
    pq1, pq2 = qu.pod_quotas(c, p1), qu.pod_quotas(c, p2)
    got, st = schedule_with_quota(e, p1, c.pods, pq1, seq)
    want_nodes, want_codes = qu.sequential(o, p2, c.pods, pq2, seq)
    assert [(s.code, s.message) for s in st] == want_codes
    bad = np.nonzero(got["node"] != want_nodes)[0]
    assert len(bad) == 0, f"placement differs first at pod {bad[0]}"
    assert e.mirror_check() == 0
    assert any(s.code != "Success" for s in st)
