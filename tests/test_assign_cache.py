"""podAssignCache informer handlers (loadaware/pod_assign_cache.go:53-117) against the reference's own vectors
(tests/golden/assign_cache.json from pod_assign_cache_test.go): the oracle on the CPU, the library's
gs_pods_on_event / gs_assign_cache_get on a one-node cluster on the GPU."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi, config, synth

CASES = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "assign_cache.json")))
EVENT = {"add": abi.GS_POD_EVENT_ADD, "update": abi.GS_POD_EVENT_UPDATE, "delete": abi.GS_POD_EVENT_DELETE}


def run(eng, case):
    c = synth.make_cluster(1, 1, config_id=9)
    c.assigned_pods = c.assigned_pods[:0]
    c.assigned_node = c.assigned_node[:0]
    c.assigned_ts = c.assigned_ts[:0]
    synth.load_into(eng, c)
    pre = np.zeros(len(case["cache"]), abi.POD_DTYPE)
    pre["uid"] = case["cache"]
    if len(pre):
        eng.assign(np.zeros(len(pre), np.uint32), pre, np.full(len(pre), c.now_ns, np.int64))
    pod = np.zeros(1, abi.POD_DTYPE)
    pod["uid"] = case["pod"]["uid"]
    pod["flags"] = abi.GS_POD_TERMINATED if case["pod"]["terminated"] else 0
    eng.pod_event(EVENT[case["event"]], [case["pod"]["node"]], pod)
    return eng.assign_cache(0), c.now_ns


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_oracle_assign_cache(case):
    from oracle import oracle as orc
    cfg = config.make_config(1, enabled=abi.GS_ENABLE_LA_FIT)
    got, now = run(orc.Oracle(cfg), case)
    assert got == [(u, now) for u in case["want"]], case["src"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_gpu_assign_cache(case):
    from koordinator_amd.engine import Engine
    cfg = config.make_config(1, enabled=abi.GS_ENABLE_LA_FIT)
    got, now = run(Engine(cfg), case)
    assert got == [(u, now) for u in case["want"]], case["src"]
