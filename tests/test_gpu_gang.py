"""Coscheduling gangs over the HIP engine: koordinator_amd/gang.py's batched driver (speculative runs of gs_schedule,
gs_pods_forget of rejected / rolled-back pods) against the reference's one-pod-at-a-time order on the oracle engine:
gang PreFilter codes, Permit statuses, final pod states, and node / score / ties / feasible of every pod that reached
the node loop, bit-exact; the HBM mirror equals a fresh host derivation afterwards. Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from koordinator_amd import abi, synth
from koordinator_amd.engine import Engine
from oracle import coscheduling as oc
from tests.test_gang import check_pair, gang_workload, run_pair

pytestmark = pytest.mark.gpu


def _engine(cfg):
    cfg.device = 0
    return Engine(cfg)


@pytest.mark.parametrize("seed", [3, 5])
def test_gangs_hip_engine_small(seed):
    c, pgs, gang_ids = gang_workload(seed=seed)
    e, o, got, gres, want, wres = run_pair(_engine, c, pgs, gang_ids)
    check_pair(got, gres, want, wres)
    assert (wres["state"] == oc.ST_REJECTED).sum() > 3
    assert e.mirror_check() == 0


def test_gangs_hip_engine_numa_1k_nodes():
    c, pgs, gang_ids = gang_workload(n_nodes=1000, n_pods=900, seed=9)
    c.pods["requests"][:, 0] *= 2
    synth.make_numa(c)
    e, o, got, gres, want, wres = run_pair(_engine, c, pgs, gang_ids, enabled=abi.GS_ENABLE_ALL)
    check_pair(got, gres, want, wres)
    assert (wres["state"] == oc.ST_BOUND).sum() > 200
    assert e.mirror_check() == 0


@pytest.mark.parametrize("chunk", [37, 128])
def test_gangs_hip_engine_chunked_calls(chunk):
    """Gangs spanning several schedule_with_gangs calls (waiting pods carried between the calls) on the HIP engine
    = the one long queue on the oracle."""
    c, pgs, gang_ids = gang_workload(seed=11)
    e, o, got, gres, want, wres = run_pair(_engine, c, pgs, gang_ids, chunk=chunk)
    check_pair(got, gres, want, wres)
    assert e.mirror_check() == 0
