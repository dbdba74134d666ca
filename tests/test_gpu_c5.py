"""Config C5 as SURVEY 8(d) specifies it: DeviceShare GPUs + Reservations + ElasticQuota in ONE run, with incremental
snapshot updates between scheduling calls. The HIP path (quota gate schedule_with_quota over gs_schedule_ext) against
the oracle's one-pod-at-a-time order (ElasticQuota PreFilter, or_schedule_ext, quota Reserve), bit-exact: quota
verdicts and status text, node, max score, ties, feasible count, the reservation and GPU minors each pod was assumed
into, both normalized plugin scores, and the final reservation / device / mirror state. Between the chunks: node
resizes and pod-count changes (gs_nodes_upsert), fresh NodeMetrics (gs_node_metrics_upsert), a reservation
removed and one turned unavailable (gs_reservations_upsert / _remove), GPU device usage changed (gs_node_devices_upsert).
The full mix runs at 3k nodes and at C5's 100k. Plus C5 at 100k nodes: every pod of a 1,500-pod run compared with the
oracle's sequential scheduleOne.
Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from koordinator_amd.quota import schedule_with_quota
from oracle import oracle as orc
from tests import quota_util as qu
from tests.test_gpu_ext import check

pytestmark = pytest.mark.gpu


def _sequential_ext(o, p, pods, ext, pq, seq):
    """The reference's order, one pod at a time: quota PreFilter, node loop (with Reservation / DeviceShare), Reserve."""
    out = np.zeros(len(pods), abi.PLACEMENT_DTYPE)
    out["node"] = -1
    xout = np.zeros(len(pods), abi.EXT_PLACEMENT_DTYPE)
    codes = []
    for i in range(len(pods)):
        q, req, np_ = pq[i]
        st = p.pre_filter(q, req, np_)
        codes.append((st.code, st.message))
        if st.is_success():
            r, x = o.schedule_ext(pods[i:i + 1], ext[i:i + 1], seq[i:i + 1])
            out[i], xout[i] = r[0], x[0]
            if r["node"][0] >= 0:
                p.reserve_pod(q, req, np_)
    return out, xout, codes


def _updates(c, k, rng):
    """Informer deltas between chunk k and k + 1 (the same calls go to the engine and the oracle)."""
    N = c.num_nodes
    idx = np.sort(rng.choice(N, N // 50, replace=False)).astype(np.uint32)
    nodes = c.nodes[idx].copy()
    nodes["allocatable"][:, 0] += 4000 * (1 + k)
    nodes["pod_count"] = np.maximum(nodes["pod_count"] - 1, 0)
    midx = np.sort(rng.choice(N, N // 20, replace=False)).astype(np.uint32)
    m = c.metrics[midx].copy()
    m["node_usage"]["cpu_milli"] = (m["node_usage"]["cpu_milli"] * 0.8).astype(np.int64)
    m["update_time_ns"] = c.now_ns - 10 * synth.SEC
    rsv = c.ext["reservations"]
    removed = rsv["uid"][k:k + 1].copy()
    unavail = rsv[len(rsv) // 2 + k:len(rsv) // 2 + k + 1].copy()
    unavail["available"] = 0
    dv = np.nonzero(c.ext["devices"]["has_device"])[0][k::37].astype(np.uint32)
    devs = c.ext["devices"][dv].copy()
    devs["gpus"]["used"][:, 0, :] = 0   # the first GPU of those nodes released
    return lambda x: (x.upsert_nodes(nodes, idx=idx), x.upsert_metrics(m, idx=midx), x.remove_reservations(removed),
                      x.upsert_reservations(unavail), x.upsert_devices(devs, idx=dv))


@pytest.mark.parametrize("n_nodes,n_pods,cfg_id", [(3000, 900, 11), (100_000, 600, 12)], ids=["3k", "100k"])
def test_c5_quota_ext_with_incremental_updates(n_nodes, n_pods, cfg_id):
    """(100k: C5's node count, the full mix — quota, reservations, GPUs, updates between calls — every pod compared)"""
    from koordinator_amd.engine import Engine
    c = synth.make_cluster(n_nodes, n_pods, config_id=cfg_id)
    synth.make_ext(c, gpu_pod_pct=15, owner_pod_pct=15)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_LA_FIT)
    a = orc.ext_args_default()
    e, o = Engine(cfg), orc.Oracle(cfg)
    for x in (e, o):
        synth.load_into(x, c)
        synth.load_ext_into(x, c, a)
    p1, p2 = qu.plugin(), qu.plugin()
    pq1, pq2 = qu.pod_quotas(c, p1), qu.pod_quotas(c, p2)
    P = len(c.pods)
    seq = np.arange(P, dtype=np.uint64)
    ext = c.ext["pod_ext"]
    rng = np.random.default_rng(11)
    gp, gx, gs_, op, ox, os_ = [], [], [], [], [], []
    for k in range(3):
        sl = slice(k * P // 3, (k + 1) * P // 3)
        r, x, st = schedule_with_quota(e, p1, c.pods[sl], pq1[sl], seq[sl], pod_ext=ext[sl])
        gp.append(r), gx.append(x), gs_.extend((s.code, s.message) for s in st)
        r2, x2, st2 = _sequential_ext(o, p2, c.pods[sl], ext[sl], pq2[sl], seq[sl])
        op.append(r2), ox.append(x2), os_.extend(st2)
        if k < 2:
            upd = _updates(c, k, rng)
            upd(e)
            upd(o)
    assert gs_ == os_, "quota verdicts / status text differ"
    assert any(code != "Success" for code, _ in gs_)
    placed = check(c, e, o, (np.concatenate(gp), np.concatenate(gx)), (np.concatenate(op), np.concatenate(ox)))
    gx_all = np.concatenate(gx)
    assert placed.sum() > 0.44 * P and (gx_all["gpu_count"] > 0).sum() > 0.022 * P
    assert (gx_all["reservation_uid"] > 0).sum() > 0.0055 * P


def test_c5_100k_nodes_every_pod():
    from tests.test_gpu_ext import run_pair
    c = synth.make_cluster(100_000, 1500, config_id=5)
    synth.make_ext(c)
    e, o, ge, oe = run_pair(c, chunks=2)
    placed = check(c, e, o, ge, oe)
    assert placed.sum() > 1400 and (ge[1]["gpu_count"] > 0).sum() > 50
