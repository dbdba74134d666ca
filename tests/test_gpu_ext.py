"""Reservation + DeviceShare on the HIP path (gs_schedule_ext) against the oracle (or_schedule_ext), bit-exact:
placement, max score, tie count, feasible count, the reservation each pod was assumed into, the GPU minors and
per-instance resources DeviceShare's Reserve allocated, both normalized plugin scores, and the final reservation and
device state. Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def run_pair(c, strategy=None, enabled=abi.GS_ENABLE_LA_FIT, chunks=1, ignored=0):
    from koordinator_amd.engine import Engine
    cfg = config.make_config(c.num_nodes, enabled=enabled)
    a = orc.ext_args_default()
    if strategy == "MostAllocated":
        a.device_scoring_type = abi.GS_SCORING_MOST_ALLOCATED
    a.fit_ignored_gpu_names = ignored
    e, o = Engine(cfg), orc.Oracle(cfg)
    for x in (e, o):
        synth.load_into(x, c)
        synth.load_ext_into(x, c, a)
    P = len(c.pods)
    seq = np.arange(P, dtype=np.uint64)
    outs = []
    for k in range(chunks):
        sl = slice(k * P // chunks, (k + 1) * P // chunks)
        outs.append(e.schedule_ext(c.pods[sl], c.ext["pod_ext"][sl], seq[sl]))
    ge = np.concatenate([x[0] for x in outs]), np.concatenate([x[1] for x in outs])
    oe = o.schedule_ext(c.pods, c.ext["pod_ext"], seq)
    return e, o, ge, oe


def check(c, e, o, ge, oe):
    (gp, gx), (op, ox) = ge, oe
    for f in ("node", "feasible"):
        bad = np.nonzero(gp[f] != op[f])[0]
        assert not len(bad), f"{f} differs at pods {bad[:10]}: gpu {gp[bad[:5]]} oracle {op[bad[:5]]}"
    placed = op["node"] >= 0
    assert np.array_equal(gp["score"][placed], op["score"][placed])
    assert np.array_equal(gp["ties"][placed], op["ties"][placed])
    for f in ("reservation_uid", "gpu_minor_mask", "gpu_count", "gpu_per_instance", "deviceshare_score",
              "reservation_score", "fail_code"):
        bad = np.nonzero((gx[f] != ox[f]).reshape(len(gx), -1).any(axis=1))[0]
        assert not len(bad), f"ext {f} differs at pods {bad[:10]}"
    for r in c.ext["reservations"]:
        a, b = e.reservation(int(r["uid"])), o.reservation(int(r["uid"]))
        if a is None or b is None:   # removed by an update between calls: removed on both sides
            assert a is None and b is None
            continue
        assert a["assigned_pods"] == b["assigned_pods"] and np.array_equal(a["allocated"], b["allocated"])
    for i in np.nonzero(c.ext["devices"]["has_device"])[0]:
        a, b = e.devices(int(i)), o.devices(int(i))
        assert np.array_equal(a["gpus"]["used"], b["gpus"]["used"]) and np.array_equal(a["requested"], b["requested"])
    assert e.mirror_check() == 0
    return placed


def test_c5_small_matches_oracle():
    c = synth.make_cluster(3000, 900, config_id=5)
    synth.make_ext(c)
    e, o, ge, oe = run_pair(c, chunks=3)
    placed = check(c, e, o, ge, oe)
    gx = ge[1]
    assert placed.sum() > 800 and (gx["gpu_count"] > 0).sum() > 40 and (gx["reservation_uid"] > 0).sum() > 5


def test_c5_dense_reservations_required_restricted():
    c = synth.make_cluster(2000, 700, config_id=6)
    synth.make_ext(c, rsv_node_pct=40, owners=10, owner_pod_pct=50, required_pct=10, gpu_pod_pct=5)
    e, o, ge, oe = run_pair(c)
    check(c, e, o, ge, oe)
    assert (ge[1]["reservation_uid"] > 0).sum() > 50
    assert (ge[1]["reservation_score"] > 0).any()


def test_c5_gpu_heavy_most_allocated():
    c = synth.make_cluster(1500, 600, config_id=7)
    synth.make_ext(c, gpu_node_pct=50, gpu_pod_pct=60, owner_pod_pct=5)
    e, o, ge, oe = run_pair(c, strategy="MostAllocated")
    check(c, e, o, ge, oe)
    assert (ge[1]["gpu_count"] > 1).any() and (ge[0]["node"] < 0).any()


def test_c5_with_numa_profile_without_policy_nodes():
    c = synth.make_cluster(1200, 400, config_id=8)
    synth.make_numa(c, numa_policy_pct=0, cpuset_pod_pct=0)
    synth.make_ext(c)
    e, o, ge, oe = run_pair(c, enabled=abi.GS_ENABLE_ALL)
    check(c, e, o, ge, oe)


def test_c5_fit_ignored_resource_group():
    """NodeResourcesFitArgs.IgnoredResourceGroups = ["koordinator.sh"]: Fit skips the koordinator.sh/* GPU names
    (DeviceShare still filters on the devices); nvidia.com/gpu stays checked."""
    c = synth.make_cluster(1500, 500, config_id=10)
    synth.make_ext(c, gpu_node_pct=30, gpu_pod_pct=40)
    # NodeInfo scalars that would fail Fit for every koordinator.sh request
    c.ext["devices"]["allocatable"][:, 1:] = 0
    ign = sum(1 << abi.GPU_NAMES[n] for n in ("koordinator.sh/gpu", "koordinator.sh/gpu-core",
                                              "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio"))
    e, o, ge, oe = run_pair(c, ignored=ign)
    check(c, e, o, ge, oe)
    assert (ge[1]["gpu_count"] > 0).sum() > 20


@pytest.mark.parametrize("ignored", [0, 0x1], ids=["checked", "x0-ignored"])
def test_c5_registered_extended_resources(ignored):
    """Extended resources outside the fixed slots and the GPU names (gs_pod_ext.xres_*): Fit's scalar check on the
    extension path, IgnoredResources per name, NodeInfo.AddPod of them on the host mirror."""
    c = synth.make_cluster(1500, 500, config_id=12)
    synth.make_ext(c, xres_node_pct=40, xres_pod_pct=20)
    from koordinator_amd.engine import Engine
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_LA_FIT)
    a = orc.ext_args_default()
    a.fit_ignored_xres = ignored
    e, o = Engine(cfg), orc.Oracle(cfg)
    for x in (e, o):
        synth.load_into(x, c)
        synth.load_ext_into(x, c, a)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    ge = e.schedule_ext(c.pods, c.ext["pod_ext"], seq)
    oe = o.schedule_ext(c.pods, c.ext["pod_ext"], seq)
    check(c, e, o, ge, oe)
    for i in np.nonzero(c.ext["devices"]["xres_allocatable"][:, 0])[0][:50]:
        assert np.array_equal(e.devices(int(i))["xres_requested"], o.devices(int(i))["xres_requested"])
    assert (c.ext["pod_ext"]["xres_request_mask"] != 0).sum() > 50


@pytest.mark.parametrize("policy_pct", [40, 100], ids=["policy40", "policy100"])
def test_c5_numa_policy_nodes_deviceshare_hints(policy_pct):
    """GPU pods on nodes with a NUMA topology policy: DeviceShare is the topology manager's second hint provider
    (deviceshare/topology_hint.go:33-214), merged with NodeNUMAResource's hints; the Filter-time affinity restricts
    DeviceShare's Allocate / Score / Reserve to the GPUs on its NUMA nodes, and NodeNUMAResource's Reserve allocates
    the zones along it. Placements, GPU minors, NUMA allocations and the final state bit-exact against the oracle."""
    # (260 / 400 pods: the oracle's permutation merge over every provider list is most of the test's time)
    c = synth.make_cluster(1500, 260 if policy_pct == 100 else 400, config_id=13 + policy_pct)
    synth.make_numa(c, numa_policy_pct=policy_pct, cpuset_pod_pct=0)
    synth.make_ext(c, gpu_node_pct=50, gpu_pod_pct=50, owner_pod_pct=0)
    e, o, ge, oe = run_pair(c, enabled=abi.GS_ENABLE_ALL)
    placed = check(c, e, o, ge, oe)
    assert np.array_equal(ge[0]["flags"][placed] & 6, oe[0]["flags"][placed] & 6)
    pol = c.numa["node_numa"]["numa_topology_policy"] != 0
    node = ge[0]["node"]
    on_pol = placed & pol[np.maximum(node, 0)]
    gpu_on_pol = on_pol & (ge[1]["gpu_count"] > 0)
    assert gpu_on_pol.sum() > 20 and ((ge[0]["flags"] & 2) != 0)[gpu_on_pol].sum() > 10
    for j in np.nonzero(on_pol)[0]:
        uid = int(c.pods["uid"][j])
        a, b = e.allocation(int(node[j]), uid), o.allocation(int(node[j]), uid)
        assert (a is None) == (b is None) and (a is None or a.tobytes() == b.tobytes()), j


@pytest.mark.parametrize("policy_pct", [0, 60], ids=["no-policy", "policy60"])
def test_c5_gpu_owner_pods_reservations_on_policy_nodes_cpuset_pods(policy_pct):
    """The §8(f) rank-2 combinations that round 4 refused (GS_EUNSUPPORTED), against the oracle, bit-exact:
    * GPU pods that match reservations: the Fit restore applies, DeviceShare's view is not restored (the reservations
      hold no devices: deviceshare/reservation.go:133-162), and DeviceShare's FilterReservation rejects every
      device-less reservation for a device pod (deviceshare/plugin.go:324-350), so a GPU pod nominates none;
    * reservations matched on NUMA-policy nodes: the restored NodeInfo through NodeNUMAResource's Filter (its
      reservation restore is empty without reserved cpusets, nodenumaresource/reservation.go:76-113), the affinity of
      the restored row, DeviceShare as the second hint provider there;
    * cpuset-bound extension pods (NUMA split on the device, takeCPUs by the host's Reserve)."""
    c = synth.make_cluster(2000, 380, config_id=21 + policy_pct)
    synth.make_numa(c, numa_policy_pct=policy_pct, cpuset_pod_pct=25)
    synth.make_ext(c, gpu_node_pct=40, gpu_pod_pct=20, rsv_node_pct=30, owners=8, owner_pod_pct=40, required_pct=10,
                   owner_gpu_pct=40)
    e, o, ge, oe = run_pair(c, enabled=abi.GS_ENABLE_ALL)
    placed = check(c, e, o, ge, oe)
    ext, gx = c.ext["pod_ext"], ge[1]
    gpu_owner = (ext["reservation_owner"] != 0) & (ext["gpu_request_mask"] != 0)
    assert (gpu_owner & placed).sum() > 20 and (gx["gpu_count"][gpu_owner] > 0).sum() > 10
    assert (gx["reservation_uid"][gpu_owner] == 0).all()   # no nomination for a device pod
    assert (gx["reservation_uid"] > 0).sum() > 20
    node = ge[0]["node"]
    flags = ge[0]["flags"]
    assert ((flags & abi.GS_PLACED_CPUSET) != 0)[placed].sum() > 20
    if policy_pct:
        pol = c.numa["node_numa"]["numa_topology_policy"] != 0
        rs_on_pol = placed & (gx["reservation_uid"] > 0) & pol[np.maximum(node, 0)]
        assert rs_on_pol.sum() > 5
    for j in np.nonzero(placed)[0]:
        uid = int(c.pods["uid"][j])
        a, b = e.allocation(int(node[j]), uid), o.allocation(int(node[j]), uid)
        assert (a is None) == (b is None) and (a is None or a.tobytes() == b.tobytes()), j


@pytest.mark.parametrize("n,numa", [(2, False), (3, True)], ids=["2ranks", "3ranks-numa"])
def test_c5_on_several_ranks_score_rows(n, numa):
    """Reservation + DeviceShare pods on several ranks (threads over the in-process device transport, the default
    score-row exchange): the plain runs between extension pods go through the sharded batch pipeline with its
    all-gathers, each extension pod runs whole on every rank. Every rank's placements, reservations, GPU minors and
    normalized scores equal the oracle's, and the ranks' device and reservation state equal it too."""
    import threading
    from koordinator_amd.engine import Engine, LocalGroup
    c = synth.make_cluster(2500, 600, config_id=33 + n)
    if numa:
        synth.make_numa(c, numa_policy_pct=40, cpuset_pod_pct=10)
    synth.make_ext(c, gpu_node_pct=30, gpu_pod_pct=15)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL if numa else abi.GS_ENABLE_LA_FIT)
    a = orc.ext_args_default()
    g = LocalGroup(n)
    engines = [Engine(cfg) for _ in range(n)]
    for r, x in enumerate(engines):
        synth.load_into(x, c)
        synth.load_ext_into(x, c, a)
        x.comm_init_local(g, r)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    res = [None] * n

    def run(r):
        try:
            outs = [engines[r].schedule_ext(c.pods[k:k + 200], c.ext["pod_ext"][k:k + 200], seq[k:k + 200])
                    for k in range(0, len(c.pods), 200)]
            res[r] = (np.concatenate([x[0] for x in outs]), np.concatenate([x[1] for x in outs]))
        except Exception as ex:   # noqa: BLE001 (reported per rank)
            res[r] = ex
    th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    synth.load_ext_into(o, c, a)
    oe = o.schedule_ext(c.pods, c.ext["pod_ext"], seq)
    for r in range(n):
        assert not isinstance(res[r], Exception) and res[r] is not None, (r, res[r])
        check(c, engines[r], o, res[r], oe)
    assert (res[0][1]["gpu_count"] > 0).sum() > 20 and (res[0][1]["reservation_uid"] > 0).sum() > 5


def test_c5_on_several_ranks_level_exchange_refused(monkeypatch):
    """Under the level exchange (GS_XCHG=levels) a rank holds only its shard's rows, so an extension pod is refused
    loudly (GS_EUNSUPPORTED) on every rank instead of being scored on part of the cluster."""
    import threading
    from koordinator_amd.engine import Engine, LocalGroup
    monkeypatch.setenv("GS_XCHG", "levels")
    c = synth.make_cluster(1000, 200, config_id=37)
    synth.make_ext(c, gpu_node_pct=30, gpu_pod_pct=20)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_LA_FIT)
    a = orc.ext_args_default()
    g = LocalGroup(2)
    engines = [Engine(cfg) for _ in range(2)]
    for r, x in enumerate(engines):
        synth.load_into(x, c)
        synth.load_ext_into(x, c, a)
        x.comm_init_local(g, r)
    res = [None] * 2

    def run(r):
        try:
            res[r] = engines[r].schedule_ext(c.pods, c.ext["pod_ext"], np.arange(len(c.pods), dtype=np.uint64))
        except Exception as ex:   # noqa: BLE001 (reported per rank)
            res[r] = ex
    th = [threading.Thread(target=run, args=(r,)) for r in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    for r in range(2):
        assert isinstance(res[r], Exception) and "score-row exchange" in str(res[r]), (r, res[r])
