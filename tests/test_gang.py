"""Coscheduling. The library's gang manager (gs_gang_*) and the independent restatement
oracle/coscheduling.py against the reference's own vectors (core/core_test.go TestPlugin_PreFilter, TestPermit), both
against each other on random event sequences, and koordinator_amd/gang.py's batched driver against the reference's
one-pod-at-a-time order with the oracle engine as the engine (CPU; tests/test_gpu_gang.py runs it on the HIP engine)."""
import numpy as np
import pytest

from koordinator_amd import abi, config, gang as gg, synth
from oracle import coscheduling as oc
from oracle import oracle as orc

SEC = 10**9


class Ids:
    """stable 64-bit keys for GetId(namespace, name) strings"""

    def __init__(self):
        self.m = {}

    def __call__(self, s):
        return self.m.setdefault(s, len(self.m) + 1)


def both_managers(timeout=10 * SEC):
    return gg.GangManager(default_timeout_ns=timeout), oc.PodGroupManager(default_timeout_ns=timeout)


# ---- core_test.go TestPlugin_PreFilter (one manager shared by the cases, as the test does). Pods: (namespace, name,
# gang label or None); pgs: (name, namespace, minMember); the expected child-cycle map is asserted where the test does.
PREFILTER_CASES = [
    dict(name="pod does not belong to any gang", pod=("ns1", "pod1", None), err=""),
    dict(name="pod belongs to a non-existing pg", pod=("gangA_ns", "pod2", "wenshiqi222"),
         err="gang has not init, gangName: gangA_ns/wenshiqi222, podName: gangA_ns/pod2"),
    dict(name="gang ResourceSatisfied", pod=("gangq_ns", "podq", "gangq"), pg=("gangq", "gangq_ns", 4),
         resource_satisfied=True, err="", cycle=1, valid=True, child_map={}),
    dict(name="pod count less than minMember", pod=("ganga_ns", "pod3", "ganga"), pods=[("ganga_ns", "pod3-1", "ganga")],
         pg=("ganga", "ganga_ns", 4), err="gang child pod not collect enough, gangName: ganga_ns/ganga, podName: ganga_ns/pod3",
         cycle=1, valid=True, child_map={}),
    dict(name="pods count equal with minMember,but is NonStrictMode", pod=("gangb_ns", "pod5", "gangb"),
         pods=[("gangb_ns", f"pod5-{k}", "gangb") for k in (1, 2, 3)], pg=("gangb", "gangb_ns", 4), nonstrict=True, err=""),
    dict(name="due to reschedule pod6's podScheduleCycle is equal with the gangScheduleCycle",
         pod=("ganga_ns", "pod6", "gangc"), pods=[("ganga_ns", f"pod6-{k}", "gangc") for k in (1, 2, 3)],
         pg=("gangc", "ganga_ns", 4), cycle_equal=True, total=5, cycle=1, child_map={"ganga_ns/pod6": 1}, valid=True,
         err="pod's schedule cycle too large, gangName: ganga_ns/gangc, podName: ganga_ns/pod6, podCycle: 1, gangCycle: 1"),
    dict(name="... but pod6's nominatedNodeName is not empty", pod=("ganga_ns", "pod6", "gangc"), nominated=True,
         pods=[("ganga_ns", f"pod6-{k}", "gangc") for k in (1, 2, 3)], pg=("gangc", "ganga_ns", 4), cycle_equal=True,
         total=5, cycle=1, valid=True, err="",
         child_map={"ganga_ns/pod6": 1, "ganga_ns/pod6-1": 1, "ganga_ns/pod6-2": 1, "ganga_ns/pod6-3": 1}),
    dict(name="StrictMode, scheduleCycle not valid due to pre pod Filter Failed", pod=("ganga_ns", "pod7", "gangd"),
         pods=[("ganga_ns", f"pod7-{k}", "gangd") for k in (1, 2, 3)], pg=("gangd", "ganga_ns", 4), cycle=1,
         child_map={"ganga_ns/pod7": 1}, valid=False, set_invalid=True,
         err="gang scheduleCycle not valid, gangName: ganga_ns/gangd, podName: ganga_ns/pod7"),
    dict(name="StrictMode, disable check scheduleCycle", pod=("ganga_ns", "pod7", "gangd"),
         pods=[("ganga_ns", f"pod7-{k}", "gangd") for k in (1, 2, 3)], pg=("gangd", "ganga_ns", 4), set_invalid=True,
         skip=True, err=""),
    dict(name="StrictMode, scheduleCycle valid, childrenNum not reach total", pod=("ganga_ns", "pod8", "gange"),
         pods=[("ganga_ns", f"pod8-{k}", "gange") for k in (1, 2, 3)], pg=("gange", "ganga_ns", 4), total=5, cycle=1,
         child_map={"ganga_ns/pod8": 1}, valid=True, err=""),
    dict(name="pods count more than minMember, childrenNum reach total", pod=("ganga_ns", "pod9", "ganga"),
         pods=[("ganga_ns", f"pod9-{k}", "ganga") for k in (1, 2, 3, 4)], total=5, err=""),
]


def _gid(ids, ns, label):
    return ids(f"{ns}/{label}") if label else 0


@pytest.mark.parametrize("which", ["library", "oracle"])
def test_prefilter_reference_vectors(which):
    lm, om = both_managers()
    m = lm if which == "library" else om
    ids = Ids()
    for case in PREFILTER_CASES:
        pgid = None
        if "pg" in case:
            name, ns, mn = case["pg"]
            pgid = ids(f"{ns}/{name}")
            s = dict(gang_id=pgid, min_member=mn, total_children=case.get("total", -1),
                     mode=gg.NONSTRICT if case.get("nonstrict") else -1)
            m.podgroup_upsert(gg.spec(**s) if which == "library" else s)
        for ns, name, label in case.get("pods", []):
            g = _gid(ids, ns, label)
            m.pod_add(g, ids(f"{ns}/{name}"))
            m.prefilter(g, ids(f"{ns}/{name}"))
        ns, name, label = case["pod"]
        g, uid = _gid(ids, ns, label), ids(f"{ns}/{name}")
        if g:
            m.pod_add(g, uid)
        gang_obj = None if pgid is None else pgid
        if case.get("set_invalid"):
            m.debug_set(pgid, 0, 0, 0) if which == "library" else setattr(om.gangs[pgid], "cycle_valid", False)
        if case.get("cycle_equal"):
            m.debug_set(pgid, uid, 1, 1) if which == "library" else om.gangs[pgid].child_cycle.__setitem__(uid, 1)
        if case.get("resource_satisfied"):
            m.debug_set(pgid, 0, 2, 1) if which == "library" else setattr(om.gangs[pgid], "once", True)
        if case.get("skip"):
            m.debug_set(0, 0, 4, 1) if which == "library" else setattr(om, "skip", True)
        code = m.prefilter(g, uid, case.get("nominated", False))
        info = m.info(pgid) if (which == "library" and pgid) else None
        ogang = om.gangs.get(pgid) if (which == "oracle" and pgid) else None
        cyc = info["schedule_cycle"] if info else (ogang.cycle if ogang else 1)
        msg = "" if code == gg.PF_OK else gg.PREFILTER_MESSAGES[code].format(
            gang=f"{ns}/{label}", pod=f"{ns}/{name}", pcycle=1, gcycle=cyc)
        assert msg == case["err"], case["name"]
        if case.get("skip"):
            m.debug_set(0, 0, 4, 0) if which == "library" else setattr(om, "skip", False)
        if gang_obj is not None and not case.get("nonstrict") and not case.get("skip"):
            valid = info["schedule_cycle_valid"] if info else ogang.cycle_valid
            assert (cyc, bool(valid)) == (case["cycle"], case["valid"]), case["name"]
            for key, want in case["child_map"].items():
                got = m.child_cycle(pgid, ids(key)) if which == "library" else ogang.child_cycle.get(ids(key), -1)
                assert got == want, (case["name"], key)
            n_entries = (sum(1 for k in ids.m if m.child_cycle(pgid, ids(k)) >= 0) if which == "library"
                         else len(ogang.child_cycle))
            assert n_entries == len(case["child_map"]), case["name"]


# ---- core_test.go TestPermit (a fresh manager per case; default timeout 10 s). pgs: (name, ns, min)
PERMIT_CASES = [
    dict(name="pod1 does not belong to any pg, allow", pod=("ns1", "pod1", None), want=gg.PERMIT_SUCCESS, wait=0),
    dict(name="pod2 belongs to a non-existing pg", pod=("ns1", "pod2", "gangnonexist"), want=gg.PERMIT_WAIT, wait=0),
    dict(name="pod3 belongs to gangA that doesn't have enough assumed pods", pod=("gangA_ns", "pod3", "gangA"),
         pods=[("gangA_ns", "pod3-1", "gangA")], pgs=[("gangA", "gangA_ns", 3)], want=gg.PERMIT_WAIT, wait=10 * SEC),
    dict(name="... but once satisfied", pod=("gangA_ns", "pod3", "gangA"), pods=[("gangA_ns", "pod3-1", "gangA")],
         pgs=[("gangA", "gangA_ns", 3)], once=True, policy="", want=gg.PERMIT_SUCCESS, wait=0),
    dict(name="... once satisfied, but matchPolicy not once satisfied", pod=("gangA_ns", "pod3", "gangA"),
         pods=[("gangA_ns", "pod3-1", "gangA")], pgs=[("gangA", "gangA_ns", 3)], once=True, policy=gg.ONLY_WAITING,
         want=gg.PERMIT_WAIT, wait=10 * SEC),
    dict(name="... with Running pods is enough, matchPolicy only-waiting", pod=("gangA_ns", "pod3", "gangA"),
         pods=[("gangA_ns", "pod3-1", "gangA")], running=[("gangA_ns", "pod3-2", "gangA")], pgs=[("gangA", "gangA_ns", 3)],
         once=True, policy=gg.ONLY_WAITING, want=gg.PERMIT_WAIT, wait=10 * SEC),
    dict(name="... with Running pods is enough, matchPolicy waiting-and-running", pod=("gangA_ns", "pod3", "gangA"),
         pods=[("gangA_ns", "pod3-1", "gangA")], running=[("gangA_ns", "pod3-2", "gangA")], pgs=[("gangA", "gangA_ns", 3)],
         once=True, policy=gg.WAITING_AND_RUNNING, want=gg.PERMIT_SUCCESS, wait=0),
    dict(name="pod4 belongs to gangB that gangA has resourceSatisfied", pod=("gangA_ns", "pod4", "gangB"),
         pods=[("gangA_ns", "pod4-1", "gangB"), ("gangA_ns", "pod4-2", "gangB")], pgs=[("gangB", "gangA_ns", 3)],
         policy="", want=gg.PERMIT_SUCCESS, wait=0),
    dict(name="pod5: gangC satisfied, gangD not", pod=("gangC_ns", "pod5", "gangC"),
         pods=[("gangC_ns", "pod5-1", "gangC"), ("gangD_ns", "pod5-2", "gangD")],
         pgs=[("gangC", "gangC_ns", 2), ("gangD", "gangD_ns", 2)], group=["gangC_ns/gangC", "gangD_ns/gangD"],
         policy="", want=gg.PERMIT_WAIT, wait=10 * SEC),
    dict(name="pod6: gangE and gangF satisfied", pod=("gangE_ns", "pod6", "gangE"),
         pods=[("gangE_ns", "pod6-1", "gangE")] + [("gangF_ns", f"pod6-{k}", "gangF") for k in (2, 3, 4)],
         pgs=[("gangE", "gangE_ns", 2), ("gangF", "gangF_ns", 3)], group=["gangE_ns/gangE", "gangF_ns/gangF"],
         policy="", want=gg.PERMIT_SUCCESS, wait=0),
]


@pytest.mark.parametrize("which", ["library", "oracle"])
@pytest.mark.parametrize("case", PERMIT_CASES, ids=[c["name"][:50] for c in PERMIT_CASES])
def test_permit_reference_vectors(which, case):
    lm, om = both_managers()
    m = lm if which == "library" else om
    ids = Ids()
    group = [ids(x) for x in case.get("group", [])]
    for name, ns, mn in case.get("pgs", []):
        gid = ids(f"{ns}/{name}")
        s = dict(gang_id=gid, min_member=mn, group=group)
        m.podgroup_upsert(gg.spec(**s) if which == "library" else s)
        # the test sets OnceResourceSatisfied and GangMatchPolicy (its zero value "" outside the three policies: 3)
        pol = case.get("policy", "")
        pol = 3 if pol == "" else pol
        if which == "library":
            m.debug_set(gid, 0, 2, int(case.get("once", False)))
            m.debug_set(gid, 0, 3, pol)
        else:
            om.gangs[gid].once, om.gangs[gid].policy = case.get("once", False), pol
    for ns, name, label in case.get("pods", []):
        g, uid = _gid(ids, ns, label), ids(f"{ns}/{name}")
        m.pod_add(g, uid)
        m.permit(g, uid, 0)
    for ns, name, label in case.get("running", []):
        g, uid = _gid(ids, ns, label), ids(f"{ns}/{name}")
        m.pod_add(g, uid)
        m.post_bind(g, uid)
    ns, name, label = case["pod"]
    g, uid = _gid(ids, ns, label), ids(f"{ns}/{name}")
    if g:
        m.pod_add(g, uid)
    st, wait, _ = m.permit(g, uid, 0)
    assert (st, wait) == (case["want"], case["wait"])


def _random_ops(rng, n_gangs, n_pods, n_ops):
    ops = []
    for _ in range(n_ops):
        r = rng.random()
        g = int(rng.integers(1, n_gangs + 1))
        u = int(rng.integers(1, n_pods + 1)) + 1000 * g
        if r < 0.06:
            ops.append(("podgroup_upsert", dict(gang_id=g, min_member=int(rng.integers(0, 5)),
                                                total_children=int(rng.integers(-1, 7)), mode=int(rng.integers(-1, 2)),
                                                match_policy=int(rng.integers(-1, 3)),
                                                wait_time_ns=int(rng.integers(-1, 3)) * SEC,
                                                group=[g] + ([g % n_gangs + 1] if rng.random() < 0.3 else []))))
        elif r < 0.25:
            annot = None
            if rng.random() < 0.3:
                annot = dict(gang_id=g, min_member=int(rng.integers(-1, 4)), total_children=int(rng.integers(-1, 5)),
                             mode=int(rng.integers(-1, 2)), match_policy=int(rng.integers(-1, 3)),
                             wait_time_ns=int(rng.integers(-1, 3)) * SEC, group=[])
            ops.append(("pod_add", g, u, bool(rng.random() < 0.1), annot))
        elif r < 0.30:
            ops.append(("pod_delete", g, u))
        elif r < 0.50:
            ops.append(("prefilter", g, u, bool(rng.random() < 0.1)))
        elif r < 0.70:
            ops.append(("permit", g, u, int(rng.integers(0, 5)) * SEC))
        elif r < 0.78:
            ops.append(("post_bind", g, u))
        elif r < 0.86:
            ops.append(("post_filter", g, u))
        elif r < 0.95:
            ops.append(("unreserve", g, u))
        elif r < 0.98:
            ops.append(("expire", int(rng.integers(0, 8)) * SEC))
        else:
            ops.append(("podgroup_delete", g))
    return ops


@pytest.mark.parametrize("seed", range(12))
def test_library_matches_restatement_on_random_events(seed):
    rng = np.random.default_rng(seed)
    lm, om = both_managers(timeout=3 * SEC)
    for op in _random_ops(rng, 5, 8, 600):
        kind = op[0]
        if kind == "podgroup_upsert":
            lm.podgroup_upsert(gg.spec(**op[1]))
            om.podgroup_upsert(op[1])
            continue
        if kind == "pod_add":
            _, g, u, assigned, annot = op
            lm.pod_add(g, u, assigned, gg.spec(**annot) if annot else None)
            om.pod_add(g, u, assigned, annot)
            continue
        a = getattr(lm, kind)(*op[1:])
        b = getattr(om, kind)(*op[1:])
        if kind == "permit":
            assert a == b, op
        else:
            assert a == b, op
    for g in range(1, 6):
        li = lm.info(g)
        og = om.gangs.get(g)
        assert (li is None) == (og is None)
        if og is not None:
            assert (li["has_init"], li["min_member"], li["total_children"], li["schedule_cycle"],
                    li["schedule_cycle_valid"], li["once_resource_satisfied"], li["children"], li["waiting"],
                    li["bound"]) == (og.has_init, og.min, og.total, og.cycle, og.cycle_valid, og.once, len(og.children),
                                     len(og.waiting), len(og.bound))
    assert lm.waiting_pods() == sorted(om.fw_waiting)


def gang_workload(n_nodes=200, n_pods=500, seed=3, gang_pct=70, tight=True):
    """A small cluster and a queue in which gangs (PodGroups, Strict and NonStrict, groups of two gangs, some gangs with
    fewer pods than minMember) interleave with plain pods; `tight` makes some pods find no node."""
    c = synth.make_cluster(n_nodes, n_pods, 2)
    rng = np.random.default_rng(seed)
    if tight:
        c.pods["requests"][:, 0] *= 6
        c.pods["requests"][:, 1] *= 3
    n_g = n_pods // 6
    pgs, gang_ids = [], np.zeros(n_pods, np.uint64)
    for g in range(1, n_g + 1):
        mode = gg.STRICT if rng.random() < 0.7 else gg.NONSTRICT
        group = [g, g + 1] if (g % 7 == 0 and g < n_g) else []
        pgs.append(dict(gang_id=g, min_member=int(rng.integers(2, 6)), total_children=int(rng.integers(-1, 8)),
                        mode=mode, match_policy=int(rng.integers(-1, 3)), wait_time_ns=60 * SEC, group=group))
    k = 0
    while k < n_pods:
        if rng.random() * 100 < gang_pct:
            g = int(rng.integers(1, n_g + 1))
            m = int(rng.integers(1, 7))
            gang_ids[k:k + m] = g
            k += m
        else:
            k += 1
    return c, pgs, gang_ids[:n_pods]


def load_gangs(mgr, pgs, pods, gang_ids, library: bool):
    for s in pgs:
        mgr.podgroup_upsert(gg.spec(**s) if library else s)
    for k in range(len(pods)):
        if gang_ids[k]:
            mgr.pod_add(int(gang_ids[k]), int(pods["uid"][k]))


def chunked_gangs(e, lm, pods, gang_ids, seq, now_ns, chunk):
    """schedule_with_gangs over consecutive chunks of the queue with one WaitingPods carried between the calls; the
    per-pod results are joined and the later calls' verdicts on earlier waiting pods applied."""
    waiting = gg.WaitingPods()
    outs, res = [], {f: [] for f in ("prefilter", "permit", "state", "node")}
    for lo in range(0, len(pods), chunk):
        o, r = gg.schedule_with_gangs(e, lm, pods[lo:lo + chunk], gang_ids[lo:lo + chunk], seq[lo:lo + chunk],
                                      now_ns=now_ns, waiting=waiting)
        outs.append(o)
        for f in res:
            res[f].append(r[f])
        res.setdefault("carried", []).append(r["carried"])
    gres = {f: np.concatenate(res[f]) for f in ("prefilter", "permit", "state", "node")}
    idx = {int(u): k for k, u in enumerate(pods["uid"])}
    for car in res["carried"]:
        for uid, st in car.items():
            gres["state"][idx[uid]] = st
    return np.concatenate(outs), gres


def run_pair(make_engine, c, pgs, gang_ids, enabled=abi.GS_ENABLE_LA_FIT, chunk=None):
    cfg = config.make_config(c.num_nodes, enabled=enabled)
    e = make_engine(cfg)
    synth.load_into(e, c)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    lm, om = gg.GangManager(), oc.PodGroupManager()
    load_gangs(lm, pgs, c.pods, gang_ids, True)
    load_gangs(om, pgs, c.pods, gang_ids, False)
    seq = np.arange(len(c.pods), dtype=np.uint64)
    if chunk:
        got, gres = chunked_gangs(e, lm, c.pods, gang_ids, seq, c.now_ns, chunk)
    else:
        got, gres = gg.schedule_with_gangs(e, lm, c.pods, gang_ids, seq, now_ns=c.now_ns)
    want, wres = oc.schedule_sequential(o, om, c.pods, gang_ids, seq, now_ns=c.now_ns)
    return e, o, got, gres, want, wres


def check_pair(got, gres, want, wres):
    for f in ("prefilter", "permit", "state", "node"):
        bad = np.nonzero(np.asarray(gres[f]) != np.asarray(wres[f]))[0]
        assert not len(bad), f"{f} differs at pods {bad[:10]}"
    ran = want["node"] >= 0
    for f in ("node", "score", "ties", "feasible"):
        assert np.array_equal(got[f][ran], want[f][ran]), f


@pytest.mark.parametrize("chunk", [37, 128])
def test_chunked_gangs_carry_waiting_pods_oracle_engine(chunk):
    """A gang spanning several schedule_with_gangs calls: the waiting pods of earlier calls are allowed, rejected and
    forgotten by later calls exactly as in the one long queue (WaitingPods carried between the calls)."""
    c, pgs, gang_ids = gang_workload(seed=11)
    e, o, got, gres, want, wres = run_pair(lambda cfg: orc.Oracle(cfg), c, pgs, gang_ids, chunk=chunk)
    check_pair(got, gres, want, wres)


def test_batched_gangs_match_sequential_order_oracle_engine():
    c, pgs, gang_ids = gang_workload()
    e, o, got, gres, want, wres = run_pair(lambda cfg: orc.Oracle(cfg), c, pgs, gang_ids)
    check_pair(got, gres, want, wres)
    st = wres["state"]
    # the workload exercises every outcome
    assert (st == oc.ST_BOUND).sum() > 20 and (st == oc.ST_WAITING).sum() > 5 and (st == oc.ST_REJECTED).sum() > 3
    assert (wres["prefilter"] != 0).sum() > 5 and ((want["node"] < 0) & (wres["prefilter"] == 0)).sum() > 3


def _big_gang(m, library, gid, n, group=()):
    s = dict(gang_id=gid, min_member=n, mode=gg.STRICT, wait_time_ns=5 * SEC, group=list(group))
    m.podgroup_upsert(gg.spec(**s) if library else s)
    uids = [gid * 10000 + k for k in range(n)]
    for u in uids:
        m.pod_add(gid, u)
    return uids


@pytest.mark.parametrize("which", ["library", "oracle"])
def test_large_strict_gang_lists_exceed_first_buffer(which):
    """A Strict gang of 100 members: Permit's allowed list, PostFilter's and Unreserve's rejection lists and the
    Permit-timeout list all exceed the driver's first 64-entry buffer. Every pod must come back exactly once and the
    manager state must equal the restatement's (a call that returned GS_EINVAL with the state already changed lost
    the pods of the retry)."""
    lm, om = both_managers()
    m = lm if which == "library" else om
    waiting = (lambda: m.waiting_pods()) if which == "library" else (lambda: sorted(om.fw_waiting))
    # Permit success: the 100th pod allows the 99 waiting ones
    uids = _big_gang(m, which == "library", 1, 100)
    for u in uids[:-1]:
        assert m.permit(1, u, 0)[0] == gg.PERMIT_WAIT
    st, _, allowed = m.permit(1, uids[-1], 0)
    assert st == gg.PERMIT_SUCCESS and sorted(allowed) == sorted(uids[:-1])
    assert waiting() == []
    # PostFilter: a FitError rejects the 99 waiting pods of another Strict gang
    uids = _big_gang(m, which == "library", 2, 100)
    for u in uids[:-1]:
        m.prefilter(2, u)
        m.permit(2, u, 0)
    rej = m.post_filter(2, uids[-1])
    assert sorted(rej) == sorted(uids[:-1]) and waiting() == []
    # Unreserve of one waiting pod rejects the other 98
    uids = _big_gang(m, which == "library", 3, 100)
    for u in uids[:-1]:
        m.permit(3, u, 0)
    rej = m.unreserve(3, uids[0])
    assert sorted(rej) == sorted(uids[1:-1]) and waiting() == []
    # Permit timeout: 99 waiting pods expire together
    uids = _big_gang(m, which == "library", 4, 100)
    for u in uids[:-1]:
        m.permit(4, u, 0)
    assert m.expire(10 * SEC) == sorted(uids[:-1]) and waiting() == []


def test_large_gang_library_matches_restatement_state():
    lm, om = both_managers()
    for which, m in (("library", lm), ("oracle", om)):
        uids = _big_gang(m, which == "library", 7, 90, group=[7, 8])
        uids8 = _big_gang(m, which == "library", 8, 40, group=[7, 8])
        for u in uids[:-1] + uids8:
            m.permit(7 if u in uids else 8, u, 0)
    a, b = lm.permit(7, 70089, 0), om.permit(7, 70089, 0)
    assert a[0] == b[0] == gg.PERMIT_SUCCESS and sorted(a[2]) == sorted(b[2]) and len(a[2]) == 129
    for g in (7, 8):
        li, og = lm.info(g), om.gangs[g]
        assert (li["waiting"], li["bound"]) == (len(og.waiting), len(og.bound))
