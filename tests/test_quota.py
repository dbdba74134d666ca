"""ElasticQuota admission (include/gpuscore.h gs_quota_*): runtime water filling, request
tree and PreFilter through the C-ABI, against the reference's own test vectors (tests/golden/quota.json, from
runtime_quota_calculator_test.go and plugin_test.go) and against the Python restatement in oracle/quota.py on
seeded random quota forests. Host functions of libgpuscore: no GPU needed."""
import ctypes as C
import json
import os
import random

import numpy as np
import pytest

from koordinator_amd import abi
from koordinator_amd.quota import ROOT, ElasticQuotaPlugin, print_resource_list
from oracle import quota as oq

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "quota.json")))
RES = ("cpu", "memory", "nvidia.com/gpu")


@pytest.fixture(scope="module")
def lib():
    return abi.load()


def _redistribute(lib, nodes, total):
    n = len(nodes)
    w, req, mn, gu, lent = (np.array([x[i] for x in nodes], np.int64) for i in range(5))
    lent = lent.astype(np.uint8)
    out = np.zeros(n, np.int64)
    assert lib.gs_quota_redistribute(abi.ptr(req), abi.ptr(mn), abi.ptr(gu), abi.ptr(w), abi.ptr(lent), n,
                                     total, abi.ptr(out)) == 0
    return out.tolist()


@pytest.mark.parametrize("case", G["redistribution"], ids=lambda c: c["name"])
def test_golden_redistribution(lib, case):
    assert _redistribute(lib, case["nodes"], case["total"]) == case["runtime"]
    nodes = {i: {"shared_weight": w, "request": r, "min": m, "guarantee": g, "allow_lent": l}
             for i, (w, r, m, g, l) in enumerate(case["nodes"])}
    oq.redistribution(nodes, case["total"])
    assert [nodes[i]["runtime"] for i in range(len(nodes))] == case["runtime"]


@pytest.mark.parametrize("case", G["runtime"], ids=lambda c: c["name"])
def test_golden_runtime(lib, case):
    p = ElasticQuotaPlugin(resources=RES, lib=lib)
    p.update_cluster_total_resource(case["total"])
    tree = oq.QuotaTree(case["total"])
    for q in case["quotas"]:
        p.on_quota_add(q["name"], max=q["max"], min=q["min"], shared_weight=q["shared_weight"])
        p.on_pod_add(q["name"], q["request"], assigned=False)
        oqq = tree.add(oq.Quota(q["name"], max=q["max"], min=q["min"], shared_weight=q["shared_weight"]))
        oqq.pod_request = dict(q["request"])
    got = p.refresh_runtime()
    tree.refresh()
    for name, want in case["runtime"].items():
        assert got[name] == want, name
        assert tree.quotas[name].runtime == want, name


DEFAULT = "koordinator-default-quota"


@pytest.mark.parametrize("case", G["prefilter_runtime"], ids=lambda c: c["name"])
def test_golden_prefilter(lib, case):
    p = ElasticQuotaPlugin(resources=RES, enable_runtime_quota=case["runtime_quota"], lib=lib)
    p.on_quota_add(DEFAULT, max=case["max"] or {"cpu": 1 << 50, "memory": 1 << 50})
    p.set_runtime(DEFAULT, case["runtime"])
    st = p.pre_filter(DEFAULT, case["request"])
    assert st.code == case["code"]
    assert st.exceed == case["exceed"]
    if st.code != "Success":
        assert st.message.startswith(f"Insufficient quotas, quotaName: {DEFAULT}, runtime: "
                                     f"{print_resource_list(case['runtime'])}, used: <empty>")
    tree = oq.QuotaTree({})
    q = tree.add(oq.Quota(DEFAULT, max=case["max"] or {"cpu": 1 << 50, "memory": 1 << 50}))
    q.runtime = dict(case["runtime"])
    code, _, bad, _ = oq.pre_filter(tree, DEFAULT, case["request"], runtime_quota=case["runtime_quota"])
    assert (code == "Success") == (case["code"] == "Success") and bad == case["exceed"]


@pytest.mark.parametrize("case", G["prefilter_check_parent"], ids=lambda c: c["name"])
def test_golden_check_parent(lib, case):
    p = ElasticQuotaPlugin(resources=RES, enable_check_parent_quota=True, lib=lib)
    par, ch = case["parent"], case["child"]
    p.on_quota_add(par["name"], max=par["max"], min=par["min"])
    p.on_quota_add(ch["name"], parent=par["name"], max=ch["max"], min=ch["min"])
    p.set_runtime(par["name"], par["runtime"])
    p.set_runtime(ch["name"], ch["runtime"])
    st = p.pre_filter(ch["name"], case["request"])
    assert st.code == case["code"] and st.quota == case["failed"] and st.exceed == case["exceed"]
    assert f"quotaNameTopo: [{' '.join(case['topo'])}]" in st.message
    tree = oq.QuotaTree({})
    tree.add(oq.Quota(par["name"], max=par["max"], min=par["min"])).runtime = dict(par["runtime"])
    tree.add(oq.Quota(ch["name"], parent=par["name"], max=ch["max"], min=ch["min"])).runtime = dict(ch["runtime"])
    code, failed, bad, topo = oq.pre_filter(tree, ch["name"], case["request"], check_parent=True)
    assert (failed, bad, topo) == (case["failed"], case["exceed"], case["topo"])


@pytest.mark.parametrize("case", G["prefilter_non_preemptible"], ids=lambda c: c["name"])
def test_golden_non_preemptible(lib, case):
    p = ElasticQuotaPlugin(resources=RES, lib=lib)
    p.update_cluster_total_resource(case["total"])
    q = case["quota"]
    p.on_quota_add(q["name"], max=q["max"], min=q["min"])
    tree = oq.QuotaTree(case["total"])
    tree.add(oq.Quota(q["name"], max=q["max"], min=q["min"]))
    for cpu, mem, np_ in case["init_pods"]:
        r = {"cpu": cpu * 1000, "memory": mem}
        p.on_pod_add(q["name"], r, assigned=True, non_preemptible=np_)
        tree.add_pod(q["name"], r, assigned=True, non_preemptible=np_)
    cpu, mem, np_ = case["pod"]
    req = {"cpu": cpu * 1000, "memory": mem}
    p.on_pod_add(q["name"], req, assigned=False, non_preemptible=np_)
    tree.add_pod(q["name"], req, assigned=False)
    rt = p.refresh_runtime()
    tree.refresh()
    if "runtime" in case:
        assert rt[q["name"]] == case["runtime"] == tree.quotas[q["name"]].runtime
    st = p.pre_filter(q["name"], req, non_preemptible=np_)
    assert st.code == case["code"] and st.exceed == case["exceed"]
    if "message" in case:
        assert st.message == case["message"]
    code, _, bad, _ = oq.pre_filter(tree, q["name"], req, non_preemptible=np_)
    assert bad == case["exceed"] and code == case.get("reason", "Success")


def test_no_quota_label_admits(lib):
    p = ElasticQuotaPlugin(resources=RES, lib=lib)
    assert p.pre_filter(None, {"cpu": 10**9}).is_success()
    st = abi.GsQuotaStatus()
    req = np.zeros(abi.GS_QUOTA_DIMS, np.int64)
    assert lib.gs_quota_prefilter(None, 0, None, None, -1, abi.ptr(req), 0, 1, C.byref(st)) == 0 and st.code == 0


def test_bad_forest_rejected(lib):
    arr = (abi.GsQuotaGroup * 2)()
    arr[0].parent, arr[1].parent = 1, 0   # a cycle
    total = np.zeros(abi.GS_QUOTA_DIMS, np.int64)
    assert lib.gs_quota_refresh_runtime(arr, 2, abi.ptr(total), None, None, None) < 0
    arr[1].parent = 5   # out of range
    assert lib.gs_quota_refresh_runtime(arr, 2, abi.ptr(total), None, None, None) < 0


def _random_forest(rng: random.Random, n: int):
    names = [f"q{i}" for i in range(n)]
    parents, specs = {}, {}
    for i, name in enumerate(names):
        parents[name] = ROOT if i == 0 or rng.random() < 0.35 else names[rng.randrange(i)]
        mx = {r: rng.randrange(0, 200_000) for r in RES if rng.random() < 0.9}
        mn = {r: rng.randrange(0, max(1, mx.get(r, 50_000))) for r in RES if rng.random() < 0.8}
        sw = None if rng.random() < 0.5 else {r: rng.randrange(0, 10) for r in RES}
        g = {r: rng.randrange(0, 30_000) for r in RES} if rng.random() < 0.2 else None
        specs[name] = dict(max=mx, min=mn, shared_weight=sw, allow_lent=rng.random() < 0.7, guaranteed=g)
    return names, parents, specs


@pytest.mark.parametrize("seed", range(40))
def test_random_forest_matches_oracle(lib, seed):
    rng = random.Random(0x6b6f6f7264 + seed)
    n = rng.randrange(1, 24)
    names, parents, specs = _random_forest(rng, n)
    total = {r: rng.randrange(0, 1_000_000) for r in RES}
    p = ElasticQuotaPlugin(resources=RES, enable_check_parent_quota=bool(seed & 1), lib=lib)
    p.update_cluster_total_resource(total)
    tree = oq.QuotaTree(total)
    for name in names:
        p.on_quota_add(name, parent=parents[name], **specs[name])
        tree.add(oq.Quota(name, parent=parents[name], **specs[name]))
    for _ in range(rng.randrange(0, 80)):
        name = rng.choice(names)
        req = {r: rng.randrange(0, 40_000) for r in RES if rng.random() < 0.8}
        assigned, np_ = rng.random() < 0.6, rng.random() < 0.3
        p.on_pod_add(name, req, assigned, np_)
        tree.add_pod(name, req, assigned, np_)
    got = p.refresh_runtime()
    tree.refresh()
    for name in names:
        assert got[name] == tree.quotas[name].runtime, name
    for _ in range(30):
        name = rng.choice(names)
        req = {r: rng.randrange(0, 60_000) for r in RES if rng.random() < 0.8}
        np_ = rng.random() < 0.3
        st = p.pre_filter(name, req, non_preemptible=np_)
        code, failed, bad, topo = oq.pre_filter(tree, name, req, non_preemptible=np_,
                                                check_parent=bool(seed & 1))
        assert st.is_success() == (code == "Success")
        if not st.is_success():
            assert (st.quota, st.exceed) == (failed, bad)
            assert st.message.startswith(code)


def test_runtime_conservation(lib):
    """Size-independent property: siblings never share out more than the parent's runtime beyond their
    guaranteed / min floors, and no lending quota gets more than its limited request."""
    rng = random.Random(7)
    for _ in range(50):
        names, parents, specs = _random_forest(rng, 30)
        total = {r: rng.randrange(0, 2_000_000) for r in RES}
        p = ElasticQuotaPlugin(resources=RES, lib=lib)
        p.update_cluster_total_resource(total)
        for name in names:
            p.on_quota_add(name, parent=parents[name], **specs[name])
            p.on_pod_add(name, {r: rng.randrange(0, 100_000) for r in RES}, assigned=False)
        rt = p.refresh_runtime()
        n = len(names)
        arr = p._array()
        lim = np.zeros((n, abi.GS_QUOTA_DIMS), np.int64)
        t, _ = p._dense(total)
        assert lib.gs_quota_refresh_runtime(arr, n, abi.ptr(t), None, abi.ptr(lim), None) == 0
        for i, name in enumerate(names):
            for d, r in enumerate(RES):
                floor = max(specs[name]["min"].get(r, 0), (specs[name]["guaranteed"] or {}).get(r, 0))
                if specs[name]["allow_lent"]:
                    assert rt[name].get(r, 0) <= max(lim[i, d], floor)


@pytest.mark.parametrize("seed", range(10))
def test_pod_delete_and_quota_update_match_oracle(lib, seed):
    """OnPodDelete / OnQuotaUpdate events between refreshes: runtime and PreFilter still match the oracle."""
    rng = random.Random(1000 + seed)
    names, parents, specs = _random_forest(rng, rng.randrange(2, 16))
    total = {r: rng.randrange(100_000, 1_000_000) for r in RES}
    p = ElasticQuotaPlugin(resources=RES, enable_check_parent_quota=True, lib=lib)
    p.update_cluster_total_resource(total)
    tree = oq.QuotaTree(total)
    for name in names:
        p.on_quota_add(name, parent=parents[name], **specs[name])
        tree.add(oq.Quota(name, parent=parents[name], **specs[name]))
    pods = []
    for _ in range(60):
        name = rng.choice(names)
        req = {r: rng.randrange(0, 40_000) for r in RES}
        a, np_ = rng.random() < 0.6, rng.random() < 0.3
        p.on_pod_add(name, req, a, np_)
        tree.add_pod(name, req, a, np_)
        pods.append((name, req, a, np_))
    for name, req, a, np_ in rng.sample(pods, 25):
        p.on_pod_delete(name, req, a, np_)
        tree.remove_pod(name, req, a, np_)
    for name in rng.sample(names, max(1, len(names) // 3)):
        mx = {r: rng.randrange(0, 200_000) for r in RES}
        p.on_quota_update(name, max=mx, allow_lent=not specs[name]["allow_lent"])
        q = tree.quotas[name]
        q.max, q.allow_lent = dict(mx), not specs[name]["allow_lent"]   # SharedWeight keeps its value
    got = p.refresh_runtime()
    tree.refresh()
    for name in names:
        assert got[name] == tree.quotas[name].runtime, name
    for _ in range(20):
        name = rng.choice(names)
        req = {r: rng.randrange(0, 60_000) for r in RES}
        st = p.pre_filter(name, req)
        code, failed, bad, _ = oq.pre_filter(tree, name, req, check_parent=True)
        assert st.is_success() == (code == "Success") and (st.is_success() or (st.quota, st.exceed) == (failed, bad))


def test_prefilter_refreshes_stale_runtime(lib):
    """PreFilter after quota / pod / total events with no explicit refresh reads the refreshed runtime
    (plugin.go:221-223 calls RefreshRuntime in every PreFilter): a quota added after the last refresh is
    limited like the oracle's, not admitted with an empty runtime."""
    rng = random.Random(42)
    for _ in range(20):
        names, parents, specs = _random_forest(rng, rng.randrange(2, 12))
        total = {r: rng.randrange(50_000, 500_000) for r in RES}
        p = ElasticQuotaPlugin(resources=RES, lib=lib)
        p.update_cluster_total_resource(total)
        tree = oq.QuotaTree(total)
        half = len(names) // 2
        for name in names[:half]:
            p.on_quota_add(name, parent=parents[name] if parents[name] in names[:half] else ROOT, **specs[name])
            tree.add(oq.Quota(name, parent=parents[name] if parents[name] in names[:half] else ROOT, **specs[name]))
        p.refresh_runtime()
        for name in names[half:]:   # after the refresh
            par = parents[name]
            p.on_quota_add(name, parent=par, **specs[name])
            tree.add(oq.Quota(name, parent=par, **specs[name]))
        for _ in range(30):
            name = rng.choice(names)
            req = {r: rng.randrange(0, 40_000) for r in RES}
            a = rng.random() < 0.5
            p.on_pod_add(name, req, a)
            tree.add_pod(name, req, a)
        tree.refresh()
        for _ in range(10):
            name = rng.choice(names)
            req = {r: rng.randrange(0, 60_000) for r in RES}
            st = p.pre_filter(name, req)
            code, failed, bad, _ = oq.pre_filter(tree, name, req)
            assert st.is_success() == (code == "Success"), name
            assert st.is_success() or (st.quota, st.exceed) == (failed, bad)


def test_used_clamps_at_zero(lib):
    """addUsedNonNegativeNoLock (quota_info.go:252-261): deleting more used than a quota holds leaves 0, in the
    C-ABI and in the oracle alike, and later PreFilter checks are not loosened by a negative used."""
    p = ElasticQuotaPlugin(resources=RES, enable_runtime_quota=False, lib=lib)   # limit = Max
    total = {"cpu": 100_000, "memory": 1 << 30}
    p.update_cluster_total_resource(total)
    tree = oq.QuotaTree(total)
    for name, par in (("a", ROOT), ("b", "a")):
        spec = dict(max={"cpu": 10_000, "memory": 1 << 28}, min={"cpu": 1_000})
        p.on_quota_add(name, parent=par, **spec)
        tree.add(oq.Quota(name, parent=par, **spec))
    p.on_pod_add("b", {"cpu": 3_000}, assigned=True, non_preemptible=True)
    tree.add_pod("b", {"cpu": 3_000}, True, True)
    p.on_pod_delete("b", {"cpu": 5_000, "memory": 7}, assigned=True, non_preemptible=True)
    tree.remove_pod("b", {"cpu": 5_000, "memory": 7}, True, True)
    for name in ("a", "b"):
        assert p.get(name, "used") == {}, name
        assert p.get(name, "non_preemptible_used") == {}, name
        assert all(v == 0 for v in tree.quotas[name].used.values())
        assert all(v == 0 for v in tree.quotas[name].non_preemptible_used.values())
    tree.refresh()
    for cpu in (9_000, 10_000, 10_001):
        st = p.pre_filter("b", {"cpu": cpu})
        code, _, _, _ = oq.pre_filter(tree, "b", {"cpu": cpu}, runtime_quota=False)
        assert st.is_success() == (code == "Success") == (cpu <= 10_000)


def test_admit_batch_error_withdraws_speculation(lib):
    """An engine failure inside schedule_with_quota withdraws the run's speculative Reserves."""
    from koordinator_amd.quota import schedule_with_quota

    class Boom:
        def schedule(self, pods, seq):
            raise RuntimeError("injected engine failure")

    p = ElasticQuotaPlugin(resources=RES, enable_runtime_quota=False, lib=lib)
    p.update_cluster_total_resource({"cpu": 100_000, "memory": 1 << 30})
    p.on_quota_add("a", max={"cpu": 50_000, "memory": 1 << 29})
    p.on_pod_add("a", {"cpu": 1_000}, assigned=True)
    pods = np.zeros(4, abi.POD_DTYPE)
    with pytest.raises(RuntimeError, match="injected"):
        schedule_with_quota(Boom(), p, pods, [("a", {"cpu": 2_000}, False)] * 4)
    assert p.get("a", "used") == {"cpu": 1_000}
