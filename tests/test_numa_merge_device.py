"""The reference's topology-manager Merge vectors (tests/golden/numa_policy.json, from
frameworkext/topologymanager/policy_test.go and policy_{best_effort,restricted,single_numa_node}_test.go) driven through
the DEVICE merge itself (gs_numa_dev.h merge_hint_lists, the code every NUMA-policy pair evaluation runs), via
gs_debug_numa_merge.

The device merge takes hint lists in the form NodeNUMAResource's provider produces them (resource_manager.go:418-532):
at most two lists (cpu, memory), hints as positions of the IterateBitMasks order, Preferred iff the mask size is the
smallest among the masks whose total covers the request. A policy_test case is encoded when its providers fit that form
after filterProvidersHints' exact equivalences (policy.go:94-126: a nil provider, a nil resource entry and a single
{nil, preferred} hint each add one any-NUMA preferred hint, which the merge ignores; an empty list and a single
{nil, not preferred} hint are the {nil, false} marker); the others are counted and named in the skip list below.
CPU tests pin the encoding (decoded back and merged by the oracle, the expected hint must come out); the GPU test
asserts the device's admit verdict and affinity against the reference's expectation."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi
from oracle import oracle as orc

G = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "numa_policy.json")))
POLICY = {"best_effort": abi.GS_NUMA_POLICY_BEST_EFFORT, "restricted": abi.GS_NUMA_POLICY_RESTRICTED,
          "single_numa_node": abi.GS_NUMA_POLICY_SINGLE_NUMA_NODE}
KORD4 = [(0xFEDB7CA69538421 >> (4 * i)) & 15 for i in range(15)]   # position -> mask (gs_numa_dev.h kOrd4)
CASES = [(pol, c) for pol, groups in G["runs"].items() for g in groups for c in G["cases"][g]]


def _bits(mask):
    return sum(1 << z for z in mask)


def _lists(case):
    """filterProvidersHints with the any-NUMA preferred lists dropped: a list of hint lists or the marker 'empty'."""
    out = []
    for prov in case["providers"]:
        if not prov:
            continue
        for r in sorted(prov):
            hs = prov[r]
            if hs is None or (len(hs) == 1 and hs[0]["mask"] is None and hs[0]["preferred"]):
                continue
            if len(hs) == 0 or (len(hs) == 1 and hs[0]["mask"] is None):
                out.append("empty")
                continue
            if any(h["mask"] is None for h in hs):
                raise ValueError("a nil mask among other hints")
            out.append(hs)
    return out


def encode(pol, case):
    """gs_merge_case of a policy_test case, or raises ValueError naming why it is outside the device's domain."""
    nz = len(G["numa_nodes"])
    valid = [i for i, m in enumerate(KORD4) if m < (1 << nz)]
    lists = _lists(case)
    if len(lists) > 2:
        raise ValueError("more than two hint lists")
    rec = np.zeros(1, abi.MERGE_CASE_DTYPE)[0]
    rec["nz"], rec["policy"] = nz, POLICY[pol]
    for k, hs in enumerate(lists):
        l = tot = 0
        if hs != "empty":
            pos = [KORD4.index(_bits(h["mask"])) for h in hs]
            if pos != sorted(set(pos)):
                raise ValueError("hints not in IterateBitMasks order")
            sizes = [len(h["mask"]) for h in hs]
            pref = [s for s, h in zip(sizes, hs) if h["preferred"]]
            if pref:
                if len(set(pref)) != 1 or min(sizes) != pref[0] or any(
                        s == pref[0] for s, h in zip(sizes, hs) if not h["preferred"]):
                    raise ValueError("Preferred is not 'smallest size'")
                extra = 0
            else:   # no hint preferred: a smaller mask covers the total without being free
                small = [i for i in valid if bin(KORD4[i]).count("1") < min(sizes) and i not in pos]
                if not small:
                    raise ValueError("no preferred hint and no smaller mask")
                extra = 1 << small[0]
            l = sum(1 << i for i in pos)
            tot = l | extra
        else:
            tot = 1 << valid[-1]   # the request is covered by the full mask, which is not free: {nil, false}
        if k == 0:
            rec["lc"], rec["totc"], rec["has_cpu"], rec["tot_c_any"] = l, tot, 1, int(tot != 0)
        else:
            rec["lm"], rec["totm"], rec["has_mem"], rec["tot_m_any"] = l, tot, 1, int(tot != 0)
    return rec


def decode(rec):
    """The hint lists a gs_merge_case stands for (filterProvidersHints output), for the oracle's merge."""
    out = []
    for l, tot, has, any_ in ((rec["lc"], rec["totc"], rec["has_cpu"], rec["tot_c_any"]),
                              (rec["lm"], rec["totm"], rec["has_mem"], rec["tot_m_any"])):
        if not has:
            continue
        if l == 0:
            if any_:
                out.append([{"mask": None, "preferred": False}])
            continue
        smin = min(bin(KORD4[i]).count("1") for i in range(15) if tot >> i & 1)
        out.append([{"mask": [z for z in range(4) if KORD4[i] >> z & 1],
                     "preferred": bin(KORD4[i]).count("1") == smin} for i in range(15) if l >> i & 1])
    return out


def encoded():
    ok, skipped = [], []
    for pol, c in CASES:
        try:
            ok.append((pol, c, encode(pol, c)))
        except ValueError as e:
            skipped.append((pol, c["name"], str(e)))
    return ok, skipped


def want(pol, case):
    exp = case["expected"]
    admit = True if pol == "best_effort" else exp["preferred"]
    if exp["mask"] is None or (pol == "single_numa_node" and len(exp["mask"]) == len(G["numa_nodes"])):
        return admit, 0, 0
    return admit, 1, _bits(exp["mask"])


def test_encoding_covers_most_cases():
    ok, skipped = encoded()
    assert len(ok) >= 25, skipped
    assert {p for p, _, _ in ok} == set(POLICY)


@pytest.mark.parametrize("pol,case", CASES, ids=[f"{p}-{c['name'][:60]}" for p, c in CASES])
def test_encoding_is_exact(pol, case):
    """Decoded back into hint lists, an encoded case merges (oracle) to the reference's expected hint."""
    try:
        rec = encode(pol, case)
    except ValueError:
        pytest.skip("outside the device merge's input domain")
    got, admit = orc.policy_merge(POLICY[pol], G["numa_nodes"], decode(rec))
    assert got == case["expected"]
    assert admit == (True if pol == "best_effort" else got["preferred"])


@pytest.mark.gpu
def test_device_merge_reference_vectors():
    from koordinator_amd import config
    from koordinator_amd.engine import Engine
    ok, skipped = encoded()
    e = Engine(config.make_config(16, device=0, enabled=abi.GS_ENABLE_ALL))
    out = e.numa_merge(np.array([r for _, _, r in ok], abi.MERGE_CASE_DTYPE))
    bad = []
    for (pol, c, _), o in zip(ok, out):
        w = want(pol, c)
        got = (bool(o["admit"]), int(o["aff_has"]), int(o["aff"]) if o["aff_has"] else 0)
        if got != (bool(w[0]), w[1], w[2]):
            bad.append((pol, c["name"], got, w))
    assert not bad, bad
    print(f"device merge: {len(ok)} reference cases identical, {len(skipped)} outside the input domain: {skipped}")


def _gen_case(rng):
    """A random gs_merge_case with DeviceShare as the second provider (gpu_hints) and the filterProvidersHints lists it
    stands for: NodeNUMAResource's cpu / memory lists (hint scores), then r identical GPU lists (score 0)."""
    rec = np.zeros(1, abi.MERGE_CASE_DTYPE)[0]
    nz = int(rng.integers(1, 5))
    valid = [i for i, m in enumerate(KORD4) if m < (1 << nz)]
    rec["nz"], rec["policy"] = nz, int(rng.choice([abi.GS_NUMA_POLICY_BEST_EFFORT, abi.GS_NUMA_POLICY_RESTRICTED,
                                                    abi.GS_NUMA_POLICY_SINGLE_NUMA_NODE]))
    rec["score"] = rng.integers(0, 101, 15)
    rec["nil_hints"] = int(rng.random() < 0.05)

    def pick():
        return sum(1 << i for i in valid if rng.random() < 0.5)
    for res in ("c", "m"):
        has = rng.random() < 0.85
        l = pick()
        tot = l | pick()
        if rng.random() < 0.1:
            l = 0   # covered in total but never free: the {nil, false} marker
        if not has:
            l = tot = 0   # a resource the pod does not request has no positions
        rec["l" + res], rec["tot" + res] = l, tot
        rec["has_cpu" if res == "c" else "has_mem"] = int(has)
        rec["tot_c_any" if res == "c" else "tot_m_any"] = int(tot != 0)
    r = int(rng.choice([2, 3]))
    gl = 0 if rng.random() < 0.1 else pick()
    sizes = [bin(KORD4[i]).count("1") for i in range(15) if gl >> i & 1]
    gmin = int(rng.integers(1, (min(sizes) if sizes else nz) + 1))
    rec["gpu_hints"] = gl | (gmin << 16) | (r << 20)
    lists = []
    if not rec["nil_hints"]:
        for l, tot, has in ((rec["lc"], rec["totc"], rec["has_cpu"]), (rec["lm"], rec["totm"], rec["has_mem"])):
            if not has or not tot:
                continue
            if l == 0:
                lists.append([{"mask": None, "preferred": False}])
                continue
            smin = min(bin(KORD4[i]).count("1") for i in range(15) if tot >> i & 1)
            lists.append([{"mask": [z for z in range(4) if KORD4[i] >> z & 1],
                           "preferred": bin(KORD4[i]).count("1") == smin, "score": int(rec["score"][i])}
                          for i in range(15) if l >> i & 1])
    if not lists:
        lists.append([{"mask": None, "preferred": True}])   # NodeNUMAResource without hints
    g = ([{"mask": [z for z in range(4) if KORD4[i] >> z & 1], "preferred": bin(KORD4[i]).count("1") == gmin}
          for i in range(15) if gl >> i & 1] or [{"mask": None, "preferred": False}])
    lists += [g] * r
    return rec, lists


@pytest.mark.gpu
def test_device_merge_with_deviceshare_provider_matches_reference():
    """merge_hint_lists_gen (the extension path's merge over NodeNUMAResource's and DeviceShare's hint lists) on random
    list sets against the reference's permutation scan (oracle, mergeFilteredHints with hint scores), bit-exact."""
    from koordinator_amd import config
    from koordinator_amd.engine import Engine
    rng = np.random.default_rng(20260)
    cases = [_gen_case(rng) for _ in range(4000)]
    recs = np.array([c[0] for c in cases], abi.MERGE_CASE_DTYPE)
    e = Engine(config.make_config(4, enabled=abi.GS_ENABLE_ALL))
    got = e.numa_merge(recs)
    assert (got["pad"] == 0).all()   # no search past its bound
    for k, (rec, lists) in enumerate(cases):
        nz = int(rec["nz"])
        hint, admit = orc.policy_merge(int(rec["policy"]), list(range(nz)), lists)
        want_has = hint["mask"] is not None
        want_aff = _bits(hint["mask"]) if want_has else 0
        g = got[k]
        assert (bool(g["admit"]), bool(g["aff_has"])) == (admit, want_has), (k, rec, lists, hint)
        if want_has:
            assert int(g["aff"]) == want_aff, (k, rec, lists, hint)
