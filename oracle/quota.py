"""ElasticQuota admission oracle — TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker, never by the
product path, which is libgpuscore's gs_quota_* in koordinator_amd/csrc/gs_quota.cpp).

A pure-Python restatement over ResourceList dicts {resource name: int} (getQuantityValue units: cpu milli,
everything else Value(); elasticquota/core/runtime_quota_calculator.go:500-505), kept close to the Go types so
missing-key semantics are explicit. Pinned by the reference's own test vectors (tests/golden/quota.json:
runtime_quota_calculator_test.go and plugin_test.go cases).
"""
from __future__ import annotations

ROOT = "koordinator-root-quota"   # extension.RootQuotaName


def redistribution(nodes: dict, total: int) -> None:
    """quotaTree.redistribution (runtime_quota_calculator.go:106-138). nodes: name -> dict(request, min,
    guarantee, shared_weight, allow_lent); sets node['runtime']."""
    to_partition, total_w, adjust = total, 0, []
    for n in nodes.values():
        m = n["min"]
        if n["guarantee"] > m:
            m = n["guarantee"]
        if n["request"] > m:
            adjust.append(n)
            total_w += n["shared_weight"]
            n["runtime"] = m
        else:
            n["runtime"] = n["request"] if n["allow_lent"] else m
        to_partition -= n["runtime"]
    if to_partition > 0:
        _iteration(to_partition, total_w, adjust)


def _iteration(total: int, total_w: int, nodes: list) -> None:
    """iterationForRedistribution (runtime_quota_calculator.go:140-166)."""
    if total_w <= 0:
        return
    again, part, again_w = [], 0, 0
    for n in nodes:
        n["runtime"] += int(float(n["shared_weight"]) * float(total) / float(total_w) + 0.5)
        if n["runtime"] < n["request"]:
            again.append(n)
            again_w += n["shared_weight"]
        else:
            part += n["runtime"] - n["request"]
            n["runtime"] = n["request"]
    if part > 0 and again:
        _iteration(part, again_w, again)


class Quota:
    """The QuotaInfo fields the admission path reads (elasticquota/core/quota_info.go)."""

    def __init__(self, name, parent=ROOT, max=None, min=None, shared_weight=None, allow_lent=True,
                 guaranteed=None):
        self.name, self.parent = name, parent
        self.max = dict(max or {})
        self.min = dict(min or {})
        self.shared_weight = dict(self.max if shared_weight is None else shared_weight)
        self.allow_lent = allow_lent
        self.guaranteed = dict(guaranteed or {})
        self.pod_request: dict = {}          # pods charged to this quota itself
        self.used: dict = {}
        self.non_preemptible_used: dict = {}
        self.request: dict = {}              # CalculateInfo.Request (settled)
        self.runtime: dict = {}


def _add(a: dict, b: dict) -> dict:
    out = dict(a)
    for k, v in b.items():
        out[k] = out.get(k, 0) + v
    return out


def _add_non_negative(a: dict, b: dict) -> dict:
    """addUsedNonNegativeNoLock (quota_info.go:252-261): quotav1.Add, then every negative entry set to 0."""
    return {k: max(0, v) for k, v in _add(a, b).items()}


class QuotaTree:
    """GroupQuotaManager, restated for a settled tree (every request delta applied, every runtime refreshed)."""

    def __init__(self, total: dict):
        self.total = dict(total)   # totalResourceExceptSystemAndDefaultUsed
        self.quotas: dict[str, Quota] = {}

    def add(self, q: Quota) -> Quota:
        self.quotas[q.name] = q
        return q

    def add_pod(self, quota: str, request: dict, assigned: bool, non_preemptible: bool = False):
        """OnPodAdd: request always, used once assigned — charged to the quota and every ancestor
        (updateGroupDeltaRequestNoLock / updateGroupDeltaUsedNoLock, group_quota_manager.go:170-255)."""
        q = self.quotas[quota]
        q.pod_request = _add(q.pod_request, request)
        if assigned:
            name = quota
            while name != ROOT:
                a = self.quotas[name]
                a.used = _add_non_negative(a.used, request)
                if non_preemptible:
                    a.non_preemptible_used = _add_non_negative(a.non_preemptible_used, request)
                name = a.parent

    def remove_pod(self, quota: str, request: dict, assigned: bool, non_preemptible: bool = False):
        """OnPodDelete: request leaves the quota (non-negative), used leaves the chain if assigned."""
        q = self.quotas[quota]
        q.pod_request = {k: max(0, q.pod_request.get(k, 0) - request.get(k, 0))
                         for k in set(q.pod_request) | set(request)}
        if assigned:
            name = quota
            while name != ROOT:
                a = self.quotas[name]
                a.used = _add_non_negative(a.used, {k: -v for k, v in request.items()})
                if non_preemptible:
                    a.non_preemptible_used = _add_non_negative(a.non_preemptible_used,
                                                               {k: -v for k, v in request.items()})
                name = a.parent

    def children(self, name: str) -> list[Quota]:
        return [q for q in self.quotas.values() if q.parent == name]

    def limit_request(self, q: Quota) -> dict:
        """getLimitRequestNoLock (quota_info.go:201-212)."""
        return {k: (min(v, q.max[k]) if k in q.max else v) for k, v in q.request.items()}

    def _settle_request(self, q: Quota) -> None:
        """recursiveUpdateGroupTreeWithDeltaRequest (group_quota_manager.go:184-224), settled: ChildRequest =
        own pods + children's limited requests; a quota that does not lend requests at least its Min."""
        child = dict(q.pod_request)
        for c in self.children(q.name):
            self._settle_request(c)
            child = _add(child, self.limit_request(c))
        child = {k: max(v, 0) for k, v in child.items()}
        if not q.allow_lent:
            for r, m in q.min.items():
                if r not in child or m > child[r]:
                    child[r] = m
        q.request = child

    def refresh(self) -> None:
        """refreshRuntimeNoLock (group_quota_manager.go:264-321) for every quota: each parent's runtime
        (the root's: total) is redistributed over its children per key of the union of all Max keys
        (updateResourceKeyNoLock :558-576, calculateRuntimeNoLock runtime_quota_calculator.go:486-492)."""
        keys = set()
        for q in self.quotas.values():
            keys |= set(q.max)
        for c in self.children(ROOT):
            self._settle_request(c)

        def down(parent: str, total: dict):
            kids = self.children(parent)
            if not kids:
                return
            for k in keys:
                nodes = {c.name: {"request": self.limit_request(c).get(k, 0), "min": c.min.get(k, 0),
                                  "guarantee": c.guaranteed.get(k, 0), "shared_weight": c.shared_weight.get(k, 0),
                                  "allow_lent": c.allow_lent} for c in kids}
                redistribution(nodes, total.get(k, 0))
                for c in kids:
                    c.runtime[k] = nodes[c.name]["runtime"]
            for c in kids:
                down(c.name, c.runtime)

        for q in self.quotas.values():
            q.runtime = {}
        down(ROOT, self.total)


def less_equal(a: dict, b: dict) -> tuple[bool, list]:
    """[upstream] quotav1.LessThanOrEqual (k8s.io/apiserver/pkg/quota/v1/resources.go): every key of b that a
    holds must satisfy a <= b. Exceeding names in sorted order (the Go map order is random)."""
    bad = sorted(k for k, v in b.items() if k in a and a[k] > v)
    return not bad, bad


def pre_filter(tree: QuotaTree, quota: str | None, request: dict, non_preemptible=False, runtime_quota=True,
               check_parent=False):
    """Plugin.PreFilter (plugin.go:210-254) + checkQuotaRecursive (plugin_helper.go:281-297).
    Returns (code, quota name that failed, exceeding names, quotaNameTopo)."""
    if not quota:
        return "Success", None, [], []

    def limit(q):
        return q.runtime if runtime_quota else q.max

    q = tree.quotas[quota]
    masked = {k: v + q.used.get(k, 0) for k, v in request.items()}
    ok, bad = less_equal(masked, limit(q))
    if not ok:
        return "Insufficient quotas", quota, bad, [quota]
    if non_preemptible:
        masked = {k: v + q.non_preemptible_used.get(k, 0) for k, v in request.items()}
        ok, bad = less_equal(masked, q.min)
        if not ok:
            return "Insufficient non-preemptible quotas", quota, bad, [quota]
    if check_parent:
        topo, name = [quota], quota
        while True:
            a = tree.quotas[name]
            ok, bad = less_equal({k: v + a.used.get(k, 0) for k, v in request.items()}, limit(a))
            if not ok:
                return "Insufficient quotas", name, bad, topo
            if a.parent == ROOT:
                break
            name = a.parent
            topo = [name] + topo
    return "Success", None, [], []
