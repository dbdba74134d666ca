"""ElasticQuota admission, host mirror of the reference plugin's PreFilter gate over libgpuscore's gs_quota_*.

Mirrors elasticquota/plugin.go:210-254 (PreFilter), plugin_helper.go:281-319 (checkQuotaRecursive,
getQuotaInfoUsedLimit) and the GroupQuotaManager state it reads (core/group_quota_manager.go): quotas form a forest
under the root quota; pods add request to their quota (and used once assigned, to it and every ancestor); the
runtime of every quota is refreshed from the cluster total through the C++ water filling
(core/runtime_quota_calculator.go:106-166). ResourceLists are {name: int} in getQuantityValue units (cpu milli,
everything else Value()). Status messages follow the reference's text; Quantity.String() is rendered for the
integral cpu / byte values the scheduler carries (cpu "Nm" or whole cores, other resources as integers).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import abi

ROOT = "koordinator-root-quota"   # extension.RootQuotaName
DEFAULT_RESOURCES = ("cpu", "memory", "nvidia.com/gpu", "ephemeral-storage",
                     "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory", "pods", "koordinator.sh/gpu")


@dataclass
class Status:
    code: str                 # "Success" | "Unschedulable"
    message: str = ""
    quota: str | None = None  # the quota whose check failed
    exceed: list = field(default_factory=list)

    def is_success(self) -> bool:
        return self.code == "Success"


def _fmt_quantity(name: str, v: int) -> str:
    if name == "cpu":
        return str(v // 1000) if v % 1000 == 0 else f"{v}m"
    return str(v)


def print_resource_list(rl: dict) -> str:
    """printResourceList (plugin_helper.go:299-312): "name:quantity" sorted, "<empty>" when empty."""
    if not rl:
        return "<empty>"
    return ",".join(sorted(f"{k}:{_fmt_quantity(k, v)}" for k, v in rl.items()))


class ElasticQuotaPlugin:
    def __init__(self, resources=DEFAULT_RESOURCES, enable_runtime_quota=True, enable_check_parent_quota=False,
                 lib=None):
        if len(resources) > abi.GS_QUOTA_DIMS:
            raise ValueError(f"at most {abi.GS_QUOTA_DIMS} resource dimensions")
        self.lib = lib or abi.load()
        self.resources = list(resources)
        self.dim = {r: i for i, r in enumerate(self.resources)}
        self.enable_runtime_quota = enable_runtime_quota
        self.enable_check_parent_quota = enable_check_parent_quota
        self.total: dict = {}
        self.names: list[str] = []
        self.index: dict[str, int] = {}
        self.groups: list[abi.GsQuotaGroup] = []
        self.parent_names: list[str] = []
        self.runtime = np.zeros((0, abi.GS_QUOTA_DIMS), np.int64)
        self.runtime_mask = np.zeros(0, np.uint32)
        # RefreshRuntime runs in every PreFilter (plugin.go:221-223) and recomputes once a request, Max/Min/weight
        # or the cluster total changed; here: every mutator marks the runtime stale, PreFilter refreshes it
        self._runtime_stale = True

    # ---- ResourceList <-> dense dimensions ----
    def _dense(self, rl: dict | None) -> tuple[np.ndarray, int]:
        out, mask = np.zeros(abi.GS_QUOTA_DIMS, np.int64), 0
        for k, v in (rl or {}).items():
            if k not in self.dim:
                raise KeyError(f"resource {k!r} has no quota dimension (configured: {self.resources})")
            out[self.dim[k]] = int(v)
            mask |= 1 << self.dim[k]
        return out, mask

    def _sparse(self, vals, mask: int) -> dict:
        return {r: int(vals[d]) for r, d in self.dim.items() if mask >> d & 1}

    # ---- GroupQuotaManager updates ----
    def update_cluster_total_resource(self, total: dict):
        """UpdateClusterTotalResource; here already net of the system / default quotas' used."""
        self.total = dict(total)
        self._runtime_stale = True

    def on_quota_add(self, name, parent=ROOT, max=None, min=None, shared_weight=None, allow_lent=True,
                     guaranteed=None):
        """OnQuotaAdd -> NewQuotaInfoFromQuota: SharedWeight defaults to Max."""
        if name in self.index:
            raise ValueError(f"quota {name!r} exists")
        g = abi.GsQuotaGroup()
        g.allow_lent = 1 if allow_lent else 0
        for fld, rl in (("max", max), ("min", min), ("shared_weight", max if shared_weight is None else shared_weight),
                        ("guaranteed", guaranteed)):
            vals, mask = self._dense(rl)
            getattr(g, fld)[:] = vals.tolist()
            if fld in ("max", "min"):
                setattr(g, fld + "_mask", mask)
        if getattr(self, "_arr", None) is not None:   # detach the views before the forest grows
            self.groups = [abi.GsQuotaGroup.from_buffer_copy(x) for x in self.groups]
            self._arr = None
        self.index[name] = len(self.names)
        self.names.append(name)
        self.parent_names.append(parent)
        self.groups.append(g)
        self._runtime_stale = True

    def _chain(self, quota: str):
        name = quota
        while name != ROOT:
            yield self.groups[self.index[name]]
            name = self.parent_names[self.index[name]]

    def on_pod_add(self, quota: str, request: dict, assigned: bool, non_preemptible: bool = False):
        """OnPodAdd: the pod's request joins its quota's request; once assigned, its used (and, for a
        non-preemptible pod, non-preemptible used) joins the quota and every ancestor."""
        vals, _ = self._dense(request)
        g = self.groups[self.index[quota]]
        for d in range(abi.GS_QUOTA_DIMS):
            g.request[d] += int(vals[d])
        self._runtime_stale = True
        if assigned:
            for a in self._chain(quota):
                for d in range(abi.GS_QUOTA_DIMS):
                    a.used[d] += int(vals[d])
                    if non_preemptible:
                        a.non_preemptible_used[d] += int(vals[d])

    def on_pod_delete(self, quota: str, request: dict, assigned: bool, non_preemptible: bool = False):
        """OnPodDelete: the pod's request leaves its quota (clamped at zero, addRequestNonNegativeNoLock) and,
        if it was assigned, its used leaves the quota and every ancestor."""
        vals, _ = self._dense(request)
        g = self.groups[self.index[quota]]
        for d in range(abi.GS_QUOTA_DIMS):
            g.request[d] = max(0, g.request[d] - int(vals[d]))
        self._runtime_stale = True
        if assigned:
            self.reserve_pod(quota, request, non_preemptible, sign=-1)

    def on_quota_update(self, name, max=None, min=None, shared_weight=None, allow_lent=None):
        """OnQuotaUpdate for the spec fields the runtime reads (Max, Min, SharedWeight, AllowLentResource);
        the next PreFilter (or refresh_runtime()) recomputes the runtime."""
        g = self.groups[self.index[name]]
        self._runtime_stale = True
        if allow_lent is not None:
            g.allow_lent = 1 if allow_lent else 0
        for fld, rl in (("max", max), ("min", min), ("shared_weight", shared_weight)):
            if rl is None:
                continue
            vals, mask = self._dense(rl)
            getattr(g, fld)[:] = vals.tolist()
            if fld in ("max", "min"):
                setattr(g, fld + "_mask", mask)

    def _array(self):
        """The forest as one ctypes array; self.groups become views into it, so native Reserve calls and
        Python-side updates see the same memory."""
        n = len(self.groups)
        if getattr(self, "_arr", None) is None or len(self._arr) != max(1, n):
            for i, p in enumerate(self.parent_names):
                self.groups[i].parent = -1 if p == ROOT else self.index[p]
            self._arr = (abi.GsQuotaGroup * max(1, n))(*self.groups)
            self.groups = [self._arr[i] for i in range(n)]
        return self._arr

    def refresh_runtime(self) -> dict:
        """RefreshRuntime for every quota; returns {quota: runtime ResourceList}."""
        n = len(self.groups)
        arr = self._array()
        total, _ = self._dense(self.total)
        self.runtime = np.zeros((max(n, 1), abi.GS_QUOTA_DIMS), np.int64)
        self.runtime_mask = np.zeros(max(n, 1), np.uint32)
        rc = self.lib.gs_quota_refresh_runtime(arr, n, abi.ptr(total), abi.ptr(self.runtime), None,
                                               abi.ptr(self.runtime_mask))
        if rc != 0:
            raise RuntimeError(f"gs_quota_refresh_runtime: {rc}")
        self._runtime_stale = False
        return {name: self._sparse(self.runtime[i], int(self.runtime_mask[i])) for i, name in enumerate(self.names)}

    def set_runtime(self, quota: str, runtime: dict):
        """What the reference's tests do with qi.CalculateInfo.Runtime = ... (plugin_test.go:686-689)."""
        self._fresh_runtime()
        vals, mask = self._dense(runtime)
        i = self.index[quota]
        self.runtime[i] = vals
        self.runtime_mask[i] = mask

    def _fresh_runtime(self):
        """The runtime PreFilter reads: recomputed when a mutator made it stale (with runtime quota enabled; with it
        disabled PreFilter reads Max and never refreshes)."""
        if self._runtime_stale and self.enable_runtime_quota:
            self.refresh_runtime()
        n = len(self.groups)
        if self.runtime.shape[0] < n:   # runtime quota disabled: quotas added since have no Runtime keys
            rt = np.zeros((n, abi.GS_QUOTA_DIMS), np.int64)
            rt[:self.runtime.shape[0]] = self.runtime
            rm = np.zeros(n, np.uint32)
            rm[:self.runtime_mask.shape[0]] = self.runtime_mask
            self.runtime, self.runtime_mask = rt, rm

    def get(self, quota: str, what: str) -> dict:
        g = self.groups[self.index[quota]]
        mask = {"max": g.max_mask, "min": g.min_mask}.get(what, (1 << abi.GS_QUOTA_DIMS) - 1)
        vals = list(getattr(g, what))
        rl = self._sparse(vals, mask)
        return rl if what in ("max", "min") else {k: v for k, v in rl.items() if v}

    # ---- PreFilter ----
    def pre_filter(self, quota: str | None, request: dict, non_preemptible: bool = False) -> Status:
        if not quota:
            return Status("Success")
        if quota not in self.index:
            return Status("Error", f"Could not find the specified ElasticQuota")
        req, req_mask = self._dense(request)
        flags = self._flags(non_preemptible)
        n = len(self.groups)
        self._fresh_runtime()
        arr = self._array()
        st = abi.GsQuotaStatus()
        rc = self.lib.gs_quota_prefilter(arr, n, abi.ptr(self.runtime), abi.ptr(self.runtime_mask),
                                         self.index[quota], abi.ptr(req), req_mask, flags, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"gs_quota_prefilter: {rc}")
        return self._status(st, quota, request)

    def _flags(self, non_preemptible: bool) -> int:
        return ((abi.GS_QUOTA_RUNTIME if self.enable_runtime_quota else 0)
                | (abi.GS_QUOTA_CHECK_PARENT if self.enable_check_parent_quota else 0)
                | (abi.GS_QUOTA_NON_PREEMPTIBLE if non_preemptible else 0))

    def _status(self, st, quota: str, request: dict) -> Status:
        """gs_quota_status -> the reference's framework.Status text (plugin.go:229-243, plugin_helper.go:287-291)."""
        if st.code == abi.GS_QUOTA_ADMIT:
            return Status("Success")
        failed = self.names[st.group]
        exceed = [r for r, d in self.dim.items() if st.exceed_mask >> d & 1]
        used = {k: v for k, v in self._sparse(list(st.used), (1 << abi.GS_QUOTA_DIMS) - 1).items() if v}
        i = st.group
        limit = (self._sparse(self.runtime[i], int(self.runtime_mask[i])) if self.enable_runtime_quota
                 else self.get(failed, "max"))
        if st.code == abi.GS_QUOTA_INSUFFICIENT_NON_PREEMPTIBLE:
            msg = (f"Insufficient non-preemptible quotas, quotaName: {failed}, min: "
                   f"{print_resource_list(self.get(failed, 'min'))}, nonPreemptibleUsed: "
                   f"{print_resource_list(used)}, pod's request: "
                   f"{print_resource_list(request)}, exceedDimensions: [{' '.join(exceed)}]")
        elif st.depth == 0:   # the pod's own quota (the first check of plugin.go:229-234)
            msg = (f"Insufficient quotas, quotaName: {failed}, runtime: {print_resource_list(limit)}, used: "
                   f"{print_resource_list(used)}, pod's request: {print_resource_list(request)}, "
                   f"exceedDimensions: [{' '.join(exceed)}]")
        else:
            topo, name = [quota], quota
            for _ in range(st.depth):
                name = self.parent_names[self.index[name]]
                topo.insert(0, name)
            msg = (f"Insufficient quotas, quotaNameTopo: [{' '.join(topo)}], runtime: {print_resource_list(limit)}, "
                   f"used: {print_resource_list(used)}, pod's request: "
                   f"{print_resource_list(request)}, exceedDimensions: [{' '.join(exceed)}]")
        return Status("Unschedulable", msg, failed, exceed)

    # ---- Reserve / Unreserve (GroupQuotaManager.ReservePod / UnreservePod, group_quota_manager.go:791-805) ----
    def reserve_pod(self, quota: str | None, request: dict, non_preemptible: bool = False, sign: int = 1):
        """The pod's request joins `used` (and non-preemptible used) of its quota and every ancestor."""
        if not quota:
            return
        req, _ = self._dense(request)
        arr = self._array()
        rc = self.lib.gs_quota_reserve(arr, len(self.groups), self.index[quota], abi.ptr(req),
                                       self._flags(non_preemptible), sign)
        if rc != 0:
            raise RuntimeError(f"gs_quota_reserve: {rc}")

    def unreserve_pod(self, quota: str | None, request: dict, non_preemptible: bool = False):
        self.reserve_pod(quota, request, non_preemptible, sign=-1)


def schedule_with_quota(engine, plugin: ElasticQuotaPlugin, pods, pod_quota, seq=None, pod_ext=None):
    """Quota-gated batched scheduleOne: per pod in order, ElasticQuota PreFilter, then (if admitted) the node
    loop of `engine.schedule` (libgpuscore gs_schedule), then quota Reserve on a placement — the reference's
    sequential order (PreFilter -> Filter/Score -> selectHost -> Reserve) kept exact while the node loop runs
    in batches.

    Admitted pods are reserved speculatively (as if placed) so that a run of admitted pods goes to the engine
    as one batch. The check is monotone in `used` (used + request <= limit), so a pod admitted under
    speculation stays admitted when an earlier pod of its batch finds no node and is unreserved; only a
    rejection can depend on the speculation: it is final when the pod is also rejected against the certain used
    (its chain's used minus the run's speculative Reserves), otherwise the run is cut before that pod, which is
    re-checked once the run's true placements are reserved. After the engine call the run is settled natively
    (gs_quota_settle_batch): speculation withdrawn, run replayed with the true placements, so statuses and used
    are those of the one-pod-at-a-time order. Runtime does not change inside a batch (it
    follows requests, which a Reserve does not touch). pod_quota[i] = (quota name or None, request
    ResourceList, non_preemptible). Returns (placements, statuses): placements in the engine's dtype with
    node = -1 for quota-rejected pods, statuses[i] = the PreFilter Status of pod i. pod_ext (gs_pod_ext per pod):
    the runs go through engine.schedule_ext (Reservation + DeviceShare, config C5) and the result is
    (placements, ext placements, statuses)."""
    pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
    n = len(pods)
    seq = np.arange(n, dtype=np.uint64) if seq is None else np.ascontiguousarray(seq, dtype=np.uint64)
    out = np.zeros(n, abi.PLACEMENT_DTYPE)
    out["node"] = -1
    xout = np.zeros(n, abi.EXT_PLACEMENT_DTYPE) if pod_ext is not None else None
    qidx = np.array([plugin.index[q] if q else -1 for q, _, _ in pod_quota], np.int32)
    reqs = np.zeros((max(n, 1), abi.GS_QUOTA_DIMS), np.int64)
    masks = np.zeros(max(n, 1), np.uint32)
    for j, (_, req, _) in enumerate(pod_quota):
        reqs[j], masks[j] = plugin._dense(req)
    flags = np.array([plugin._flags(np_) for _, _, np_ in pod_quota] or [0], np.uint32)
    plugin._fresh_runtime()
    arr = plugin._array()
    ng = len(plugin.groups)
    st = (abi.GsQuotaStatus * max(n, 1))()
    consumed = C.c_uint32()
    i = 0
    while i < n:
        rc = plugin.lib.gs_quota_admit_batch(
            arr, ng, abi.ptr(plugin.runtime), abi.ptr(plugin.runtime_mask), qidx[i:].ctypes.data,
            reqs[i:].ctypes.data, masks[i:].ctypes.data, flags[i:].ctypes.data, n - i,
            C.byref(st, i * C.sizeof(abi.GsQuotaStatus)), C.byref(consumed))
        if rc != 0 or consumed.value == 0:
            raise RuntimeError(f"gs_quota_admit_batch: rc={rc} consumed={consumed.value}")
        j = i + consumed.value
        seg = np.array([p for p in range(i, j) if st[p].code == abi.GS_QUOTA_ADMIT], np.int64)
        if len(seg):
            try:
                if pod_ext is None:
                    res = engine.schedule(pods[seg], seq[seg])
                else:
                    res, xres = engine.schedule_ext(pods[seg], pod_ext[seg], seq[seg])
                    xout[seg] = xres
            except Exception:
                # the run's speculative Reserves leave the forest (used as before the run), then the error surfaces
                for p in seg:
                    if qidx[p] >= 0:
                        plugin.lib.gs_quota_reserve(arr, ng, int(qidx[p]), reqs[p].ctypes.data, int(flags[p]), -1)
                raise
            out[seg] = res
        # withdraw the speculation and replay the run with the true placements (exact statuses and used)
        placed = np.ascontiguousarray(out["node"][i:j], dtype=np.int32)
        rc = plugin.lib.gs_quota_settle_batch(
            arr, ng, abi.ptr(plugin.runtime), abi.ptr(plugin.runtime_mask), qidx[i:].ctypes.data,
            reqs[i:].ctypes.data, masks[i:].ctypes.data, flags[i:].ctypes.data, j - i, abi.ptr(placed),
            C.byref(st, i * C.sizeof(abi.GsQuotaStatus)))
        if rc != 0:
            raise RuntimeError(f"gs_quota_settle_batch: {rc}")
        i = j
    statuses = [plugin._status(st[p], pod_quota[p][0], pod_quota[p][1]) for p in range(n)]
    return (out, statuses) if pod_ext is None else (out, xout, statuses)
