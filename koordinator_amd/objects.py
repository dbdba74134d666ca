"""Host-side decoding of Kubernetes-shaped object specs into the C-ABI structs.

In production this decoding is done by the Go wrapper with the reference's own helpers
(resourceapi.PodRequestsAndLimits, schedutil.GetNonzeroRequests, extension.GetPodPriorityClassWithDefault,
extension.GetNodeRawAllocatable, extension.GetCustomUsageThresholds — see INTEGRATION.md). This module
restates those helpers for specs written as plain dicts, so tests and the bench can build clusters:

  pod  = {"namespace": "default", "name": "p", "priority": 9999, "labels": {...}, "daemonset": False,
          "containers": [{"requests": {"cpu": "16", "memory": "32Gi"}, "limits": {...}}],
          "init_containers": [...], "overhead": {...}}
  node = {"allocatable": {"cpu": "96", "memory": "512Gi", "pods": 110}, "requested": {...},
          "annotations": {"raw_allocatable": {...}, "usage_thresholds": {...}}}
"""
from __future__ import annotations

import hashlib
import re
from decimal import Decimal
from fractions import Fraction

import numpy as np

from . import abi

RESOURCE_SLOTS = {
    "cpu": abi.GS_RES_CPU,
    "memory": abi.GS_RES_MEMORY,
    "ephemeral-storage": abi.GS_RES_EPHEMERAL,
    "kubernetes.io/batch-cpu": abi.GS_RES_BATCH_CPU,
    "kubernetes.io/batch-memory": abi.GS_RES_BATCH_MEMORY,
    "kubernetes.io/mid-cpu": abi.GS_RES_MID_CPU,
    "kubernetes.io/mid-memory": abi.GS_RES_MID_MEMORY,
}
AGG_TYPES = {"avg": abi.GS_AGG_AVG, "p50": abi.GS_AGG_P50, "p90": abi.GS_AGG_P90,
             "p95": abi.GS_AGG_P95, "p99": abi.GS_AGG_P99, "": abi.GS_AGG_NONE}
PRIORITY_CLASSES = {"koord-prod": abi.GS_PRIO_PROD, "koord-mid": abi.GS_PRIO_MID,
                    "koord-batch": abi.GS_PRIO_BATCH, "koord-free": abi.GS_PRIO_FREE}

_SUFFIX = {
    "": Fraction(1), "m": Fraction(1, 1000), "k": Fraction(10**3), "M": Fraction(10**6), "G": Fraction(10**9),
    "T": Fraction(10**12), "P": Fraction(10**15), "E": Fraction(10**18),
    "Ki": Fraction(2**10), "Mi": Fraction(2**20), "Gi": Fraction(2**30), "Ti": Fraction(2**40),
    "Pi": Fraction(2**50), "Ei": Fraction(2**60),
}
_QRE = re.compile(r"^([+-]?[0-9.]+)([a-zA-Z]*)$")


def parse_quantity(q) -> Fraction:
    """resource.MustParse -> exact rational value (numbers pass through)."""
    if isinstance(q, (int, np.integer)):
        return Fraction(int(q))
    m = _QRE.match(str(q).strip())
    if not m:
        raise ValueError(f"bad quantity {q!r}")
    return Fraction(Decimal(m.group(1))) * _SUFFIX[m.group(2)]


def _ceil(fr: Fraction) -> int:
    return -((-fr.numerator) // fr.denominator)


def slot_value(slot: int, q) -> int:
    """getResourceValue (loadaware/helper.go:146-151): cpu -> MilliValue, else Value (both round up)."""
    v = parse_quantity(q)
    return _ceil(v * 1000) if slot == abi.GS_RES_CPU else _ceil(v)


def name_key(namespace: str, name: str) -> int:
    """Stable 64-bit key for "namespace/name" (helper.go:142-144 getPodNamespacedName)."""
    return int.from_bytes(hashlib.blake2b(f"{namespace}/{name}".encode(), digest_size=8).digest(), "little")


def _rl(d: dict | None) -> dict[int, int]:
    out = {}
    for k, v in (d or {}).items():
        if k not in RESOURCE_SLOTS:
            continue
        s = RESOURCE_SLOTS[k]
        out[s] = slot_value(s, v)
    return out


def kube_qos(pod: dict) -> str:
    """[upstream] v1qos.GetPodQOS (pkg/apis/core/v1/helper/qos) over the QoS compute resources cpu/memory."""
    reqs, lims = {}, {}
    is_guaranteed = True
    for c in pod.get("containers", []) + pod.get("init_containers", []):
        for k, v in (c.get("requests") or {}).items():
            q = parse_quantity(v)
            if k in ("cpu", "memory") and q > 0:
                reqs[k] = reqs.get(k, 0) + q
        found = set()
        for k, v in (c.get("limits") or {}).items():
            q = parse_quantity(v)
            if k in ("cpu", "memory") and q > 0:
                found.add(k)
                lims[k] = lims.get(k, 0) + q
        if not {"cpu", "memory"} <= found:
            is_guaranteed = False
    if not reqs and not lims:
        return "BestEffort"
    if is_guaranteed:
        for k, v in reqs.items():
            if lims.get(k) != v:
                is_guaranteed = False
                break
    if is_guaranteed and len(reqs) == len(lims):
        return "Guaranteed"
    return "Burstable"


def priority_class(pod: dict) -> int:
    """extension.GetPodPriorityClassWithDefault (apis/extension/priority_utils.go:26-47)."""
    labels = pod.get("labels") or {}
    if "koordinator.sh/priority-class" in labels:
        return PRIORITY_CLASSES.get(labels["koordinator.sh/priority-class"], abi.GS_PRIO_NONE) or _qos_default(pod)
    p = pod.get("priority")
    if p is not None:
        if 9000 <= p <= 9999:
            return abi.GS_PRIO_PROD
        if 7000 <= p <= 7999:
            return abi.GS_PRIO_MID
        if 5000 <= p <= 5999:
            return abi.GS_PRIO_BATCH
        if 3000 <= p <= 3999:
            return abi.GS_PRIO_FREE
    return _qos_default(pod)


def _qos_default(pod: dict) -> int:
    labels = pod.get("labels") or {}
    q = labels.get("koordinator.sh/qosClass", "")
    if q not in ("LSE", "LSR", "LS", "BE", "SYSTEM"):
        kq = kube_qos(pod)
        q = {"Guaranteed": "LSR", "Burstable": "LS", "BestEffort": "BE"}[kq]
    if q in ("SYSTEM", "LSE", "LSR", "LS"):
        return abi.GS_PRIO_PROD
    if q == "BE":
        return abi.GS_PRIO_BATCH
    return abi.GS_PRIO_NONE


def make_pod(spec: dict) -> np.void:
    """Decode a pod spec: PodRequestsAndLimits + GetNonzeroRequests + priority class."""
    rec = np.zeros(1, abi.POD_DTYPE)[0]
    ns, name = spec.get("namespace", "default"), spec.get("name", "pod")
    rec["uid"] = spec.get("uid", name_key(ns, name + "#uid"))
    rec["name_key"] = name_key(ns, name)
    req = [0] * abi.GS_NUM_RES
    lim = [0] * abi.GS_NUM_RES
    nz = [0, 0]
    mask = 0
    for c in spec.get("containers", []):
        r, l = _rl(c.get("requests")), _rl(c.get("limits"))
        for s, v in r.items():
            req[s] += v
            mask |= 1 << s
        for s, v in l.items():
            lim[s] += v
        raw_req = c.get("requests") or {}
        nz[0] += slot_value(0, raw_req["cpu"]) if "cpu" in raw_req else 100          # DefaultMilliCPURequest
        nz[1] += slot_value(1, raw_req["memory"]) if "memory" in raw_req else 200 * 1024 * 1024
    for c in spec.get("init_containers", []):
        r, l = _rl(c.get("requests")), _rl(c.get("limits"))
        for s, v in r.items():
            mask |= 1 << s
            req[s] = max(req[s], v)
        for s, v in l.items():
            lim[s] = max(lim[s], v)
        raw_req = c.get("requests") or {}
        nzc = slot_value(0, raw_req["cpu"]) if "cpu" in raw_req else 100
        nzm = slot_value(1, raw_req["memory"]) if "memory" in raw_req else 200 * 1024 * 1024
        nz[0], nz[1] = max(nz[0], nzc), max(nz[1], nzm)
    for s, v in _rl(spec.get("overhead")).items():
        req[s] += v
        lim[s] += v if lim[s] else 0
        if s < 2:
            nz[s] += v
        mask |= 1 << s
    rec["requests"] = req
    rec["limits"] = lim
    rec["nonzero_requests"] = nz
    rec["request_mask"] = mask
    rec["priority_class"] = priority_class(spec)
    rec["flags"] = (abi.GS_POD_DAEMONSET if spec.get("daemonset") else 0) | \
                   (abi.GS_POD_TERMINATED if spec.get("terminated") else 0)
    return rec


def _mask_vals(d: dict | None) -> tuple[list[int], int]:
    vals, mask = [0, 0], 0
    for k, v in (d or {}).items():
        if k == "cpu":
            vals[0], mask = int(v), mask | abi.GS_USAGE_CPU
        elif k == "memory":
            vals[1], mask = int(v), mask | abi.GS_USAGE_MEMORY
        else:
            mask |= abi.GS_USAGE_OTHER
    return vals, mask


def make_node(spec: dict) -> np.void:
    rec = np.zeros(1, abi.NODE_DTYPE)[0]
    alloc = _rl(spec.get("allocatable"))
    a = [0] * abi.GS_NUM_RES
    for s, v in alloc.items():
        a[s] = v
    rec["allocatable"] = a
    r = [0] * abi.GS_NUM_RES
    for s, v in _rl(spec.get("requested")).items():
        r[s] = v
    rec["requested"] = r
    nzr = spec.get("nonzero_requested")
    rec["nonzero_requested"] = [slot_value(0, nzr["cpu"]), slot_value(1, nzr["memory"])] if nzr else [r[0], r[1]]
    rec["allowed_pod_number"] = int((spec.get("allocatable") or {}).get("pods", 110))
    rec["pod_count"] = int(spec.get("pod_count", 0))
    ann = spec.get("annotations") or {}
    raw = ann.get("raw_allocatable")
    if raw is not None:
        m = 0
        vals = [0, 0]
        for k, v in raw.items():
            if k == "cpu":
                vals[0], m = slot_value(0, v), m | abi.GS_USAGE_CPU
            elif k == "memory":
                vals[1], m = slot_value(1, v), m | abi.GS_USAGE_MEMORY
            else:
                m |= abi.GS_USAGE_OTHER
        rec["raw_allocatable"] = vals
        rec["raw_allocatable_mask"] = m
    ut = ann.get("usage_thresholds")
    if ut is not None:
        flags = abi.GS_NODE_CUSTOM_THRESHOLDS
        v, m = _mask_vals(ut.get("usageThresholds"))
        rec["custom_usage_thresholds"], rec["custom_usage_mask"] = v, m
        v, m = _mask_vals(ut.get("prodUsageThresholds"))
        rec["custom_prod_usage_thresholds"], rec["custom_prod_usage_mask"] = v, m
        agg = ut.get("aggregatedUsage")
        rec["custom_agg_type"] = abi.GS_AGG_NONE
        if agg is not None:
            flags |= abi.GS_NODE_CUSTOM_AGGREGATED
            v, m = _mask_vals(agg.get("usageThresholds"))
            rec["custom_agg_usage_thresholds"], rec["custom_agg_usage_mask"] = v, m
            rec["custom_agg_type"] = AGG_TYPES[agg.get("usageAggregationType", "")]
            rec["custom_agg_duration_ns"] = int(agg.get("usageAggregatedDurationSeconds", 0) * 10**9)
        rec["custom_flags"] = flags
    else:
        rec["custom_agg_type"] = abi.GS_AGG_NONE
    return rec


def make_usage(rec, d: dict | None) -> None:
    m = 0
    for k, v in (d or {}).items():
        if k == "cpu":
            rec["cpu_milli"] = slot_value(0, v)
            m |= abi.GS_USAGE_CPU
        elif k == "memory":
            rec["memory"] = slot_value(1, v)
            m |= abi.GS_USAGE_MEMORY
        else:
            m |= abi.GS_USAGE_OTHER
    rec["mask"] = m


def make_metric(spec: dict | None, now_ns: int, lister: dict | None = None):
    """Decode a NodeMetric spec. Times are seconds relative to `now` ("update_time_rel": -10).
    lister: {(ns, name): priority_class} of pods the pod lister knows.
    Returns (gs_node_metric record, list of gs_pod_metric records)."""
    rec = np.zeros(1, abi.METRIC_DTYPE)[0]
    if spec is None:
        return rec, []
    rec["exists"] = 1
    if spec.get("update_time_rel") is not None:
        rec["has_update_time"] = 1
        rec["update_time_ns"] = now_ns + int(round(spec["update_time_rel"] * 10**9))
    if spec.get("report_interval_s") is not None:
        rec["has_report_interval"] = 1
        rec["report_interval_s"] = int(spec["report_interval_s"])
    nm = spec.get("node_metric")
    if nm is not None:
        rec["has_node_metric"] = 1
        make_usage(rec["node_usage"], nm.get("node_usage"))
        aggs = nm.get("aggregated", [])
        rec["n_aggregated"] = len(aggs)
        for i, ag in enumerate(aggs):
            a = rec["aggregated"][i]
            a["duration_ns"] = int(ag.get("duration_s", 0) * 10**9)
            tm = 0
            for t, usage in ag.get("usage", {}).items():
                ti = AGG_TYPES[t]
                tm |= 1 << ti
                make_usage(a["usage"][ti], usage)
            a["type_mask"] = tm
    pms = []
    lister = lister or {}
    for pm in spec.get("pods_metric", []):
        r = np.zeros(1, abi.POD_METRIC_DTYPE)[0]
        ns, name = pm.get("namespace", "default"), pm["name"]
        r["name_key"] = name_key(ns, name)
        if (ns, name) in lister:
            r["in_lister"] = 1
            r["priority_class"] = lister[(ns, name)]
        make_usage(r["usage"], pm.get("usage"))
        pms.append(r)
    return rec, pms
