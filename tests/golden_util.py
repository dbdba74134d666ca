"""Builds oracle/engine state from the transcribed golden fixtures (tests/golden/loadaware.json)."""
import json
import os

import numpy as np

from koordinator_amd import abi, config, objects

NOW = 1_700_000_000 * 10**9
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "loadaware.json")


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def build(case, engine_cls):
    """Instantiate engine_cls(cfg) (Oracle or Engine) with one node set up as the case describes."""
    la = config.loadaware_args(**case.get("args", {}))
    cfg = config.make_config(1, la=la)
    eng = engine_cls(cfg)
    eng.set_now(NOW)
    node = objects.make_node({**case["node"], "annotations": {"usage_thresholds": case["custom"]}}
                             if "custom" in case else case["node"])
    eng.upsert_nodes(np.array([node], abi.NODE_DTYPE))
    lister = {}
    for p in case.get("lister", []):
        lister[(p.get("namespace", "default"), p["name"])] = objects.priority_class(p)
    for a in case.get("assigned", []):
        lister[(a["pod"].get("namespace", "default"), a["pod"]["name"])] = objects.priority_class(a["pod"])
    pod_spec = case.get("pod") or {}
    if pod_spec.get("name"):
        lister[(pod_spec.get("namespace", "default"), pod_spec["name"])] = objects.priority_class(pod_spec)
    m, pms = objects.make_metric(case.get("metric"), NOW, lister)
    offs = np.array([0, len(pms)], np.uint32)
    eng.upsert_metrics(np.array([m], abi.METRIC_DTYPE), np.array(pms, abi.POD_METRIC_DTYPE) if pms else None,
                       offs if pms else None)
    if case.get("assigned"):
        pods = np.array([objects.make_pod(a["pod"]) for a in case["assigned"]], abi.POD_DTYPE)
        ts = np.array([NOW + int(round(a["ts_rel"] * 1e9)) for a in case["assigned"]], np.int64)
        eng.assign(np.zeros(len(pods), np.uint32), pods, ts)
    pod = objects.make_pod(pod_spec)
    return eng, pod
