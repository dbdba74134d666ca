"""Incremental snapshot-update throughput: how fast informer deltas reach the HBM
mirror. Each round mutates a random 1% of the C5 cluster's nodes — NodeInfo (requested / pod count, as an
Assume/Bind or a pod deletion changes it), their NodeMetric (fresh usage + update time) and the LoadAware assign cache
(one pod assigned per touched node) — through the C-ABI (gs_nodes_upsert, gs_node_metrics_upsert, gs_pods_assign),
then schedules one pod, which flushes the deltas (host re-derivation of every touched row + one pinned H2D copy + the
scatter kernel) before its eval pass. The delta cost is that round's time minus the same one-pod schedule with
nothing pending; rows/s = touched rows / delta cost. Needs an MI355X.

    python scripts/bench_delta.py [--nodes 100000] [--rounds 20] [--frac 0.01]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--frac", type=float, default=0.01)
    args = ap.parse_args()
    from koordinator_amd import abi, config, synth
    from koordinator_amd.engine import Engine
    c = synth.make_cluster(args.nodes, 4 * args.rounds + 64, config_id=5)
    synth.make_ext(c)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_LA_FIT)
    e = Engine(cfg)
    synth.load_into(e, c)
    ext_args = abi.GsExtArgs()
    abi.load().gs_ext_args_default(abi.C.byref(ext_args))
    synth.load_ext_into(e, c, ext_args)
    rng = np.random.default_rng(5)
    pods = c.pods
    seq = np.arange(len(pods), dtype=np.uint64)
    k = 0

    def one_pod():
        nonlocal k
        t0 = time.perf_counter()
        e.schedule(pods[k:k + 1], seq[k:k + 1])
        e.synchronize()
        k += 1
        return time.perf_counter() - t0

    for _ in range(5):
        one_pod()
    base = float(np.median([one_pod() for _ in range(args.rounds)]))
    e.reset_stats()
    n_touch = max(1, int(args.nodes * args.frac))
    rows, up_s, delta_s = [], [], []
    uid = 1 << 40
    for r in range(args.rounds):
        idx = np.sort(rng.choice(args.nodes, n_touch, replace=False)).astype(np.uint32)
        nodes = c.nodes[idx].copy()
        nodes["requested"][:, 0] = np.minimum(nodes["requested"][:, 0] + 500, nodes["allocatable"][:, 0])
        nodes["requested"][:, 1] = np.minimum(nodes["requested"][:, 1] + (1 << 30), nodes["allocatable"][:, 1])
        nodes["pod_count"] += 1
        m = c.metrics[idx].copy()
        m["node_usage"]["cpu_milli"] = (m["node_usage"]["cpu_milli"] * 0.9).astype(np.int64)
        m["update_time_ns"] = c.now_ns - 5 * 10**9
        ap_ = np.resize(c.pods, n_touch).copy()   # (the cluster's pending pods repeated, fresh uids)
        ap_["uid"] = np.arange(uid, uid + n_touch, dtype=np.uint64)
        uid += n_touch
        ts = np.full(n_touch, c.now_ns - 10**9, np.int64)
        t0 = time.perf_counter()
        e.upsert_nodes(nodes, idx=idx)
        e.upsert_metrics(m, idx=idx)
        e.assign(idx, ap_, ts)
        t1 = time.perf_counter()
        t_sched = one_pod()
        up_s.append(t1 - t0)
        delta_s.append(t1 - t0 + t_sched - base)
        rows.append(n_touch)
    st = e.stats()
    d = float(np.median(delta_s))
    out = {"metric": "incremental snapshot-update throughput (C5 cluster, LoadAware + Fit rows)",
           "nodes": args.nodes, "rows_per_round": n_touch, "rounds": args.rounds,
           "events_per_row": "gs_nodes_upsert + gs_node_metrics_upsert + gs_pods_assign (1 pod)",
           "host_upsert_ms_median": 1e3 * float(np.median(up_s)),
           "one_pod_schedule_ms_base": 1e3 * base, "delta_cost_ms_median": 1e3 * d,
           "rows_per_s": n_touch / d if d > 0 else None,
           "h2d_bytes_per_row": st["delta_bytes"] / max(1, st["delta_rows"]),
           "h2d_bytes_per_round": st["delta_bytes"] / max(1, args.rounds),
           "h2d_rows_total": st["delta_rows"],
           "note": "delta cost = host upserts + (one-pod schedule with the deltas pending - without): host row "
                   "re-derivation, pinned H2D copy of the rows and the scatter kernel"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
