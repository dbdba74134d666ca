"""Quota-gated scheduling throughput on one GPU: the C3 workload of bench.py (50k nodes, NodeNUMAResource
profile) with every pod charged to one of 200 ElasticQuotas (20 parents x 10 children, check-parent on), the
gate in front of gs_schedule (koordinator_amd.quota.schedule_with_quota), against the same pods ungated.
Prints one JSON line. Run: python scripts/bench_quota_gate.py [--steps 10]"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--pods-per-step", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()

    from koordinator_amd import abi, config, synth
    from koordinator_amd.engine import Engine
    from koordinator_amd.quota import ElasticQuotaPlugin, schedule_with_quota

    P, total = args.pods_per_step, (args.warmup + args.steps) * args.pods_per_step
    cluster = synth.make_cluster(args.nodes, total, config_id=2)
    synth.make_numa(cluster)
    cfg = config.make_config(args.nodes, enabled=abi.GS_ENABLE_ALL)
    cap_cpu = int(cluster.nodes["allocatable"][:, 0].sum())
    cap_mem = int(cluster.nodes["allocatable"][:, 1].sum())

    def forest():
        p = ElasticQuotaPlugin(resources=("cpu", "memory"), enable_check_parent_quota=True)
        p.update_cluster_total_resource({"cpu": cap_cpu, "memory": cap_mem})
        for t in range(20):
            p.on_quota_add(f"t{t}", max={"cpu": cap_cpu // 16, "memory": cap_mem // 16},
                           min={"cpu": cap_cpu // 40, "memory": cap_mem // 40})
            for k in range(10):
                # a few children are tight: their pods hit the quota and get rejected
                frac = 20_000 if k == 0 else 2_000
                p.on_quota_add(f"t{t}-{k}", parent=f"t{t}", max={"cpu": cap_cpu // frac, "memory": cap_mem // frac},
                               min={"cpu": cap_cpu // 800, "memory": cap_mem // 800}, allow_lent=k % 3 != 0)
        return p

    pods, seq = cluster.pods, np.arange(total, dtype=np.uint64)
    names = [f"t{(i * 7) % 20}-{(i * 13) % 10}" for i in range(total)]
    pq = [(names[i], {"cpu": int(pods["requests"][i, 0]), "memory": int(pods["requests"][i, 1])},
           bool(i % 4 == 0)) for i in range(total)]

    def run(gated: bool):
        eng = Engine(cfg)
        synth.load_into(eng, cluster)
        plugin = forest()
        for q, req, _ in pq:
            plugin.on_pod_add(q, req, assigned=False)
        plugin.refresh_runtime()
        calls = []

        class Counting:
            def schedule(self, p, s):
                calls.append(len(p))
                return eng.schedule(p, s)

        def step(s):
            sl = slice(s * P, (s + 1) * P)
            if gated:
                out, st = schedule_with_quota(Counting(), plugin, pods[sl], pq[sl], seq[sl])
                return out, sum(x.code != "Success" for x in st)
            return eng.schedule(pods[sl], seq[sl]), 0

        for w in range(args.warmup):
            step(w)
        eng.synchronize()
        calls.clear()
        t0 = time.perf_counter()
        placed = rejected = 0
        for s in range(args.warmup, args.warmup + args.steps):
            out, r = step(s)
            placed += int((out["node"] >= 0).sum())
            rejected += r
        eng.synchronize()
        dt = time.perf_counter() - t0
        eng.close()
        return {"pods_per_s": args.steps * P / dt, "placed_per_s": placed / dt, "placed": placed, "quota_rejected": rejected,
                "engine_calls": len(calls), "mean_engine_batch": float(np.mean(calls)) if calls else None}

    ungated = run(False)
    gated = run(True)
    print(json.dumps({"workload": f"C3 {args.nodes} nodes x {args.steps * P} pods, 200 ElasticQuotas (20x10), "
                                  f"check-parent, 25% non-preemptible", "ungated": ungated, "gated": gated,
                      "note": "pods_per_s counts every decided pod (quota-rejected pods do no node work)"}))


if __name__ == "__main__":
    main()
