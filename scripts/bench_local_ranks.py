"""Multi-rank rehearsal on ONE GPU over the in-process device transport (gs_comm_init_local): N ranks as threads of
this process, each an Engine over its node shard of the C3 bench cluster, the level all-gathers stream-ordered on the
device (as ncclAllGather runs them; score rows by default, GS_XCHG=levels the candidate level lists), every rank
scheduling the same queue in 2048-pod steps. Prints one JSON line:
the wall-clock pods/s of the slowest rank and, per rank, the batch chain's parts (eval pass, levels + exchange,
commit). All N ranks share the box's one GPU, so this is not a scaling point: it measures what the sharded flow
costs per batch — the merged-list commit against one rank's commit. N = 1 runs the single-rank path
(no group).

    python scripts/bench_local_ranks.py [--ranks 2] [--nodes 50000] [--steps 10] [--warmup 2]
"""
import argparse
import hashlib
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=50_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods-per-step", type=int, default=2048)
    ap.add_argument("--sync", action="store_true", help="blocking gs_schedule per step (default: submit one ahead)")
    args = ap.parse_args()
    from koordinator_amd import abi, config, synth
    from koordinator_amd.engine import Engine, LocalGroup

    n = args.ranks
    P = args.pods_per_step
    total = (args.warmup + args.steps) * P
    c = synth.make_cluster(args.nodes, total, config_id=2)
    synth.make_numa(c)
    cfg = config.make_config(args.nodes, batch_size=128, enabled=abi.GS_ENABLE_ALL)
    g = LocalGroup(n) if n > 1 else None
    engines = [Engine(cfg) for _ in range(n)]
    for r, e in enumerate(engines):
        if g is not None:
            e.comm_init_local(g, r)
        synth.load_into(e, c)
    seq = np.arange(total, dtype=np.uint64)
    bar = threading.Barrier(n)
    res = [None] * n

    def run(r):
        e = engines[r]
        try:
            for w in range(args.warmup):
                e.schedule(c.pods[w * P:(w + 1) * P], seq[w * P:(w + 1) * P])
            e.synchronize()
            e.reset_stats()
            bar.wait()
            t0 = time.perf_counter()
            outs = []
            s0, s1 = args.warmup, args.warmup + args.steps
            if args.sync:
                for s in range(s0, s1):
                    outs.append(e.schedule(c.pods[s * P:(s + 1) * P], seq[s * P:(s + 1) * P])["node"].copy())
            else:   # each step submitted before the previous one is waited for, as bench.py does
                h = e.schedule_submit(c.pods[s0 * P:(s0 + 1) * P], seq[s0 * P:(s0 + 1) * P])
                for s in range(s0 + 1, s1 + 1):
                    h2 = e.schedule_submit(c.pods[s * P:(s + 1) * P], seq[s * P:(s + 1) * P]) if s < s1 else None
                    outs.append(e.schedule_wait(h)["node"].copy())
                    h = h2
            placed = sum(int((o >= 0).sum()) for o in outs)
            e.synchronize()
            res[r] = (time.perf_counter() - t0, placed, e.stats(), np.concatenate(outs))
        except Exception as ex:   # noqa: BLE001
            res[r] = ex
            bar.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for r in range(n):
        if isinstance(res[r], Exception):
            raise SystemExit(f"rank {r}: {res[r]}")
    same = all(np.array_equal(res[0][3], res[r][3]) for r in range(n))
    dt = max(x[0] for x in res)
    per = []
    for r in range(n):
        st = res[r][2]
        b = max(1, st["batches"])
        per.append({"rank": r, "wall_s": round(res[r][0], 4), "batches": st["batches"],
                    "eval_ms_per_batch": round(st["eval_ms"] / b, 4), "levels_ms_per_batch": round(st["cand_ms"] / b, 4),
                    "commit_ms_per_batch": round(st["commit_ms"] / b, 4),
                    "exchange_ms_per_batch": round(st["exchange_ms"] / b, 4)})
    print(json.dumps({"metric": "pods/s, N ranks as threads on one GPU (device transport)", "ranks": n,
                      "exchange": (os.environ.get("GS_XCHG") or "scores") if n > 1 else None,
                      "nodes": args.nodes, "pods": args.steps * P, "pods_per_s": args.steps * P / dt,
                      "placed": res[0][1], "identical_placements_on_every_rank": bool(same),
                      "placements_sha1": hashlib.sha1(res[0][3].tobytes()).hexdigest()[:16], "per_rank": per,
                      "config": "C3 (NUMA profile), 2048-pod steps (" + ("blocking gs_schedule" if args.sync else
                                "gs_schedule_submit one ahead") + "), batch 128; every rank on the box's one GPU",
                      "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES")}))


if __name__ == "__main__":
    main()
