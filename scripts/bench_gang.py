"""Coscheduling throughput on the GPU engine: the C3 bench cluster (50k nodes, NUMA profile) and a queue
in which a share of the pods belong to Strict gangs (PodGroups of `--gang-size` pods, minMember = size), scheduled by
koordinator_amd.gang.schedule_with_gangs (speculative engine runs + gang replay) in 2048-pod calls, against the same
queue without gangs through Engine.schedule. Prints one JSON line. Needs an MI355X.

    python scripts/bench_gang.py [--nodes 50000] [--pods 20480] [--gang-pct 25] [--gang-size 8]
"""
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
    ap.add_argument("--pods", type=int, default=20_480)
    ap.add_argument("--gang-pct", type=int, default=25)
    ap.add_argument("--gang-size", type=int, default=8)
    ap.add_argument("--chunk", type=int, default=2048)
    ap.add_argument("--run-cap", type=int, default=192, help="schedule_with_gangs run_cap (pods per engine call)")
    args = ap.parse_args()
    from koordinator_amd import abi, config, synth
    from koordinator_amd import gang as gg
    from koordinator_amd.engine import Engine

    warm = args.chunk
    total = warm + args.pods
    c = synth.make_cluster(args.nodes, total, config_id=2)
    synth.make_numa(c)
    cfg = config.make_config(args.nodes, batch_size=128, enabled=abi.GS_ENABLE_ALL)
    rng = np.random.default_rng(7)
    gang_ids = np.zeros(total, np.uint64)
    n_g, k = 0, warm
    g = args.gang_pct / 100.0
    p_start = g / (args.gang_size * (1 - g) + g)   # a gang starts here: ~gang_pct% of the pods end up in gangs
    while k + args.gang_size <= total:
        if rng.random() < p_start:
            n_g += 1
            gang_ids[k:k + args.gang_size] = n_g
            k += args.gang_size
        else:
            k += 1
    seq = np.arange(total, dtype=np.uint64)
    pods = c.pods

    def engine():
        e = Engine(cfg)
        synth.load_into(e, c)
        e.schedule(pods[:warm], seq[:warm])   # warm-up: same state for both runs
        e.synchronize()
        return e

    # plain: the same queue, no gang gates
    e = engine()
    t0 = time.perf_counter()
    for lo in range(warm, total, args.chunk):
        e.schedule(pods[lo:lo + args.chunk], seq[lo:lo + args.chunk])
    e.synchronize()
    plain_s = time.perf_counter() - t0
    del e

    e = engine()
    mgr = gg.GangManager()
    for g in range(1, n_g + 1):
        mgr.podgroup_upsert(gg.spec(g, args.gang_size, mode=gg.STRICT, wait_time_ns=60 * 10**9))
    for i in range(warm, total):
        if gang_ids[i]:
            mgr.pod_add(int(gang_ids[i]), int(pods["uid"][i]))
    states, carried, waiting = [], {}, gg.WaitingPods()
    calls = {"schedule": 0, "schedule_s": 0.0, "forget": 0, "forget_s": 0.0, "run_pods": []}
    sched, forget = e.schedule, e.forget

    def timed_schedule(p, q):
        t = time.perf_counter()
        r = sched(p, q)
        calls["schedule"] += 1
        calls["schedule_s"] += time.perf_counter() - t
        calls["run_pods"].append(len(p))
        return r

    def counted_forget(nodes, p):
        calls["forget"] += 1
        t = time.perf_counter()
        r = forget(nodes, p)
        calls["forget_s"] += time.perf_counter() - t
        return r

    e.schedule, e.forget = timed_schedule, counted_forget
    t0 = time.perf_counter()
    for lo in range(warm, total, args.chunk):
        hi = min(total, lo + args.chunk)
        _, res = gg.schedule_with_gangs(e, mgr, pods[lo:hi], gang_ids[lo:hi], seq[lo:hi], waiting=waiting,
                                        run_cap=args.run_cap)
        states.append(res["state"])
        carried.update(res["carried"])
    e.synchronize()
    gang_s = time.perf_counter() - t0
    st = np.concatenate(states)
    idx = {int(u): k - warm for k, u in enumerate(pods["uid"]) if k >= warm}
    for uid, s_new in carried.items():   # later calls' verdicts on pods left waiting by earlier calls
        st[idx[uid]] = s_new
    n = total - warm
    gang_pods = int(np.count_nonzero(gang_ids[warm:]))
    print(json.dumps({
        "metric": "decided pods/s with Coscheduling gates (schedule_with_gangs)", "nodes": args.nodes, "pods": n,
        "gangs": n_g, "gang_size": args.gang_size, "gang_pods": gang_pods,
        "pods_per_s": n / gang_s, "plain_pods_per_s": n / plain_s,
        "bound": int(np.count_nonzero(st == gg.ST_BOUND)), "waiting": int(np.count_nonzero(st == gg.ST_WAITING)),
        "rejected": int(np.count_nonzero(st == gg.ST_REJECTED)),
        "unschedulable": int(np.count_nonzero(st == gg.ST_UNSCHEDULABLE)),
        "engine_calls": calls["schedule"], "engine_s": calls["schedule_s"], "forget_calls": calls["forget"],
        "forget_s": calls["forget_s"], "run_pods_mean": float(np.mean(calls["run_pods"])) if calls["run_pods"] else 0.0,
        "run_pods_single": int(sum(1 for x in calls["run_pods"] if x == 1)),
        "total_s": gang_s,
        "config": "C3 (NUMA profile), 2048-pod calls after one 2048-pod warm-up call, batch 128, gangs Strict with "
                  "minMember = gang size, PodGroups known up front; one GPU"}))


if __name__ == "__main__":
    main()
