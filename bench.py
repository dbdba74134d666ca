"""Benchmark of the koord-scheduler Filter/Score hot path on MI355X (BASELINE.json metric).

A step = one pass of the hot path over one batch of synthetic pending pods: the scheduleOne loop
(NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource Filter over every node, their Scores, selectHost,
assume + Reserve incl. NUMA allocation and cpuset selection) for `--pods-per-step` pods, sequentially, against
the 50k-node synthetic C3 cluster (weak scaling: 50k nodes per GPU, node-sharded, RCCL all-gather of per-shard
candidate lists per batch). `--profile la-fit` drops NodeNUMAResource (the C2 plugin set).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Prints ONE JSON line on rank 0 (value = whole-job pod x node evaluations per second).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "pod×node Filter+Score evals/sec + pods/sec at 50k nodes, 1/2/4/8 GPUs"
HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def cpu_baseline(cluster, cfg, sample_pods: int, threads: int) -> dict:
    """The CPU restatement of the reference Go path (oracle, kind "port") on a bounded sample."""
    from oracle import oracle as orc
    o = orc.Oracle(cfg)
    from koordinator_amd import synth
    synth.load_into(o, cluster)
    pods = cluster.pods[:sample_pods]
    t0 = time.perf_counter()
    o.schedule(pods, nthreads=threads)
    dt = time.perf_counter() - t0
    return {"evals_per_s": sample_pods * cluster.num_nodes / dt, "pods_per_s": sample_pods / dt, "seconds": dt}


PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")


def pmc_traffic() -> tuple[float | None, str | None]:
    """HBM bytes per eval pass from the committed rocprofv3 PMC summary (scripts/gpu_profile.sh ->
    scripts/pmc_summary.py): counters cannot be read from inside this process, so the figure is the one measured
    by the separate --pmc passes over this same bench command."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        return float(d["eval_pass"]["hbm_bytes_per_launch"]), os.path.relpath(PMC_FILE, ROOT)
    except (OSError, KeyError, ValueError):
        return None, None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nodes-per-gpu", type=int, default=50_000)
    ap.add_argument("--pods-per-step", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--cpu-sample-pods", type=int, default=400)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile", choices=["c3", "la-fit"], default="c3")
    ap.add_argument("--sample-pct", type=int, default=None,
                    help="node sampling (percentageOfNodesToScore; 0 = adaptive) instead of every node (one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("run N>1 under torch.distributed.run (one process per GPU)")
    import torch
    import torch.distributed as dist
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs an MI355X (no GPU visible)")
    torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from koordinator_amd import config, synth
    from koordinator_amd.engine import Engine, unique_id

    n_nodes = args.nodes_per_gpu * world
    total_pods = (args.warmup + args.steps) * args.pods_per_step
    cluster = synth.make_cluster(n_nodes, total_pods, config_id=2)
    numa = args.profile == "c3"
    if numa:
        synth.make_numa(cluster)
    from koordinator_amd import abi
    if args.sample_pct is not None and world > 1:
        raise SystemExit("--sample-pct runs on one GPU")
    cfg = config.make_config(n_nodes, device=local_rank, batch_size=args.batch,
                             enabled=abi.GS_ENABLE_ALL if numa else abi.GS_ENABLE_LA_FIT,
                             percentage_of_nodes_to_score=args.sample_pct)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16")), 16)
        r16 = cpu_baseline(cluster, cfg, args.cpu_sample_pods, threads)
        r1 = cpu_baseline(cluster, cfg, max(20, args.cpu_sample_pods // 8), 1)
        nall = len(os.sched_getaffinity(0)) or 1
        rall = cpu_baseline(cluster, cfg, args.cpu_sample_pods, nall) if nall > threads else r16
        cpu = {"value": r16["evals_per_s"], "unit": "evals/s", "cores": threads, "kind": "port",
               "sample": f"first {args.cpu_sample_pods} pods of the same {n_nodes}-node cluster, sequential "
                         f"scheduleOne with Filter/Score fanned out over {threads} threads "
                         f"(parallelize.Until emulation, parallelism={threads}); CPU restatement of the "
                         f"reference Go path (oracle/), not the Go binary",
               "pods_per_s": r16["pods_per_s"], "seconds": r16["seconds"],
               "single_thread_evals_per_s": r1["evals_per_s"],
               "all_cores": {"threads": nall, "evals_per_s": rall["evals_per_s"], "pods_per_s": rall["pods_per_s"]}}

    eng = Engine(cfg)
    if world > 1:
        uid = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init_rccl(uid[0], world, rank)
    synth.load_into(eng, cluster)

    pods = cluster.pods
    seq = np.arange(total_pods, dtype=np.uint64)
    P = args.pods_per_step
    for w in range(args.warmup):
        eng.schedule(pods[w * P:(w + 1) * P], seq[w * P:(w + 1) * P])
    eng.synchronize()
    eng.reset_stats()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    placed = 0
    for s in range(args.warmup, args.warmup + args.steps):
        out = eng.schedule(pods[s * P:(s + 1) * P], seq[s * P:(s + 1) * P])
        placed += int((out["node"] >= 0).sum())
    eng.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    st = eng.stats()
    pods_timed = args.steps * P
    evals = pods_timed * n_nodes
    value = evals / dt
    launches = max(1, st["eval_launches"])
    avg_launch_ms = st["eval_ms"] / launches
    pairs_per_launch = st["eval_pairs"] / launches
    bytes_per_launch = pairs_per_launch * st["node_row_bytes"]
    achieved = bytes_per_launch / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    traffic, traffic_src = pmc_traffic() if numa else (None, None)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "pods_per_s": pods_timed / dt,
            "config": {
                "workload": (f"C3: {n_nodes} nodes ({args.nodes_per_gpu}/GPU) x {P} pods/step, sequential scheduleOne "
                             "with NodeResourcesFit(LeastAllocated) + LoadAwareScheduling + NodeNUMAResource filter+"
                             "score (30% NUMA-policy nodes, 20% LSE/LSR cpuset pods), selectHost, assume+Reserve"
                             if numa else
                             f"C2 plugin set at C3 scale: {n_nodes} nodes ({args.nodes_per_gpu}/GPU) x {P} pods/step, "
                             "NodeResourcesFit(LeastAllocated)+LoadAwareScheduling filter+score, selectHost, "
                             "assume+Reserve"),
                "nodes": n_nodes, "pods_per_step": P, "batch": args.batch, "parallelism": f"node-shard x{world}",
                "level_list_cap": 2048,
                "node_sampling": None if args.sample_pct is None else {
                    "percentage_of_nodes_to_score": args.sample_pct,
                    "num_feasible_nodes_to_find": int(abi.load().gs_num_feasible_nodes_to_find(n_nodes, args.sample_pct)),
                    "note": "findNodesThatPassFilters rotation window (parallelism-1 order); every node is still "
                            "evaluated by the eval pass, value counts pods x nodes"},
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_unit": "bytes per eval pass (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction)",
                "traffic_source": traffic_src,
                "kernel": "eval pass = eval_kernel + eval_numa_kernel (one launch each per batch)",
                "bytes_per_eval": st["node_row_bytes"],
                "avg_launch_us": avg_launch_ms * 1e3,
                "pairs_per_launch": pairs_per_launch,
                "note": f"algorithmic bytes = {st['node_row_bytes']} B node row per pod x node eval (un-batched "
                        "convention); eval_kernel reads each row once per group of 16 pods (eval_numa_kernel: "
                        "once per 2 pods), so frac > 1 would mean reuse; avg_launch_us is the HIP-event time of the "
                        "pass on the library stream",
            },
            "breakdown_ms": {"eval": st["eval_ms"], "cand": st["cand_ms"], "commit": st["commit_ms"],
                             "exchange": st["exchange_ms"], "batches": st["batches"], "cuts": st["cuts"],
                             "slowpath_pods": st["slowpath_pods"]},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
