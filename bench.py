"""Benchmark of the koord-scheduler Filter/Score hot path on MI355X (BASELINE.json metric).

A step = one pass of the hot path over one batch of synthetic pending pods: the scheduleOne loop
(NodeResourcesFit + LoadAwareScheduling + NodeNUMAResource Filter over every node, their Scores, selectHost,
assume + Reserve incl. NUMA allocation and cpuset selection) for `--pods-per-step` pods, sequentially, against
the 50k-node synthetic C3 cluster. Several GPUs: strong scaling by default (the metric's 50k nodes in total,
node-sharded, RCCL all-gather of each shard's score rows per batch, the one-GPU commit replicated on every rank);
`--scaling weak`
gives every GPU 50k nodes. `--profile la-fit` drops NodeNUMAResource (the C2 plugin set).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
    (rehearsal of the sharded flow on a one-GPU box: N processes on device 0, all-gather over gloo through the
     library's host-callback transport: ... bench.py --gpus N --transport gloo --share-gpu)

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


def cpu_baseline(cluster, cfg, pods, seq, given, sample_start: int, sample_pods: int, threads: int) -> dict:
    """The CPU restatement of the reference Go path (oracle, kind "port") on the state the GPU's timed region started
    from: the oracle replays the GPU's placements of pods [0, sample_start) (the warm-up steps), then runs the full
    scheduleOne on the next pods — an untimed warm-up chunk, then 5 timed chunks (median pods/s) with Filter / Score /
    selectHost / Reserve timed separately, then a single-thread chunk."""
    from oracle import oracle as orc
    from koordinator_amd import synth
    o = orc.Oracle(cfg)
    synth.load_into(o, cluster)
    if sample_start:
        o.schedule_replay(pods[:sample_start], given[:sample_start], seq[:sample_start], nthreads=threads)
    i = sample_start
    warm = max(8, sample_pods // 10)
    o.schedule(pods[i:i + warm], seq[i:i + warm], nthreads=threads)
    i += warm
    o.phase_times()
    # the timed pods one scheduleOne at a time (the reference's loop), their times grouped into 5 chunks by a
    # stratified random draw: the pods are split by kind (QoS x priority class, required / preferred CPU bind policy,
    # exclusive policy, whole CPUs requested: a cpuset-bound LSE / LSR pod's Filter runs takeCPUs on every node whose
    # bind policy is required and costs ~20 plain pods, with a spread set by those attributes), each kind in a fixed
    # random order dealt round-robin over the chunks, so every chunk holds the same mix and its rate differs from the
    # others by the cost spread within a kind only (plain random chunks of 198 pods spread ±15-26%)
    n_t = max(5, sample_pods - warm)
    per = np.zeros(n_t)
    for j in range(n_t):
        t0 = time.perf_counter()
        o.schedule(pods[i + j:i + j + 1], seq[i + j:i + j + 1], nthreads=threads)
        per[j] = time.perf_counter() - t0
    tp = pods[i:i + n_t]
    i += n_t
    kind = ((tp["qos_class"].astype(np.int64) * 16 + tp["priority_class"]) * 1000 +
            tp["required_cpu_bind_policy"].astype(np.int64) * 100 + tp["preferred_cpu_bind_policy"] * 10 +
            tp["preferred_cpu_exclusive_policy"]) * 100 + tp["requests"][:, 0] // 1000
    rng = np.random.default_rng(20260)
    chunk_of = np.empty(n_t, np.int64)
    dealt = 0
    for k in np.unique(kind):
        idx = rng.permutation(np.nonzero(kind == k)[0])
        chunk_of[idx] = (dealt + np.arange(len(idx))) % 5
        dealt += len(idx)
    chunk = n_t // 5
    rates = [float((chunk_of == c).sum() / per[chunk_of == c].sum()) for c in range(5)]
    secs = float(per.sum())
    phases = o.phase_times()
    n1 = max(4, chunk // 8)
    t0 = time.perf_counter()
    o.schedule(pods[i:i + n1], seq[i:i + n1], nthreads=1)
    r1 = n1 / (time.perf_counter() - t0)
    pods_per_s = float(np.median(rates))
    return {"pods_per_s": pods_per_s, "evals_per_s": pods_per_s * cluster.num_nodes, "seconds": secs,
            "chunks": 5, "chunk_pods": chunk, "chunk_pods_per_s": rates,
            "chunk_spread": (max(rates) - min(rates)) / (2 * pods_per_s), "all_pods_per_s": float(n_t / secs),
            "phase_share": {k: v / max(secs, 1e-12) for k, v in phases.items()},
            "single_thread_pods_per_s": r1, "single_thread_evals_per_s": r1 * cluster.num_nodes,
            "sample": f"pods {sample_start}..{i + n1} of the timed workload on the GPU's state at the start of the timed "
                      f"region (oracle replay of the {sample_start} warm-up placements); {warm} warm-up pods, {n_t} timed "
                      f"pods at {threads} threads one scheduleOne at a time, rates of 5 chunks of ~{chunk} pods drawn "
                      f"at random within each pod kind (QoS x priority class, CPU bind / exclusive policies, CPUs; equal "
                      f"kind mix per chunk; median), {n1} "
                      f"pods at 1 thread"}


def cpu_baseline_c5(cluster, cfg, ext_args, pods, seq, sample_pods: int) -> dict:
    """C5: the oracle's one-thread scheduleOne with the Reservation / DeviceShare restatement (or_schedule_ext) on the
    first pods of the workload from the fresh cluster state (the ext restatement has no replay mode)."""
    from oracle import oracle as orc
    from koordinator_amd import synth
    o = orc.Oracle(cfg)
    synth.load_into(o, cluster)
    synth.load_ext_into(o, cluster, ext_args)
    n = max(8, sample_pods)
    t0 = time.perf_counter()
    out = o.schedule_ext(pods[:n], cluster.ext["pod_ext"][:n], seq[:n])[0]
    dt = time.perf_counter() - t0
    return {"pods_per_s": n / dt, "evals_per_s": n / dt * cluster.num_nodes, "seconds": dt, "placements": out,
            "sample": f"pods 0..{n} of the workload on the fresh cluster, one thread (or_schedule_ext: Fit + LoadAware + "
                      "DeviceShare + Reservation restatement)"}


class _ThreadedOracle:
    """The oracle engine with its Filter / Score fan-out over `threads` host threads, for the gang sample's sequential
    reference order (schedule / forget as Engine has them)."""

    def __init__(self, o, threads: int):
        self.o, self.threads = o, threads

    def schedule(self, pods, seq=None):
        return self.o.schedule(pods, seq, nthreads=self.threads)

    def forget(self, nodes, pods):
        return self.o.forget(nodes, pods)


def cpu_gang_sample(cluster, cfg, warm: int, given, pods, seq, gang_ids, specs, sample: int, threads: int) -> dict:
    """The gang extra's CPU leg: the oracle replays the GPU's warm-up placements, then runs the reference's
    one-pod-at-a-time Coscheduling order (oracle/coscheduling.py schedule_sequential) over the first `sample` pods of the
    gang queue; returns its decisions and rate (the caller compares them with the GPU's)."""
    from oracle import oracle as orc
    from oracle import coscheduling as oc
    from koordinator_amd import synth
    o = orc.Oracle(cfg)
    synth.load_into(o, cluster)
    o.schedule_replay(pods[:warm], given[:warm], seq[:warm], nthreads=threads)
    om = oc.PodGroupManager()
    for sp in specs:
        om.podgroup_upsert(sp)
    for k in range(warm, len(gang_ids)):
        if gang_ids[k]:
            om.pod_add(int(gang_ids[k]), int(pods["uid"][k]))
    hi = warm + sample
    t0 = time.perf_counter()
    want, wres = oc.schedule_sequential(_ThreadedOracle(o, threads), om, pods[warm:hi], gang_ids[warm:hi], seq[warm:hi])
    return {"want": want, "wres": wres, "seconds": time.perf_counter() - t0}


def extra_c5(P: int, steps: int, nodes: int, sample: int) -> dict:
    """C5 beside the headline: 100k nodes, LoadAware + Fit + DeviceShare + Reservation, one warm-up step
    and `steps` timed steps of P pods through gs_schedule_ext; the first `sample` pods (warm-up step) checked against
    the oracle's restatement from the same fresh cluster, which is also the CPU line."""
    import torch
    from koordinator_amd import abi, config, synth
    from koordinator_amd.engine import Engine
    total = (1 + steps) * P
    c = synth.make_cluster(nodes, total, config_id=5)
    synth.make_ext(c)
    cfg = config.make_config(nodes, device=0, batch_size=128, enabled=abi.GS_ENABLE_LA_FIT)
    eng = Engine(cfg)
    synth.load_into(eng, c)
    ea = abi.GsExtArgs()
    abi.load().gs_ext_args_default(abi.C.byref(ea))
    synth.load_ext_into(eng, c, ea)
    pods, ext = c.pods, c.ext["pod_ext"]
    seq = np.arange(total, dtype=np.uint64)
    first = eng.schedule_ext(pods[:P], ext[:P], seq[:P])[0]
    eng.synchronize()
    eng.reset_stats()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    placed = 0
    for s in range(1, 1 + steps):
        out = eng.schedule_ext(pods[s * P:(s + 1) * P], ext[s * P:(s + 1) * P], seq[s * P:(s + 1) * P])[0]
        placed += int((out["node"] >= 0).sum())
    eng.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    st = eng.stats()
    del eng
    r = cpu_baseline_c5(c, cfg, ea, pods, seq, sample)
    want = r.pop("placements")
    bad = [f for f in ("node", "score", "ties", "feasible") if not np.array_equal(first[f][:sample], want[f][:sample])]
    return {"pods_per_s": steps * P / dt, "evals_per_s": steps * P * nodes / dt, "steps": steps, "pods_per_step": P,
            "nodes": nodes, "ms_per_step": dt / steps * 1e3, "placed": placed,
            "batches": st["batches"], "workload": "C5: Fit(LeastAllocated) + LoadAware + DeviceShare (GPU) + Reservation "
                                                  "filter+score with normalize, selectHost, assume+Reserve; 20% GPU "
                                                  "nodes, 5% nodes with reservations, ~10% owner pods, ~10% GPU pods; "
                                                  "blocking gs_schedule_ext per step",
            "parity_sample": {"pods": sample, "fields": ["node", "score", "ties", "feasible"], "mismatched_fields": bad,
                              "ok": not bad, "what": "the first pods of the untimed warm-up step against the oracle's "
                                                     "sequential restatement (or_schedule_ext) from the same cluster"},
            "cpu_baseline": {"value": r["evals_per_s"], "unit": "evals/s", "cores": 1, "kind": "port",
                             "pods_per_s": r["pods_per_s"], "seconds": r["seconds"], "sample": r["sample"]}}


def extra_gang(cluster, cfg, P: int, calls: int, sample: int, threads: int, gang_pct: int = 25, gang_size: int = 8,
               run_cap: int = 192) -> dict:
    """Coscheduling beside the headline: the headline's C3 cluster from a fresh engine, one 2048-pod
    warm-up call, then `calls` calls of P pods of which ~gang_pct% are in Strict gangs of gang_size
    (koordinator_amd.gang.schedule_with_gangs: speculative engine runs + gang replay); the first `sample` pods of the gang
    queue checked against the reference's one-pod-at-a-time order on the oracle (gang PreFilter codes; node, score, ties,
    feasible of the pods that reached the node loop)."""
    import torch
    from koordinator_amd import gang as gg, synth
    from koordinator_amd.engine import Engine
    warm = P
    total = warm + calls * P
    pods = cluster.pods[:total]
    seq = np.arange(total, dtype=np.uint64)
    rng = np.random.default_rng(7)
    gang_ids = np.zeros(total, np.uint64)
    n_g, k = 0, warm
    g = gang_pct / 100.0
    p_start = g / (gang_size * (1 - g) + g)
    while k + gang_size <= total:
        if rng.random() < p_start:
            n_g += 1
            gang_ids[k:k + gang_size] = n_g
            k += gang_size
        else:
            k += 1
    specs = [dict(gang_id=j, min_member=gang_size, mode=gg.STRICT, wait_time_ns=60 * 10**9) for j in range(1, n_g + 1)]
    e = Engine(cfg)
    synth.load_into(e, cluster)
    wout = e.schedule(pods[:warm], seq[:warm])
    given = np.where(wout["node"] >= 0, wout["node"], -2).astype(np.int32)
    mgr = gg.GangManager()
    for sp in specs:
        mgr.podgroup_upsert(gg.spec(**sp))
    for j in range(warm, total):
        if gang_ids[j]:
            mgr.pod_add(int(gang_ids[j]), int(pods["uid"][j]))
    e.synchronize()
    torch.cuda.synchronize()
    waiting = gg.WaitingPods()
    states, carried, first = [], {}, None
    t0 = time.perf_counter()
    for lo in range(warm, total, P):
        hi = min(total, lo + P)
        out, res = gg.schedule_with_gangs(e, mgr, pods[lo:hi], gang_ids[lo:hi], seq[lo:hi], waiting=waiting,
                                          run_cap=run_cap)
        if first is None:
            first = (out, res)
        states.append(res["state"])
        carried.update(res["carried"])
    e.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del e
    st = np.concatenate(states)
    idx = {int(u): j - warm for j, u in enumerate(pods["uid"]) if j >= warm}
    for uid, s_new in carried.items():
        st[idx[uid]] = s_new
    r = cpu_gang_sample(cluster, cfg, warm, given, pods, seq, gang_ids, specs, sample, threads)
    want, wres = r["want"], r["wres"]
    got, gres = first
    bad = []
    if not np.array_equal(np.asarray(gres["prefilter"])[:sample], np.asarray(wres["prefilter"])):
        bad.append("prefilter")
    ran = want["node"] >= 0
    for f in ("node", "score", "ties", "feasible"):
        if not np.array_equal(got[f][:sample][ran], want[f][ran]):
            bad.append(f)
    n = total - warm
    return {"pods_per_s": n / dt, "pods": n, "calls": calls, "pods_per_call": P, "nodes": cluster.num_nodes,
            "seconds": dt, "gangs": n_g, "gang_size": gang_size, "gang_pods": int(np.count_nonzero(gang_ids[warm:])),
            "bound": int(np.count_nonzero(st == gg.ST_BOUND)), "waiting": int(np.count_nonzero(st == gg.ST_WAITING)),
            "rejected": int(np.count_nonzero(st == gg.ST_REJECTED)),
            "unschedulable": int(np.count_nonzero(st == gg.ST_UNSCHEDULABLE)),
            "workload": "C3 (NUMA profile) with Coscheduling: Strict gangs (minMember = size, PodGroups known up front), "
                        f"schedule_with_gangs run cap {run_cap}; decided pods/s",
            "parity_sample": {"pods": sample, "ran_node_loop": int(ran.sum()), "mismatched_fields": bad, "ok": not bad,
                              "what": "the first pods of the gang queue against oracle/coscheduling.py's one-pod-at-a-time "
                                      "order on the oracle engine after replaying the same warm-up placements"},
            "cpu_baseline": {"pods_per_s": sample / r["seconds"], "cores": threads, "kind": "port",
                             "seconds": r["seconds"], "sample": f"{sample} pods, one scheduleOne at a time with the gang "
                                                                 f"gates, Filter/Score over {threads} threads"}}


def host_cpus() -> dict:
    """The host CPUs the CPU baseline runs on: logical CPUs of the machine (nproc), the ones this process may run on
    (affinity), the cgroup CPU quota (a box's share of the machine), and the CPU model."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": None,
            "model": None}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                info["cgroup_quota_cpus"] = int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = info["affinity"]
    if info["cgroup_quota_cpus"]:
        usable = min(usable, max(1, int(info["cgroup_quota_cpus"])))
    info["usable"] = usable
    return info


PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")


def pmc_summary() -> tuple[dict | None, str | None]:
    """Per-kernel HBM bytes per launch from the committed rocprofv3 PMC summary (scripts/gpu_profile.sh ->
    scripts/pmc_summary.py; separate --pmc FETCH_SIZE / WRITE_SIZE passes over a 1-step run of this bench): counters
    cannot be read from inside this process."""
    try:
        with open(PMC_FILE) as f:
            return json.load(f), os.path.relpath(PMC_FILE, ROOT)
    except (OSError, ValueError):
        return None, None


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--nodes", type=int, default=50_000,
                    help="cluster nodes (strong scaling: in total, the metric's 50k; weak: per GPU)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--pods-per-step", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--cpu-sample-pods", type=int, default=2200)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile", choices=["c3", "la-fit", "c5"], default="c3",
                    help="c5: 100k nodes, LoadAware + Fit + DeviceShare + Reservation (SURVEY 8(d) C5, see --nodes)")
    ap.add_argument("--sample-pct", type=int, default=None,
                    help="node sampling (percentageOfNodesToScore; 0 = adaptive) instead of every node (one GPU)")
    ap.add_argument("--transport", choices=["rccl", "gloo"], default="rccl",
                    help="several ranks: RCCL all-gather (production) or gloo through the host-callback transport")
    ap.add_argument("--share-gpu", action="store_true", help="every rank on device 0 (gloo rehearsal on one GPU)")
    ap.add_argument("--sync", action="store_true", help="one blocking gs_schedule per step (no submission ahead)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the C5 and Coscheduling sub-objects of the default (one-GPU, C3) line")
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
    gloo = world > 1 and args.transport == "gloo"
    if args.share_gpu and not gloo:
        raise SystemExit("--share-gpu needs --transport gloo (RCCL takes one GPU per rank)")
    device = 0 if args.share_gpu else local_rank
    torch.cuda.set_device(device)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if gloo:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from koordinator_amd import config, synth
    from koordinator_amd.engine import Engine, unique_id

    n_nodes = args.nodes if args.scaling == "strong" else args.nodes * world
    total_pods = (args.warmup + args.steps) * args.pods_per_step
    c5 = args.profile == "c5"
    if c5 and world > 1:
        raise SystemExit("--profile c5 runs on one GPU (the C5 bench is a one-GPU configuration)")
    cluster = synth.make_cluster(n_nodes, total_pods, config_id=5 if c5 else 2)
    numa = args.profile == "c3"
    if numa:
        synth.make_numa(cluster)
    if c5:
        synth.make_ext(cluster)
    from koordinator_amd import abi
    if args.sample_pct is not None and world > 1 and os.environ.get("GS_XCHG") == "levels":
        raise SystemExit("--sample-pct on several GPUs needs the score-row exchange")
    cfg = config.make_config(n_nodes, device=device, batch_size=args.batch,
                             enabled=abi.GS_ENABLE_ALL if numa else abi.GS_ENABLE_LA_FIT,
                             percentage_of_nodes_to_score=args.sample_pct)

    eng = Engine(cfg)
    if gloo:
        def allgather(data: bytes):
            t = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            out = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(out, t)
            return [x.numpy().tobytes() for x in out]
        eng.comm_init_callback(world, rank, allgather)
    elif world > 1:
        uid = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        eng.comm_init_rccl(uid[0], world, rank)
    synth.load_into(eng, cluster)
    ext_args = None
    if c5:
        ext_args = abi.GsExtArgs()
        abi.load().gs_ext_args_default(abi.C.byref(ext_args))
        synth.load_ext_into(eng, cluster, ext_args)
        pod_ext = cluster.ext["pod_ext"]

    def run(lo, hi):
        if c5:
            return eng.schedule_ext(pods[lo:hi], pod_ext[lo:hi], seq[lo:hi])[0]
        return eng.schedule(pods[lo:hi], seq[lo:hi])

    pods = cluster.pods
    seq = np.arange(total_pods, dtype=np.uint64)
    given = np.full(total_pods, -1, np.int32)   # the GPU's placements (the CPU baseline replays the warm-up ones)
    P = args.pods_per_step
    for w in range(args.warmup):
        out = run(w * P, (w + 1) * P)
        given[w * P:(w + 1) * P] = np.where(out["node"] >= 0, out["node"], -2)
    eng.synchronize()
    eng.reset_stats()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    placed = 0
    if args.sync or c5:
        for s in range(args.warmup, args.warmup + args.steps):
            out = run(s * P, (s + 1) * P)
            placed += int((out["node"] >= 0).sum())
    else:
        # each step's pods are submitted before the previous step is waited for (gs_schedule_submit): the batch
        # pipeline runs on across steps, as a scheduler draining its queue chunk by chunk
        s0 = args.warmup
        h = eng.schedule_submit(pods[s0 * P:(s0 + 1) * P], seq[s0 * P:(s0 + 1) * P])
        for s in range(s0 + 1, args.warmup + args.steps + 1):
            h2 = eng.schedule_submit(pods[s * P:(s + 1) * P], seq[s * P:(s + 1) * P]) if s < args.warmup + args.steps else None
            out = eng.schedule_wait(h)
            placed += int((out["node"] >= 0).sum())
            h = h2
    eng.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device="cpu" if gloo else "cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    st = eng.stats()
    pods_timed = args.steps * P
    evals = pods_timed * n_nodes
    value = evals / dt
    bpe = st["node_row_bytes"]
    # BASELINE.md §4 / SURVEY §8(d): roofline.achieved = evals/s over the timed steps x algorithmic bytes per eval
    achieved = value * bpe / 1e9
    batches = max(1, st["batches"])
    launches = max(1, st["eval_launches"])
    eval_us = st["eval_ms"] / launches * 1e3
    pairs_per_launch = st["eval_pairs"] / launches
    eval_achieved = pairs_per_launch * bpe / (eval_us * 1e-6) / 1e9 if eval_us > 0 else 0.0
    step_ms = dt / args.steps * 1e3
    pmc, pmc_src = pmc_summary() if numa else (None, None)
    kpmc = (pmc or {}).get("kernels", {})

    def pmc_bytes(prefix):
        ks = [k for k in kpmc if k.startswith(prefix)]
        return sum(kpmc[k]["hbm_bytes_per_launch"] for k in ks) if ks else None

    traffic_step = None
    # one-time setup kernels of the profiled run (the mirror upload, buffer fills): not per-step traffic
    setup = ("gs::scatter_rows_kernel", "gs::node_prep_kernel")
    if kpmc:
        # the profiled run's step count: commit_spec_kernel launches once per batch
        commit = next((v for k, v in kpmc.items() if k.startswith("gs::commit_spec_kernel<false")), {})
        steps_in_pmc = max(1.0, commit.get("dispatches", 0) / max(1.0, batches / args.steps))
        traffic_step = sum(v["hbm_bytes_per_launch"] * v["dispatches"] for k, v in kpmc.items()
                           if k.startswith("gs::") and not k.startswith(setup)) / steps_in_pmc
    kernels = {
        "eval_pass": {"kernels": "gather_numa_kernel -> eval_numa_tile_kernel (full batches) beside eval_kernel on a second "
                                 "stream, one launch each per batch",
                      "avg_launch_us": eval_us, "pairs_per_launch": pairs_per_launch,
                      "achieved_GBps": eval_achieved, "frac": eval_achieved / HBM_PEAK_GBPS,
                      "pmc_bytes_per_launch": (pmc_bytes("gs::eval") or 0) + (pmc_bytes("gs::gather_numa") or 0)
                      if pmc_bytes("gs::eval") else None,
                      "share_of_step": st["eval_ms"] / args.steps / step_ms},
        "patch_cand_interval": {"what": "from the eval pass's end (HIP event) to the commit kernel's start (the "
                                        "batch's end event minus the commit's own s_memrealtime duration): "
                                        "cand_kernel beside the previous batch's commit, the wait for that commit, "
                                        "then fix_levels_kernel (its landed rows re-evaluated and folded into the "
                                        "levels); the kernels' own durations are in the rocprof summary",
                                "critical_path": "only fix_levels_kernel (~32 us per batch in the kernel trace) and "
                                                 "its launch gap are on the commit chain; the rest of the interval "
                                                 "runs beside, or waits for, the previous batch's commit",
                                "avg_us": st["cand_ms"] / batches * 1e3,
                                "pmc_bytes_per_launch": (pmc_bytes("gs::cand") or 0) + (pmc_bytes("gs::fix_levels") or 0)
                                if (pmc_bytes("gs::cand") or pmc_bytes("gs::fix_levels")) else None,
                                "share_of_step": st["cand_ms"] / args.steps / step_ms},
        "commit_kernel": {"bound": "latency: one workgroup walks the batch's pods in order (selectHost, Reserve, "
                                   "re-scoring of the rows earlier pods landed on)",
                          "avg_launch_us": st["commit_ms"] / batches * 1e3,
                          "us_per_pod": st["commit_ms"] * 1e3 / max(1, st["pods"]),
                          "pmc_bytes_per_launch": pmc_bytes("gs::commit"),
                          "share_of_step": st["commit_ms"] / args.steps / step_ms},
    }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and c5:
        r = cpu_baseline_c5(cluster, cfg, ext_args, pods, seq, args.cpu_sample_pods // 4)
        r.pop("placements")
        cpu = {"value": r["evals_per_s"], "unit": "evals/s", "cores": 1, "kind": "port", "pods_per_s": r["pods_per_s"],
               "seconds": r["seconds"], "sample": r["sample"]}
    elif rank == 0 and world == 1 and not args.no_cpu_baseline:
        hc = host_cpus()
        threads = min(hc["usable"], 16)
        sample_start = args.warmup * P
        r = cpu_baseline(cluster, cfg, pods, seq, given, sample_start, args.cpu_sample_pods, threads)
        # run B: every usable host core; the same as run A when the box's CPU share is 16 or less
        rb = None
        if hc["usable"] > threads:
            rb = cpu_baseline(cluster, cfg, pods, seq, given, sample_start, args.cpu_sample_pods, hc["usable"])
        cpu = {"value": r["evals_per_s"], "unit": "evals/s", "cores": threads, "kind": "port", "host": hc,
               "all_cores": ({"cores": hc["usable"], "value": rb["evals_per_s"], "pods_per_s": rb["pods_per_s"],
                              "chunk_pods_per_s": rb["chunk_pods_per_s"]} if rb else
                             {"cores": threads, "note": f"all usable host cores = {hc['usable']} (affinity "
                                                        f"{hc['affinity']}, cgroup quota {hc['cgroup_quota_cpus']}): "
                                                        "run A is already every usable core"}),
               "sample": r["sample"] + f"; sequential scheduleOne with Filter/Score fanned out over {threads} threads "
                         "(parallelize.Until emulation, parallelism=16 = the reference default and this box's CPU "
                         "share); CPU restatement of the reference Go path (oracle/), not the Go binary",
               "pods_per_s": r["pods_per_s"], "seconds": r["seconds"], "chunk_pods_per_s": r["chunk_pods_per_s"],
               "chunk_spread": r["chunk_spread"], "all_pods_per_s": r["all_pods_per_s"],
               "phase_share": r["phase_share"], "single_thread_evals_per_s": r["single_thread_evals_per_s"],
               "single_thread_pods_per_s": r["single_thread_pods_per_s"]}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": step_ms,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "pods_per_s": pods_timed / dt,
            "config": {
                "workload": (f"C5: {n_nodes} nodes ({world} GPU) x {P} pods/step, NodeResourcesFit(LeastAllocated) + "
                             "LoadAwareScheduling + DeviceShare (GPU) + Reservation filter+score with normalize, selectHost, "
                             "assume+Reserve; 20% GPU nodes, 5% nodes with reservations, ~10% owner pods, ~10% GPU pods"
                             if c5 else
                             f"C3: {n_nodes} nodes ({args.scaling} scaling over {world} GPU) x {P} pods/step, "
                             "sequential scheduleOne with NodeResourcesFit(LeastAllocated) + LoadAwareScheduling + "
                             "NodeNUMAResource filter+score (30% NUMA-policy nodes, 20% LSE/LSR cpuset pods), "
                             "selectHost, assume+Reserve"
                             if numa else
                             f"C2 plugin set at C3 scale: {n_nodes} nodes ({args.scaling} scaling over {world} GPU) x "
                             f"{P} pods/step, NodeResourcesFit(LeastAllocated)+LoadAwareScheduling filter+score, "
                             "selectHost, assume+Reserve"),
                "nodes": n_nodes, "pods_per_step": P, "batch": args.batch,
                "submission": "blocking gs_schedule per step" if (args.sync or c5)
                              else "gs_schedule_submit one step ahead (the batch pipeline runs across steps)",
                "parallelism": f"node-shard x{world}" + ("" if world == 1 else
                               ", candidate levels all-gathered, merged-list commit on every rank"
                               if os.environ.get("GS_XCHG") == "levels" else
                               ", score rows all-gathered, the one-shard commit replicated on every rank") +
                               (" (gloo host-callback all-gather, every rank on one GPU: a rehearsal, not a scaling "
                                "point)" if args.share_gpu else ""),
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
                "traffic": traffic_step,
                "traffic_unit": "HBM bytes per step, the per-batch gs:: kernels (rocprofv3 PMC: 2 x FETCH_SIZE + "
                                "WRITE_SIZE, gfx950 correction; one-time mirror upload / node_prep excluded; steps = "
                                "commit_spec_kernel dispatches / batches per step)",
                "traffic_source": pmc_src,
                "bytes_per_eval": bpe,
                "convention": "BASELINE.md §4 / SURVEY §8(d): achieved = evals/s over the driver-timed steps x "
                              "bytes_per_eval (the node row one un-batched pod x node evaluation reads)",
                "kernels": kernels,
            },
            "breakdown_ms": {"eval": st["eval_ms"], "cand": st["cand_ms"], "commit": st["commit_ms"],
                             "exchange": st["exchange_ms"], "batches": st["batches"], "cuts": st["cuts"],
                             "slowpath_pods": st["slowpath_pods"]},
            "cpu_baseline": cpu,
        }
        if world == 1 and args.profile == "c3" and args.sample_pct is None and not args.no_extras:
            # the C5 and Coscheduling configurations beside the headline (extra keys; the C3 line above is unchanged)
            del eng
            t_x = time.perf_counter()
            line["c5"] = extra_c5(P, steps=10, nodes=100_000, sample=40)
            line["c5"]["wall_s_incl_setup"] = round(time.perf_counter() - t_x, 2)
            t_x = time.perf_counter()
            line["gang"] = extra_gang(cluster, cfg, P, calls=5, sample=40, threads=min(16, host_cpus()["usable"]))
            line["gang"]["wall_s_incl_setup"] = round(time.perf_counter() - t_x, 2)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
