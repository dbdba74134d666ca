"""Full-size parity, every pod: the GPU placements of a full-size run (saved by tests/test_gpu_fullsize.py on the GPU box
into gpurun_out/, committed under tests/golden/fullsize/) against the CPU oracle's sequential scheduleOne over the same
regenerated synthetic cluster — node, max score, tie count and feasible count of EVERY pod (no sampling, no replay).
Runs in the build container (no GPU): about 4e9 pod x node evaluations for the north-star workload.

    python scripts/full_parity.py bench       # C3, 50,000 nodes, the bench's 20,480 pods (calls of 2,048)
    python scripts/full_parity.py northstar   # C3, 100,000 nodes x 50,000 pods (one call)

Writes profiles/<ROUND>_full_parity_<workload>.json (ROUND from the environment, default r04)."""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WORKLOADS = {
    # name: (nodes, pods, config_id, GPU call size)
    "bench": (50_000, 20_480, 2, 2048),
    "northstar": (100_000, 50_000, 3, 50_000),
}


def placements_path(name: str) -> str:
    return os.path.join(ROOT, "tests", "golden", "fullsize", f"placements_{name}.npz")


def main() -> None:
    name = sys.argv[1] if len(sys.argv) > 1 else "bench"
    threads = int(os.environ.get("THREADS", os.cpu_count() or 1))
    from koordinator_amd import abi, config, synth
    from oracle import oracle as orc
    nodes, P, cid, step = WORKLOADS[name]
    with np.load(placements_path(name), allow_pickle=False) as z:
        got = z["placements"].view(abi.PLACEMENT_DTYPE).reshape(-1)
        meta = json.loads(str(z["meta"]))
    assert len(got) == P, (len(got), P)
    c = synth.make_cluster(nodes, P, config_id=cid)
    synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, batch_size=128, enabled=abi.GS_ENABLE_ALL)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    seq = np.arange(P, dtype=np.uint64)
    t0 = time.perf_counter()
    want = np.zeros(P, abi.PLACEMENT_DTYPE)
    chunk = 1024
    for k in range(0, P, chunk):
        want[k:k + chunk] = o.schedule(c.pods[k:k + chunk], seq[k:k + chunk], nthreads=threads)
        if (k // chunk) % 8 == 0:
            print(f"{name}: {k + chunk}/{P} pods, {time.perf_counter() - t0:.0f} s", flush=True)
    dt = time.perf_counter() - t0
    res = {"workload": name, "nodes": nodes, "pods": P, "config_id": cid, "gpu_call_pods": step,
           "gpu_run": meta, "oracle_threads": threads, "oracle_seconds": dt, "fields": {}}
    ok = True
    for f in ("node", "score", "ties", "feasible"):
        bad = np.nonzero(got[f] != want[f])[0]
        res["fields"][f] = {"mismatches": int(len(bad)), "first": [int(i) for i in bad[:10]]}
        ok = ok and len(bad) == 0
    res["placed"] = int((got["node"] >= 0).sum())
    res["identical"] = ok
    out = os.path.join(ROOT, "profiles", f"{os.environ.get('ROUND', 'r04')}_full_parity_{name}.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
