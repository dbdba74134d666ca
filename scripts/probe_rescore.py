"""Diagnostics on the GPU: cycles of one re-scoring job of the speculative commit (gs_debug_pair_probe mode 1: one row,
64 pods one per lane over the row's hint table) on the bench's C3 cluster, split by the row's kind (NUMA topology
policy or not) and by the pods' mix (all plain, all cpuset, the queue's mix).

    python scripts/probe_rescore.py > gpurun_out/probe_rescore.json
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from koordinator_amd import abi, config, synth
    from koordinator_amd.engine import Engine
    c = synth.make_cluster(50_000, 2048, config_id=2)
    synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, device=0, enabled=abi.GS_ENABLE_ALL)
    e = Engine(cfg)
    synth.load_into(e, c)
    recs = c.numa["node_numa"]
    pol = np.array([int(r["numa_topology_policy"]) for r in recs])
    rng = np.random.default_rng(7)
    policy_nodes = rng.choice(np.nonzero(pol != 0)[0], 48, replace=False)
    plain_nodes = rng.choice(np.nonzero(pol == 0)[0], 48, replace=False)
    pods = c.pods
    cs = np.nonzero(pods["cpuset"] if "cpuset" in pods.dtype.names else np.zeros(len(pods), bool))[0]
    mixes = {"queue": pods[:64]}
    out = {}
    for mix, pv in mixes.items():
        for kind, nodes in (("policy", policy_nodes), ("plain", plain_nodes)):
            _, warm, cold = e.pair_probe(pv, nodes, np.zeros(len(nodes), np.int32), 1)
            out[f"{mix}/{kind}"] = {"median_cycles": float(np.median(warm)), "p90": float(np.percentile(warm, 90)),
                                    "max": float(warm.max()), "cold_median": float(np.median(cold))}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
