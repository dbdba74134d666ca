"""Debug helper: schedule a small NUMA cluster with the default commit kernel and print the first differences
against the oracle (node, score, ties, feasible)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from koordinator_amd import abi, config, synth
from koordinator_amd.engine import Engine
from oracle import oracle as orc

for nodes, pods, numa in ((2000, 256, True), (2000, 256, False)):
    c = synth.make_cluster(nodes, pods, 1)
    if numa:
        synth.make_numa(c)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL if numa else abi.GS_ENABLE_LA_FIT)
    e, o = Engine(cfg), orc.Oracle(cfg)
    synth.load_into(e, c)
    synth.load_into(o, c)
    got = e.schedule(c.pods)
    want = o.schedule(c.pods)
    print("numa" if numa else "la-fit", "mirror", e.mirror_check(), "stats", e.stats())
    for f in ("node", "score", "ties", "feasible"):
        bad = np.nonzero(got[f] != want[f])[0]
        print(f, len(bad), bad[:8], got[f][bad[:8]], want[f][bad[:8]])
