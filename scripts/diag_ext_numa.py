"""Diagnostics for the extension path on NUMA-policy clusters: engine and oracle pod by pod (one pod per call), stop
at the first difference and print the pod, both results, and the state of the nodes involved."""
import sys
import numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from koordinator_amd import abi, config, synth
from koordinator_amd.engine import Engine
from oracle import oracle as orc

pct = int(sys.argv[1]) if len(sys.argv) > 1 else 100
c = synth.make_cluster(1500, 600, config_id=13 + pct)
synth.make_numa(c, numa_policy_pct=pct, cpuset_pod_pct=0)
synth.make_ext(c, gpu_node_pct=50, gpu_pod_pct=50, owner_pod_pct=0)
cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL)
a = orc.ext_args_default()
e, o = Engine(cfg), orc.Oracle(cfg)
for x in (e, o):
    synth.load_into(x, c)
    synth.load_ext_into(x, c, a)
nn = c.numa["node_numa"]
for j in range(len(c.pods)):
    sl = slice(j, j + 1)
    seq = np.array([j], np.uint64)
    gp, gx = e.schedule_ext(c.pods[sl], c.ext["pod_ext"][sl], seq)
    op, ox = o.schedule_ext(c.pods[sl], c.ext["pod_ext"][sl], seq)
    same = all(gp[f][0] == op[f][0] for f in ("node", "feasible", "score", "ties"))
    same = same and all(np.array_equal(gx[f], ox[f]) for f in ("gpu_minor_mask", "gpu_count"))
    if not same:
        print("first difference at pod", j)
        print(" pod requests", c.pods["requests"][j][:3], "mask", c.pods["request_mask"][j], "qos",
              c.pods["qos_class"][j], "prio", c.pods["priority_class"][j])
        print(" ext", c.ext["pod_ext"][j])
        print(" gpu   ", gp[0], gx[0])
        print(" oracle", op[0], ox[0])
        for i in {int(gp["node"][0]), int(op["node"][0])} - {-1}:
            print(" node", i, "policy", nn["numa_topology_policy"][i], "zones", nn["num_zones"][i],
                  [(int(z["node_id"]), int(z["cpu_milli"]), int(z["memory"])) for z in nn["zones"][i][:nn["num_zones"][i]]],
                  "bind", nn["node_cpu_bind_policy"][i])
            d = e.devices(i)
            print("  devices", [(int(g["minor"]), int(g["numa_node"]), list(g["total"]), list(g["used"]))
                                for g in d["gpus"][:d["num_gpus"]]], "has", d["has_device"])
            print("  oracle hints", orc.device_topology_hints(o.devices(i), c.ext["pod_ext"][j]))
        sys.exit(1)
    if gp["node"][0] >= 0:
        i = int(gp["node"][0])
        uid = int(c.pods["uid"][j])
        ga, oa = e.allocation(i, uid), o.allocation(i, uid)
        if (ga is None) != (oa is None) or (ga is not None and ga.tobytes() != oa.tobytes()):
            print("allocation differs at pod", j, "node", i, ga, oa)
            sys.exit(1)
print("no difference over", len(c.pods), "pods")
