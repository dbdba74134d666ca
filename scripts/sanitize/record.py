"""Records oracle workloads as call scripts for the sanitizer runs (scripts/sanitize/run.sh).

The recorder stands in for an Oracle / Engine: synth.load_into / load_ext_into and the schedule calls write each call
and its arrays (the ABI structs' bytes) into a file that san_host (ASan + UBSan build of the oracle and the host
library sources) replays call by call. Format: records of u32 op, u32 narr, then narr x (u64 nbytes, bytes); nbytes
= 2^64-1 is a NULL array.
"""
from __future__ import annotations

import os
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from koordinator_amd import abi, config, synth  # noqa: E402

OPS = {"create": 1, "set_now": 2, "nodes": 3, "metrics": 4, "assign": 5, "topo": 6, "numa": 7, "alloc": 8,
       "schedule": 9, "evaluate": 10, "ext_conf": 11, "devices": 12, "rsv": 13, "schedule_ext": 14}
NULL = (1 << 64) - 1


def fnv(h: int, b: bytes) -> int:
    a = np.frombuffer(b, np.uint8)
    for x in a.tolist():
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


class Recorder:
    """Records every call and forwards it to the (unsanitized) oracle, whose placements' FNV-1a is the replay's
    expected value."""

    def __init__(self, path: str, cfg):
        from oracle import oracle as orc
        self.path = path
        self.f = open(path, "wb")
        self.o = orc.Oracle(cfg)
        self.h = 1469598103934665603
        self._rec("create", bytes(cfg))

    def _rec(self, op: str, *arrs):
        self.f.write(struct.pack("<II", OPS[op], len(arrs)))
        for a in arrs:
            if a is None:
                self.f.write(struct.pack("<Q", NULL))
                continue
            b = a if isinstance(a, (bytes, bytearray)) else np.ascontiguousarray(a).tobytes()
            self.f.write(struct.pack("<Q", len(b)))
            self.f.write(b)

    def close(self):
        self.f.close()
        with open(self.path + ".expect", "w") as f:
            f.write(f"{self.h:016x}\n")
        self.o.close()

    # the Engine / Oracle calls synth.load_into and load_ext_into make
    def set_now(self, now_ns):
        self._rec("set_now", np.array([now_ns], np.int64))
        self.o.set_now(now_ns)

    def upsert_nodes(self, nodes, idx=None):
        self._rec("nodes", None if idx is None else np.asarray(idx, np.uint32), np.asarray(nodes, abi.NODE_DTYPE))
        self.o.upsert_nodes(nodes, idx)

    def upsert_metrics(self, metrics, pod_metrics=None, offsets=None, idx=None):
        self._rec("metrics", None if idx is None else np.asarray(idx, np.uint32), np.asarray(metrics, abi.METRIC_DTYPE),
                  None if pod_metrics is None else np.asarray(pod_metrics, abi.POD_METRIC_DTYPE),
                  None if offsets is None else np.asarray(offsets, np.uint32))
        self.o.upsert_metrics(metrics, pod_metrics, offsets, idx)

    def assign(self, node_idx, pods, ts):
        self._rec("assign", np.asarray(node_idx, np.uint32), np.asarray(pods, abi.POD_DTYPE), np.asarray(ts, np.int64))
        self.o.assign(node_idx, pods, ts)

    def register_topology(self, topo):
        self._rec("topo", np.atleast_1d(np.asarray(topo, abi.TOPOLOGY_DTYPE)))
        return self.o.register_topology(topo)

    def upsert_numa(self, numa, idx=None):
        self._rec("numa", None if idx is None else np.asarray(idx, np.uint32), np.asarray(numa, abi.NODE_NUMA_DTYPE))
        self.o.upsert_numa(numa, idx)

    def update_allocations(self, node_idx, allocs):
        self._rec("alloc", np.asarray(node_idx, np.uint32), np.asarray(allocs, abi.POD_ALLOCATION_DTYPE))
        self.o.update_allocations(node_idx, allocs)

    def ext_configure(self, args):
        self._rec("ext_conf", bytes(args))
        self.o.ext_configure(args)

    def upsert_devices(self, devs, idx=None):
        self._rec("devices", None if idx is None else np.asarray(idx, np.uint32), np.asarray(devs, abi.NODE_DEVICES_DTYPE))
        self.o.upsert_devices(devs, idx)

    def upsert_reservations(self, rsv):
        self._rec("rsv", np.asarray(rsv, abi.RESERVATION_DTYPE))
        self.o.upsert_reservations(rsv)

    def schedule(self, pods, seq=None, nthreads=1):
        seq = np.arange(len(pods), dtype=np.uint64) if seq is None else np.asarray(seq, np.uint64)
        self._rec("schedule", np.asarray(pods, abi.POD_DTYPE), seq, np.array([nthreads], np.int64))
        self.h = fnv(self.h, self.o.schedule(pods, seq, nthreads).tobytes())

    def evaluate(self, pods):
        self._rec("evaluate", np.asarray(pods, abi.POD_DTYPE))
        self.o.evaluate(pods)

    def schedule_ext(self, pods, ext, seq=None):
        seq = np.arange(len(pods), dtype=np.uint64) if seq is None else np.asarray(seq, np.uint64)
        self._rec("schedule_ext", np.asarray(pods, abi.POD_DTYPE), np.asarray(ext, abi.POD_EXT_DTYPE), seq)
        out, eo = self.o.schedule_ext(pods, ext, seq)
        self.h = fnv(fnv(self.h, out.tobytes()), eo.tobytes())


def main(out_dir: str):
    os.makedirs(out_dir, exist_ok=True)
    # C2 plugin set (Fit + LoadAware): plain pods, the serial and the parallelize.Until worker-pool paths
    c = synth.make_cluster(2000, 400, 1)
    r = Recorder(os.path.join(out_dir, "c2.bin"), config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_LA_FIT))
    synth.load_into(r, c)
    r.evaluate(c.pods[:8])
    r.schedule(c.pods[:200], nthreads=1)
    r.schedule(c.pods[200:], np.arange(200, 400, dtype=np.uint64), nthreads=4)
    r.close()
    # C3 (+ NodeNUMAResource: hints, topology-manager merge, NUMA split, takeCPUs cpusets)
    c = synth.make_cluster(1500, 300, 3)
    synth.make_numa(c)
    r = Recorder(os.path.join(out_dir, "c3.bin"), config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL))
    synth.load_into(r, c)
    r.evaluate(c.pods[:8])
    r.schedule(c.pods[:150], nthreads=1)
    r.schedule(c.pods[150:], np.arange(150, 300, dtype=np.uint64), nthreads=4)
    r.close()
    # C5 (Reservation + DeviceShare on NUMA-policy nodes, extended resources)
    from oracle import oracle as orc
    c = synth.make_cluster(1200, 300, 5)
    synth.make_numa(c)
    synth.make_ext(c, xres_node_pct=20, xres_pod_pct=10)
    r = Recorder(os.path.join(out_dir, "c5.bin"), config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL))
    synth.load_into(r, c)
    synth.load_ext_into(r, c, orc.ext_args_default())
    r.schedule_ext(c.pods, c.ext["pod_ext"])
    r.close()
    write_corpus(os.path.join(out_dir, "ingest.corpus"))
    print("recorded", sorted(os.listdir(out_dir)))


def write_corpus(path: str):
    """The ingest decoders' inputs: the reference vectors of tests/golden/ingest.json and the documented shapes of
    every annotation the decoders read (kind 1 quantity, 2 cpuset, 3 node annotation, 4 resource-spec, 5 cpu-topology,
    6 node label + kubelet policy text)."""
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "ingest.json")))
    recs = []
    for case in g["amplification_ratio"] + g["raw_allocatable"]:
        for k, v in case["annotations"].items():
            recs.append((3, k, v))
    for case in g["cpuset_parse"]:
        recs.append((2, "", case["s"]))
    for q in ["1", "100m", "1.5", "2Gi", "512Mi", "1e3", "1E-3", "0.001", "9223372036854775807", "1Ki", "-5", "3.25k",
              "12345678901234567890", ".5", "5.", "+7", "1.0000000001"]:
        recs.append((1, "", q))
    ann = {
        "scheduling.koordinator.sh/usage-thresholds": [
            '{"usageThresholds":{"cpu":65,"memory":80,"nvidia.com/gpu":10},"prodUsageThresholds":{"memory":70}}',
            '{"usageThresholds":{"cpu":65},"aggregatedUsage":{"usageThresholds":{"cpu":70},"usageAggregationType":"p95",'
            '"usageAggregatedDuration":"5m30s"}}',
            '{"aggregatedUsage":{"usageAggregatedDuration":"5x"}}'],
        "node.koordinator.sh/raw-allocatable": ['{"cpu":"96","memory":"512Gi"}'],
        "node.koordinator.sh/resource-amplification-ratio": ['{"cpu":1.5}', '{"cpu":1.22,"memory":1}'],
        "node.koordinator.sh/reservation": [
            '{"resources":{"cpu":"2","memory":"4Gi"}}', '{"reservedCPUs":"0-3","applyPolicy":"Default"}',
            '{"resources":{"cpu":"1500m"},"applyPolicy":"ReservedCPUsOnly"}'],
        "kubelet.koordinator.sh/cpu-manager-policy": ['{"policy":"static","options":{"full-pcpus-only":"true"},'
                                                      '"reservedCPUs":"0-1"}', '{"policy":"none"}'],
        "node.koordinator.sh/pod-cpu-allocs": ['[{"namespace":"a","name":"b","uid":"u","cpuset":"4-7","managedByKubelet":true}]'],
        "node.koordinator.sh/system-qos-resource": ['{"cpuset":"8-9","cpusetExclusive":true}'],
    }
    for k, vs in ann.items():
        for v in vs:
            recs.append((3, k, v))
    for v in ['{"requiredCPUBindPolicy":"FullPCPUs","preferredCPUExclusivePolicy":"PCPULevel"}',
              '{"preferredCPUBindPolicy":"SpreadByPCPUs"}', '{"preferredCPUBindPolicy":1}', '{"preferredCPUBindPolicy":""}']:
        recs.append((4, "", v))
    detail = [{"id": c, "core": c // 2, "socket": c // 32, "node": c // 16} for c in range(64)]
    recs.append((5, "", json.dumps({"detail": detail})))
    recs.append((5, "", json.dumps({"detail": detail[:3] + [{"id": 300, "core": 1, "socket": 0, "node": 0}]})))
    for k, v in [("node.koordinator.sh/cpu-bind-policy", "FullPCPUsOnly"),
                 ("node.koordinator.sh/numa-topology-policy", "SingleNUMANode"),
                 ("node.koordinator.sh/numa-allocate-strategy", "MostAllocated")]:
        recs.append((6, k, v))
        recs.append((6, k, '{"policy":"static","options":{"full-pcpus-only":"true"}}'))
    with open(path, "wb") as f:
        for kind, k, v in recs:
            kb, vb = k.encode(), v.encode()
            f.write(struct.pack("<III", kind, len(kb), len(vb)))
            f.write(kb)
            f.write(vb)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scripts", "sanitize", "build"))
