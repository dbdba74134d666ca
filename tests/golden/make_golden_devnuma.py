"""Generates tests/golden/devnuma.json: reference test vectors of DeviceShare as a NUMA topology hint provider
(SURVEY 8(f) rank 2), transcribed by hand from the reference's Go tests into data (gpu-core / gpu-memory-ratio in
percent units, gpu-memory in bytes, NUMA affinities as lists of NUMA node ids).

  deviceshare/device_allocator_test.go:49-57   fakeDeviceCR: 8 GPUs (minors 0-3 on NUMA node 0 / socket 0, minors 4-7
                                                on NUMA node 1 / socket 1; 100 core, 100 ratio, 83201216Ki each), and
                                                fakeDeviceCRWithoutTopology (:59-67, the same GPUs without a Topology)
  deviceshare/topology_hint_test.go:40-282     TestPlugin_GetPodTopologyHints, GPU cases (the RDMA / FPGA / joint-
                                                allocation cases are outside the device path's GPU-only scope)
  deviceshare/topology_hint_test.go:284-430    TestPlugin_Allocate, GPU case ("allocate gpu&rdma by affinity")

Cases marked "derived" are not in the reference tables: they follow from the same code on the CR without topology
(numaTopology.nodes is empty, so IterateBitMasks visits no mask and the provider returns an empty map; an
allocator with a NUMA affinity skips devices without a Topology, device_allocator.go:148-152).

    python tests/golden/make_golden_devnuma.py
"""
import json
import os

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "devnuma.json")
Ki = 1024
GPU_MEM = 83201216 * Ki


def gpus(topology=True, used=None):
    used = used or {}
    out = []
    for m in range(8):
        out.append({"minor": m, "numa_node": (0 if m < 4 else 1) if topology else -1,
                    "total": {"core": 100, "ratio": 100, "memory": GPU_MEM},
                    "used": used.get(m, {})})
    return out


def main():
    core_ratio_100 = {"core": 100, "ratio": 100}
    hints_two_numa = [[[0], True], [[1], True], [[0, 1], False]]
    cases = [
        {"name": "generate gpu hints (gpu part of gpu&rdma)", "src": "deviceshare/topology_hint_test.go:63-91",
         "gpus": gpus(), "request": core_ratio_100,
         "want": {"koordinator.sh/gpu-core": hints_two_numa, "koordinator.sh/gpu-memory": hints_two_numa,
                  "koordinator.sh/gpu-memory-ratio": hints_two_numa}},
        {"name": "generate gpu hints with assigned devices", "src": "deviceshare/topology_hint_test.go:92-122",
         "gpus": gpus(used={0: {"core": 100, "ratio": 100}}), "request": {"core": 400, "ratio": 400},
         "want": {n: [[[1], True], [[0, 1], False]] for n in
                  ("koordinator.sh/gpu-core", "koordinator.sh/gpu-memory", "koordinator.sh/gpu-memory-ratio")}},
        {"name": "derived: devices without topology give no hints", "src": "device_allocator_test.go:59-67 + "
         "topology_hint.go:120-213", "gpus": gpus(topology=False), "request": core_ratio_100, "want": {}},
    ]
    allocate = [
        {"name": "allocate gpu by affinity", "src": "deviceshare/topology_hint_test.go:306-315",
         "gpus": gpus(), "request": {"core": 100, "memory": 8 * Ki * Ki * Ki}, "numa_nodes": [0], "ok": True},
        {"name": "derived: affinity without device topology", "src": "device_allocator.go:148-152",
         "gpus": gpus(topology=False), "request": {"core": 100, "memory": 8 * Ki * Ki * Ki}, "numa_nodes": [0],
         "ok": False},
        {"name": "derived: no affinity without device topology", "src": "device_allocator.go:148-152",
         "gpus": gpus(topology=False), "request": {"core": 100, "memory": 8 * Ki * Ki * Ki}, "numa_nodes": None,
         "ok": True},
        {"name": "derived: 400% on the NUMA node holding a used GPU", "src": "topology_hint_test.go:92-122 + "
         "device_allocator.go:139-163", "gpus": gpus(used={0: {"core": 100, "ratio": 100}}),
         "request": {"core": 400, "ratio": 400}, "numa_nodes": [0], "ok": False},
    ]
    with open(OUT, "w") as f:
        json.dump({"topology_hints": cases, "allocate": allocate}, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
