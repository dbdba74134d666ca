"""ctypes wrappers of the ingest decoders (include/gpuscore.h, gs_decode_*): annotation / label text -> ABI structs.

Pure host functions of libgpuscore (no device call): usable without a GPU."""
from __future__ import annotations

import ctypes as C

import numpy as np

from koordinator_amd import abi


class DecodeError(ValueError):
    def __init__(self, what: str, rc: int):
        super().__init__(f"{what}: rc={rc}")
        self.rc = rc


def _chk(rc: int, what: str):
    if rc != 0:
        raise DecodeError(what, rc)


def _enc(s):
    return None if s is None else s.encode()


def _kv(d: dict | None):
    d = d or {}
    arr = (abi.GsKv * max(1, len(d)))()
    for i, (k, v) in enumerate(d.items()):
        arr[i].key, arr[i].value = k.encode(), v.encode()
    return arr, len(d)


def quantity(s: str) -> tuple[int, int]:
    """resource.Quantity -> (Value(), MilliValue())"""
    v, mv = C.c_int64(), C.c_int64()
    _chk(abi.load().gs_decode_quantity(s.encode(), C.byref(v), C.byref(mv)), f"quantity {s!r}")
    return v.value, mv.value


def cpuset(s: str) -> list[int]:
    w = (C.c_uint64 * abi.GS_CPU_WORDS)()
    _chk(abi.load().gs_decode_cpuset(s.encode(), w), f"cpuset {s!r}")
    return [c for c in range(abi.GS_MAX_CPUS) if (w[c >> 6] >> (c & 63)) & 1]


def node_annotations(annotations: dict, node=None, numa=None):
    """-> (gs_node, gs_node_numa) with the annotation-derived fields filled"""
    node = node if node is not None else abi.GsNode()
    numa = numa if numa is not None else abi.GsNodeNuma()
    arr, n = _kv(annotations)
    _chk(abi.load().gs_decode_node_annotations(arr, n, C.byref(node), C.byref(numa)), "node annotations")
    return node, numa


def node_reservation_trim(annotations: dict, node) -> bool:
    """TransformNodeWithNodeReservation on node.allocatable / allowed_pod_number in place; True when trimmed"""
    arr, n = _kv(annotations)
    rc = abi.load().gs_node_reservation_trim(arr, n, C.byref(node))
    if rc < 0:
        raise DecodeError("node reservation", rc)
    return rc == 1


def node_reserved_cpus(annotations: dict) -> tuple[list[int], int, bool]:
    """GetReservedCPUs -> (reserved cpu ids, numReservedCPUs, reservedCPUs parsed)"""
    w = (C.c_uint64 * abi.GS_CPU_WORDS)()
    num = C.c_int32()
    arr, n = _kv(annotations)
    rc = abi.load().gs_node_reserved_cpus(arr, n, w, C.byref(num))
    if rc < 0:
        raise DecodeError("node reserved cpus", rc)
    return [c for c in range(abi.GS_MAX_CPUS) if (w[c >> 6] >> (c & 63)) & 1], num.value, rc == 0


def nrt_reserved_cpus(annotations: dict) -> list[int]:
    """TopologyOptions.ReservedCPUs from the NRT annotations"""
    w = (C.c_uint64 * abi.GS_CPU_WORDS)()
    arr, n = _kv(annotations)
    _chk(abi.load().gs_decode_nrt_reserved_cpus(arr, n, w), "nrt reserved cpus")
    return [c for c in range(abi.GS_MAX_CPUS) if (w[c >> 6] >> (c & 63)) & 1]


def node_labels(labels: dict, kubelet_cpu_manager_policy: str | None = None,
                kubelet_topology_policy: str | None = None, numa=None):
    numa = numa if numa is not None else abi.GsNodeNuma()
    arr, n = _kv(labels)
    _chk(abi.load().gs_decode_node_labels(arr, n, _enc(kubelet_cpu_manager_policy), _enc(kubelet_topology_policy),
                                          C.byref(numa)), "node labels")
    return numa


def resource_spec(json_text: str | None, pod=None):
    pod = pod if pod is not None else abi.GsPod()
    _chk(abi.load().gs_decode_resource_spec(_enc(json_text), C.byref(pod)), "resource-spec")
    return pod


def cpu_topology(json_text: str | None):
    t = abi.GsCpuTopology()
    _chk(abi.load().gs_decode_cpu_topology(_enc(json_text), C.byref(t)), "cpu-topology")
    return t


def topology_arrays(t) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    n = t.num_cpus
    return (np.array(t.core_id[:n], np.int32), np.array(t.socket_id[:n], np.uint8), np.array(t.node_id[:n], np.uint8))
