"""ctypes wrapper of oracle/liboracle.so — the CPU restatement used as the parity checker.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (checker) and bench.py's
cpu_baseline leg. The product package koordinator_amd/ never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from koordinator_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
P = C.c_void_p


def build() -> None:
    subprocess.check_call(["make", "-s", "-C", HERE])


def _load() -> C.CDLL:
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    sig = {
        "or_create": (P, [C.POINTER(abi.GsConfig)]),
        "or_destroy": (None, [P]),
        "or_set_now": (C.c_int, [P, C.c_int64]),
        "or_nodes_upsert": (C.c_int, [P, P, P, C.c_uint32]),
        "or_node_metrics_upsert": (C.c_int, [P, P, P, C.c_uint32, P, P]),
        "or_pods_assign": (C.c_int, [P, P, P, P, C.c_uint32]),
        "or_pods_unassign": (C.c_int, [P, P, P, C.c_uint32]),
        "or_estimate_pod": (C.c_int, [C.POINTER(abi.GsLoadAwareArgs), P, P, P]),
        "or_estimate_node": (C.c_int, [P, P]),
        "or_loadaware_filter": (C.c_int, [P, P, C.c_uint32, P]),
        "or_loadaware_score": (C.c_int, [P, P, C.c_uint32, P]),
        "or_fit_filter": (C.c_int, [P, P, C.c_uint32, P]),
        "or_fit_score": (C.c_int, [P, P, C.c_uint32, P]),
        "or_evaluate": (C.c_int, [P, P, C.c_uint32, P, P, P]),
        "or_schedule": (C.c_int, [P, P, C.c_uint32, P, P, C.c_int]),
        "or_tiebreak_intn": (C.c_int32, [C.c_uint64, C.c_uint64, C.c_int64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _chk(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"oracle {what} failed: {rc}")


class Oracle:
    """Mirror of koordinator_amd.engine.Engine's interface, computed by the CPU restatement."""

    def __init__(self, cfg: abi.GsConfig):
        self.cfg = cfg
        self.n = cfg.num_nodes
        self._h = lib().or_create(C.byref(cfg))
        if not self._h:
            raise RuntimeError("or_create failed")

    def close(self):
        if self._h:
            lib().or_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def set_now(self, now_ns: int):
        _chk(lib().or_set_now(self._h, int(now_ns)), "set_now")

    def upsert_nodes(self, nodes: np.ndarray, idx: np.ndarray | None = None):
        nodes = np.ascontiguousarray(nodes, dtype=abi.NODE_DTYPE)
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.uint32)
        _chk(lib().or_nodes_upsert(self._h, abi.ptr(idx), abi.ptr(nodes), len(nodes)), "nodes_upsert")

    def upsert_metrics(self, metrics, pod_metrics=None, offsets=None, idx=None):
        metrics = np.ascontiguousarray(metrics, dtype=abi.METRIC_DTYPE)
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.uint32)
        if pod_metrics is not None:
            pod_metrics = np.ascontiguousarray(pod_metrics, dtype=abi.POD_METRIC_DTYPE)
            offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        _chk(lib().or_node_metrics_upsert(self._h, abi.ptr(idx), abi.ptr(metrics), len(metrics),
                                          abi.ptr(pod_metrics), abi.ptr(offsets)), "metrics_upsert")

    def assign(self, node_idx, pods, ts):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        _chk(lib().or_pods_assign(self._h, abi.ptr(node_idx), abi.ptr(pods), abi.ptr(ts), len(pods)), "assign")

    def unassign(self, node_idx, pods):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        _chk(lib().or_pods_unassign(self._h, abi.ptr(node_idx), abi.ptr(pods), len(pods)), "unassign")

    # plugin-level
    def loadaware_filter(self, pod, node: int) -> bool:
        out = C.c_int32()
        p = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        _chk(lib().or_loadaware_filter(self._h, abi.ptr(p), node, C.addressof(out)), "la_filter")
        return bool(out.value)

    def loadaware_score(self, pod, node: int) -> int:
        out = C.c_int64()
        p = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        _chk(lib().or_loadaware_score(self._h, abi.ptr(p), node, C.addressof(out)), "la_score")
        return out.value

    def fit_filter(self, pod, node: int) -> int:
        out = C.c_uint32()
        p = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        _chk(lib().or_fit_filter(self._h, abi.ptr(p), node, C.addressof(out)), "fit_filter")
        return out.value

    def fit_score(self, pod, node: int) -> int:
        out = C.c_int64()
        p = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        _chk(lib().or_fit_score(self._h, abi.ptr(p), node, C.addressof(out)), "fit_score")
        return out.value

    def evaluate(self, pods):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        P_, N = len(pods), self.n
        scores = np.empty((P_, N), np.int16)
        codes = np.empty((P_, N), np.uint16)
        plugin = np.empty((P_, N, abi.GS_NUM_PLUGINS), np.int16)
        _chk(lib().or_evaluate(self._h, abi.ptr(pods), P_, abi.ptr(scores), abi.ptr(codes), abi.ptr(plugin)),
             "evaluate")
        return scores, codes, plugin

    def schedule(self, pods, seq=None, nthreads: int = 1):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        if seq is None:
            seq = np.arange(len(pods), dtype=np.uint64)
        seq = np.ascontiguousarray(seq, dtype=np.uint64)
        out = np.zeros(len(pods), abi.PLACEMENT_DTYPE)
        _chk(lib().or_schedule(self._h, abi.ptr(pods), len(pods), abi.ptr(seq), abi.ptr(out), int(nthreads)),
             "schedule")
        return out


def estimate_pod(args: abi.GsLoadAwareArgs, pod) -> tuple[int, int, int]:
    out = np.zeros(2, np.int64)
    mask = C.c_uint32()
    p = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
    _chk(lib().or_estimate_pod(C.byref(args), abi.ptr(p), abi.ptr(out), C.addressof(mask)), "estimate_pod")
    return int(out[0]), int(out[1]), mask.value


def estimate_node(node) -> tuple[int, int]:
    out = np.zeros(2, np.int64)
    n = np.ascontiguousarray(np.atleast_1d(node), dtype=abi.NODE_DTYPE)
    _chk(lib().or_estimate_node(abi.ptr(n), abi.ptr(out)), "estimate_node")
    return int(out[0]), int(out[1])


def tiebreak_intn(seed: int, seq: int, cnt: int) -> int:
    return lib().or_tiebreak_intn(seed, seq, cnt)
