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
        "or_pods_forget": (C.c_int, [P, P, P, C.c_uint32]),
        "or_estimate_pod": (C.c_int, [C.POINTER(abi.GsLoadAwareArgs), P, P, P]),
        "or_estimate_node": (C.c_int, [P, P]),
        "or_loadaware_filter": (C.c_int, [P, P, C.c_uint32, P]),
        "or_loadaware_score": (C.c_int, [P, P, C.c_uint32, P]),
        "or_fit_filter": (C.c_int, [P, P, C.c_uint32, P]),
        "or_fit_score": (C.c_int, [P, P, C.c_uint32, P]),
        "or_evaluate": (C.c_int, [P, P, C.c_uint32, P, P, P]),
        "or_schedule": (C.c_int, [P, P, C.c_uint32, P, P, C.c_int]),
        "or_num_feasible_nodes_to_find": (C.c_uint32, [C.c_uint32, C.c_int32]),
        "or_next_start_node_index": (C.c_uint32, [P]),
        "or_schedule_replay": (C.c_int, [P, P, C.c_uint32, P, P, P, C.c_int]),
        "or_tiebreak_intn": (C.c_int32, [C.c_uint64, C.c_uint64, C.c_int64]),
        "or_phase_times": (C.c_int, [P, P]),
        "or_topology_register": (C.c_int, [P, P, P]),
        "or_nodes_numa_upsert": (C.c_int, [P, P, P, C.c_uint32]),
        "or_numa_allocations_update": (C.c_int, [P, P, P, C.c_uint32]),
        "or_numa_allocations_release": (C.c_int, [P, P, P, C.c_uint32]),
        "or_numa_allocation_get": (C.c_int, [P, C.c_uint32, C.c_uint64, P]),
        "or_set_hint_order": (C.c_int, [P, C.c_int]),
        "or_numa_topology_hints": (C.c_int, [P, P, C.c_uint32, P, P, P, C.c_uint32, P]),
        "or_take_cpus_test": (C.c_int, [C.c_int] * 5 + [P, P, P] + [C.c_int] * 4 + [P]),
        "or_policy_merge": (C.c_int, [C.c_int, C.c_uint64, C.c_int, P, P, P, P, P, P, P]),
        "or_policy_merge_scored": (C.c_int, [C.c_int, C.c_uint64, C.c_int, P, P, P, P, P, P, P, P]),
        "or_iterate_bitmasks": (C.c_int, [P, C.c_int, P, C.c_int]),
        "or_pods_on_event": (C.c_int, [P, C.c_int, P, P, C.c_uint32]),
        "or_assign_cache_get": (C.c_int, [P, C.c_uint32, P, P, C.c_uint32]),
        "or_node_allocation_script": (C.c_int, [C.c_int] * 5 + [P, P, P, P, P, P]),
        "or_available_numa_test": (C.c_int, [C.c_int] * 4 + [C.c_double, C.c_int64, C.c_int64, C.c_int64, C.c_int,
                                                              P, P, P, P]),
        "or_ext_args_default": (None, [C.POINTER(abi.GsExtArgs)]),
        "or_ext_configure": (C.c_int, [P, C.POINTER(abi.GsExtArgs)]),
        "or_node_devices_upsert": (C.c_int, [P, P, P, C.c_uint32]),
        "or_node_devices_get": (C.c_int, [P, C.c_uint32, P]),
        "or_reservations_upsert": (C.c_int, [P, P, C.c_uint32]),
        "or_reservations_remove": (C.c_int, [P, P, C.c_uint32]),
        "or_reservation_get": (C.c_int, [P, C.c_uint64, P]),
        "or_schedule_ext": (C.c_int, [P, P, P, C.c_uint32, P, P, P]),
        "or_score_reservation": (C.c_int64, [P, P]),
        "or_default_normalize_score": (C.c_int, [C.c_int64, C.c_int, P, C.c_uint32]),
        "or_reservation_node_scores": (C.c_int, [P, P, P, C.c_uint32, P, P, P]),
        "or_device_score": (C.c_int64, [C.POINTER(abi.GsExtArgs), P, P]),
        "or_device_filter": (C.c_uint32, [P, P]),
        "or_device_topology_hints": (C.c_int, [P, P, P, P, C.c_uint32, P, P]),
        "or_device_allocate": (C.c_uint32, [P, P, C.c_int, C.c_uint64]),
        "or_device_score_node": (C.c_int64, [C.POINTER(abi.GsExtArgs), P, P, P, C.c_uint32]),
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

    def forget(self, node_idx, pods):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        _chk(lib().or_pods_forget(self._h, abi.ptr(node_idx), abi.ptr(pods), len(pods)), "forget")

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

    # NodeNUMAResource state
    def register_topology(self, topo) -> int:
        t = np.ascontiguousarray(np.atleast_1d(topo), dtype=abi.TOPOLOGY_DTYPE)
        out = C.c_int32()
        _chk(lib().or_topology_register(self._h, abi.ptr(t), C.addressof(out)), "topology_register")
        return out.value

    def upsert_numa(self, numa, idx=None):
        numa = np.ascontiguousarray(numa, dtype=abi.NODE_NUMA_DTYPE)
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.uint32)
        _chk(lib().or_nodes_numa_upsert(self._h, abi.ptr(idx), abi.ptr(numa), len(numa)), "nodes_numa_upsert")

    def update_allocations(self, node_idx, allocs):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        allocs = np.ascontiguousarray(allocs, dtype=abi.POD_ALLOCATION_DTYPE)
        _chk(lib().or_numa_allocations_update(self._h, abi.ptr(node_idx), abi.ptr(allocs), len(allocs)), "alloc_update")

    def release_allocations(self, node_idx, uids):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        uids = np.ascontiguousarray(uids, dtype=np.uint64)
        _chk(lib().or_numa_allocations_release(self._h, abi.ptr(node_idx), abi.ptr(uids), len(uids)), "alloc_release")

    def allocation(self, node: int, uid: int):
        out = np.zeros(1, abi.POD_ALLOCATION_DTYPE)
        rc = lib().or_numa_allocation_get(self._h, node, uid, abi.ptr(out))
        if rc < 0:
            _chk(rc, "allocation_get")
        return out[0] if rc == 1 else None

    def topology_hints(self, pod, node: int = 0):
        """resourceManager.GetTopologyHints on `node`: None (nil map) or {resource slot: [(mask, preferred), ...]}."""
        pod = np.ascontiguousarray(np.atleast_1d(pod), dtype=abi.POD_DTYPE)
        cap = 64
        res, masks = np.zeros(cap, np.int32), np.zeros(cap, np.uint64)
        pref, cnt = np.zeros(cap, np.uint8), np.zeros(1, np.uint32)
        rc = lib().or_numa_topology_hints(self._h, abi.ptr(pod), node, abi.ptr(res), abi.ptr(masks), abi.ptr(pref), cap,
                                          abi.ptr(cnt))
        if rc < 0:
            _chk(rc, "topology_hints")
        if rc == 1:
            return None
        if rc > 0:
            raise RuntimeError(f"topology_hints: PreFilter / bind status {rc}")
        out = {}
        for k in range(int(cnt[0])):
            lst = out.setdefault(int(res[k]), [])
            if pref[k] != 2:
                lst.append((int(masks[k]), bool(pref[k])))
        return out

    def set_hint_order(self, reverse: bool):
        _chk(lib().or_set_hint_order(self._h, int(reverse)), "set_hint_order")

    def schedule(self, pods, seq=None, nthreads: int = 1):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        if seq is None:
            seq = np.arange(len(pods), dtype=np.uint64)
        seq = np.ascontiguousarray(seq, dtype=np.uint64)
        out = np.zeros(len(pods), abi.PLACEMENT_DTYPE)
        _chk(lib().or_schedule(self._h, abi.ptr(pods), len(pods), abi.ptr(seq), abi.ptr(out), int(nthreads)),
             "schedule")
        return out

    def phase_times(self) -> dict:
        """Seconds per scheduleOne phase since the last call (then reset): filter, score, select, reserve."""
        out = np.zeros(4, np.float64)
        _chk(lib().or_phase_times(self._h, abi.ptr(out)), "phase_times")
        return dict(zip(("filter", "score", "select", "reserve"), out.tolist()))

    @property
    def next_start_node_index(self) -> int:
        return int(lib().or_next_start_node_index(self._h))

    def pod_event(self, event: int, node_idx, pods):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        idx = np.ascontiguousarray(node_idx, dtype=np.int32)
        _chk(lib().or_pods_on_event(self._h, event, abi.ptr(idx), abi.ptr(pods), len(pods)), "pods_on_event")

    def assign_cache(self, node: int) -> list[tuple[int, int]]:
        u = np.zeros(256, np.uint64)
        t = np.zeros(256, np.int64)
        n = lib().or_assign_cache_get(self._h, node, abi.ptr(u), abi.ptr(t), 256)
        _chk(min(n, 0), "assign_cache_get")
        return list(zip(u[:n].tolist(), t[:n].tolist()))

    # ---- Reservation + DeviceShare
    def ext_configure(self, args: abi.GsExtArgs):
        _chk(lib().or_ext_configure(self._h, C.byref(args)), "ext_configure")

    def upsert_devices(self, devs, idx=None):
        devs = np.ascontiguousarray(devs, dtype=abi.NODE_DEVICES_DTYPE)
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.uint32)
        _chk(lib().or_node_devices_upsert(self._h, abi.ptr(idx), abi.ptr(devs), len(devs)), "node_devices_upsert")

    def devices(self, node: int):
        out = np.zeros(1, abi.NODE_DEVICES_DTYPE)
        _chk(lib().or_node_devices_get(self._h, node, abi.ptr(out)), "node_devices_get")
        return out[0]

    def upsert_reservations(self, rsv):
        rsv = np.ascontiguousarray(rsv, dtype=abi.RESERVATION_DTYPE)
        _chk(lib().or_reservations_upsert(self._h, abi.ptr(rsv), len(rsv)), "reservations_upsert")

    def remove_reservations(self, uids):
        uids = np.ascontiguousarray(uids, dtype=np.uint64)
        _chk(lib().or_reservations_remove(self._h, abi.ptr(uids), len(uids)), "reservations_remove")

    def reservation(self, uid: int):
        out = np.zeros(1, abi.RESERVATION_DTYPE)
        rc = lib().or_reservation_get(self._h, uid, abi.ptr(out))
        return out[0] if rc == 1 else None

    def schedule_ext(self, pods, ext, seq=None):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        ext = np.ascontiguousarray(ext, dtype=abi.POD_EXT_DTYPE)
        if seq is None:
            seq = np.arange(len(pods), dtype=np.uint64)
        seq = np.ascontiguousarray(seq, dtype=np.uint64)
        out = np.zeros(len(pods), abi.PLACEMENT_DTYPE)
        eo = np.zeros(len(pods), abi.EXT_PLACEMENT_DTYPE)
        _chk(lib().or_schedule_ext(self._h, abi.ptr(pods), abi.ptr(ext), len(pods), abi.ptr(seq), abi.ptr(out),
                                   abi.ptr(eo)), "schedule_ext")
        return out, eo

    def schedule_replay(self, pods, given, seq=None, nthreads: int = 1):
        """Pods with given[i] >= 0 are placed on that node (Filter there for the affinity, Reserve, assume);
        given[i] == -2 replays a FitError (nothing assumed); given[i] == -1 runs scheduleOne on the replayed state."""
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        if seq is None:
            seq = np.arange(len(pods), dtype=np.uint64)
        seq = np.ascontiguousarray(seq, dtype=np.uint64)
        given = np.ascontiguousarray(given, dtype=np.int32)
        assert len(given) == len(pods) and len(seq) == len(pods)
        out = np.zeros(len(pods), abi.PLACEMENT_DTYPE)
        _chk(lib().or_schedule_replay(self._h, abi.ptr(pods), len(pods), abi.ptr(seq), abi.ptr(given),
                                      abi.ptr(out), int(nthreads)), "schedule_replay")
        return out


def node_allocation_script(topology, ops):
    """ops: [("add", uid, cpus, excl) | ("release", uid) | ("available", max_ref, preferred_cpus)]; returns the
    available-CPU lists of the "available" ops and the final RefCount per CPU (dict, allocated CPUs only)."""
    n = len(ops)
    op = np.zeros(n, np.int32)
    uid = np.zeros(n, np.uint64)
    sets = np.zeros((n, 4), np.uint64)
    arg = np.zeros(n, np.int32)
    for k, o in enumerate(ops):
        cpus = o[2] if o[0] in ("add", "available") else []
        if o[0] == "add":
            op[k], uid[k], arg[k] = 0, o[1], o[3]
        elif o[0] == "release":
            op[k], uid[k] = 1, o[1]
        else:
            op[k], arg[k] = 2, o[1]
        for c in cpus:
            sets[k, c >> 6] |= np.uint64(1 << (c & 63))
    out = np.zeros((n, 4), np.uint64)
    ref = np.zeros(256, np.int32)
    _chk(lib().or_node_allocation_script(*topology, n, abi.ptr(op), abi.ptr(uid), abi.ptr(sets), abi.ptr(arg),
                                         abi.ptr(out), abi.ptr(ref)), "node_allocation_script")
    avail = [[c for c in range(256) if int(out[k, c >> 6]) >> (c & 63) & 1] for k in range(n) if ops[k][0] == "available"]
    return avail, {c: int(ref[c]) for c in range(256) if ref[c] >= 0}


def available_numa_test(topology, amp, zone_cpu, zone_mem, alloc_cpu0, n_cpuset):
    av = np.zeros(4, np.int64)
    al = np.zeros(4, np.int64)
    am = np.zeros(1, np.uint32)
    lm = np.zeros(1, np.uint32)
    _chk(lib().or_available_numa_test(*topology, amp, zone_cpu, zone_mem, alloc_cpu0, n_cpuset, abi.ptr(av),
                                      abi.ptr(am), abi.ptr(al), abi.ptr(lm)), "available_numa_test")
    avail = {z: {r: int(av[2 * z + r]) for r in range(2) if am[0] >> (2 * z + r) & 1} for z in range(2)}
    alloc = {z: {r: int(al[2 * z + r]) for r in range(2) if lm[0] >> (2 * z + r) & 1}
             for z in range(2) if lm[0] >> (4 + z) & 1}
    return avail, alloc


def ext_args_default() -> abi.GsExtArgs:
    a = abi.GsExtArgs()
    lib().or_ext_args_default(C.byref(a))
    return a


def score_reservation(pod, rsv) -> int:
    """scoreReservation (reservation/scoring.go:183-203)."""
    p = np.ascontiguousarray(np.atleast_1d(pod), abi.POD_DTYPE)
    r = np.ascontiguousarray(np.atleast_1d(rsv), abi.RESERVATION_DTYPE)
    return int(lib().or_score_reservation(abi.ptr(p), abi.ptr(r)))


def default_normalize_score(max_priority: int, reverse: bool, scores) -> list[int]:
    s = np.ascontiguousarray(scores, dtype=np.int64)
    _chk(lib().or_default_normalize_score(max_priority, int(reverse), abi.ptr(s), len(s)), "normalize")
    return s.tolist()


def reservation_node_scores(pod, rsv_per_node, nodes, pod_requested) -> list[int]:
    """Reservation PreScore + Score (reservation/scoring.go:42-160, nominator.go:140-190) per node."""
    p = np.ascontiguousarray(np.atleast_1d(pod), abi.POD_DTYPE)
    flat = [r for rs in rsv_per_node for r in rs]
    rs = np.ascontiguousarray(np.array(flat, dtype=abi.RESERVATION_DTYPE) if flat else np.zeros(1, abi.RESERVATION_DTYPE))
    off = np.zeros(len(rsv_per_node) + 1, np.uint32)
    off[1:] = np.cumsum([len(x) for x in rsv_per_node])
    nd = np.ascontiguousarray(nodes, abi.NODE_DTYPE)
    pr = np.ascontiguousarray(pod_requested, abi.NODE_DTYPE)
    raw = np.zeros(len(rsv_per_node), np.int64)
    _chk(lib().or_reservation_node_scores(abi.ptr(p), abi.ptr(rs), abi.ptr(off), len(rsv_per_node), abi.ptr(nd),
                                          abi.ptr(pr), abi.ptr(raw)), "reservation_node_scores")
    return raw.tolist()


def device_score(args: abi.GsExtArgs, devs, ext) -> int:
    d = np.ascontiguousarray(np.atleast_1d(devs), abi.NODE_DEVICES_DTYPE)
    e = np.ascontiguousarray(np.atleast_1d(ext), abi.POD_EXT_DTYPE)
    return int(lib().or_device_score(C.byref(args), abi.ptr(d), abi.ptr(e)))


def device_filter(devs, ext) -> int:
    d = np.ascontiguousarray(np.atleast_1d(devs), abi.NODE_DEVICES_DTYPE)
    e = np.ascontiguousarray(np.atleast_1d(ext), abi.POD_EXT_DTYPE)
    return int(lib().or_device_filter(abi.ptr(d), abi.ptr(e)))


def device_topology_hints(devs, ext):
    """DeviceShare GetPodTopologyHints on one node (topology_hint.go:33-214, GPU type): None for an invalid request,
    {} for no hints, else {resource name: [(NUMA node ids, preferred), ...]} (identical lists per name)."""
    d = np.ascontiguousarray(np.atleast_1d(devs), abi.NODE_DEVICES_DTYPE)
    e = np.ascontiguousarray(np.atleast_1d(ext), abi.POD_EXT_DTYPE)
    masks = np.zeros(64, np.uint64)
    pref = np.zeros(64, np.uint8)
    cnt, names = C.c_uint32(), C.c_uint32()
    rc = lib().or_device_topology_hints(abi.ptr(d), abi.ptr(e), abi.ptr(masks), abi.ptr(pref), 64, C.addressof(cnt),
                                        C.addressof(names))
    if rc < 0:
        return None
    if rc == 0:
        return {}
    lst = [([b for b in range(64) if int(masks[k]) >> b & 1], bool(pref[k])) for k in range(cnt.value)]
    keys = {0: "koordinator.sh/gpu-core", 1: "koordinator.sh/gpu-memory-ratio", 2: "koordinator.sh/gpu-memory"}
    return {keys[r]: list(lst) for r in range(3) if names.value >> r & 1}


def device_allocate(devs, ext, numa_nodes=None) -> int:
    """DeviceShare.Allocate with a NUMA affinity (topology_hint.go:57-106): 0 ok, else the failure code."""
    d = np.ascontiguousarray(np.atleast_1d(devs), abi.NODE_DEVICES_DTYPE)
    e = np.ascontiguousarray(np.atleast_1d(ext), abi.POD_EXT_DTYPE)
    m = 0
    for b in (numa_nodes or []):
        m |= 1 << b
    return int(lib().or_device_allocate(abi.ptr(d), abi.ptr(e), int(numa_nodes is not None), m))


def device_score_node(args: abi.GsExtArgs, total, free, request, request_mask) -> int:
    """resourceAllocationScorer.scoreNode (deviceshare/scoring.go:213-243) over gpu-core, gpu-memory-ratio, gpu-memory."""
    t = np.ascontiguousarray(total, np.int64)
    f = np.ascontiguousarray(free, np.int64)
    q = np.ascontiguousarray(request, np.int64)
    return int(lib().or_device_score_node(C.byref(args), abi.ptr(t), abi.ptr(f), abi.ptr(q), request_mask))


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


def num_feasible_nodes_to_find(num_all_nodes: int, pct: int) -> int:
    return int(lib().or_num_feasible_nodes_to_find(num_all_nodes, pct))


def tiebreak_intn(seed: int, seq: int, cnt: int) -> int:
    return lib().or_tiebreak_intn(seed, seq, cnt)


def take_cpus_test(topology, max_ref, available, alloc_ref, alloc_excl, needed, bind, excl, strategy):
    """takeCPUs on buildCPUTopologyForTest(*topology); returns (ok, sorted cpu list)."""
    words = np.zeros(4, np.uint64)
    for c in available:
        words[c >> 6] |= np.uint64(1) << np.uint64(c & 63)
    ref = np.ascontiguousarray(alloc_ref, dtype=np.int32)
    ex = np.ascontiguousarray(alloc_excl, dtype=np.int32)
    out = np.zeros(4, np.uint64)
    rc = lib().or_take_cpus_test(*[int(x) for x in topology], int(max_ref), abi.ptr(words), abi.ptr(ref), abi.ptr(ex),
                                 int(needed), int(bind), int(excl), int(strategy), abi.ptr(out))
    cpus = [c for c in range(256) if (int(out[c >> 6]) >> (c & 63)) & 1]
    return rc == 0, cpus


def policy_merge(policy: int, numa_nodes, lists) -> tuple[dict, bool]:
    """topologymanager Policy.Merge over filterProvidersHints' lists (each a list of {"mask": bits|None,
    "preferred": bool, "score": int (optional, 0)}) -> (merged hint, admit)."""
    lens = np.array([len(l) for l in lists], np.int32)
    flat = [h for l in lists for h in l]
    has = np.array([h["mask"] is not None for h in flat], np.uint8)
    masks = np.array([sum(1 << b for b in (h["mask"] or [])) for h in flat], np.uint64)
    pref = np.array([bool(h["preferred"]) for h in flat], np.uint8)
    scores = np.array([int(h.get("score", 0)) for h in flat], np.int64)
    oh, om, op = np.zeros(1, np.uint8), np.zeros(1, np.uint64), np.zeros(1, np.uint8)
    nm = sum(1 << b for b in numa_nodes)
    admit = lib().or_policy_merge_scored(policy, nm, len(lists), lens.ctypes.data, has.ctypes.data, masks.ctypes.data,
                                         pref.ctypes.data, scores.ctypes.data, oh.ctypes.data, om.ctypes.data,
                                         op.ctypes.data)
    bits = [b for b in range(64) if int(om[0]) >> b & 1] if oh[0] else None
    return {"mask": bits, "preferred": bool(op[0])}, bool(admit)


def iterate_bitmasks(bits) -> list[int]:
    """bitmask.IterateBitMasks visit order (masks as integers)."""
    b = np.array(bits, np.int32)
    n = lib().or_iterate_bitmasks(b.ctypes.data, len(b), None, 0)
    out = np.zeros(max(n, 1), np.uint64)
    lib().or_iterate_bitmasks(b.ctypes.data, len(b), out.ctypes.data, n)
    return [int(x) for x in out[:n]]

