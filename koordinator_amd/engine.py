"""Python host mirror of the plugin interface over libgpuscore's C-ABI.

`Engine` is one scheduler profile (NodeResourcesFit + LoadAwareScheduling) on one GPU. Its methods map
1:1 onto the C-ABI, which in turn replaces the reference plugin entry points:

  Engine(cfg)            loadaware.New / noderesources.NewFit        (load_aware.go:76-110)
  set_now                time.Now injection                           (helper.go:36-41, pod_assign_cache.go:30)
  upsert_nodes           scheduler cache snapshot (NodeInfo)          ([upstream] Cache.UpdateSnapshot)
  upsert_metrics         NodeMetric informer                          (load_aware.go:95,133,278)
  assign / unassign      podAssignCache.assign / unAssign             (pod_assign_cache.go:53-80)
  evaluate               RunFilterPlugins + RunScorePlugins per node  (load_aware.go:123-171,269-335)
  schedule               scheduleOne loop incl. selectHost + Reserve  ([upstream] schedule_one.go)

The product path has no CPU fallback: if libgpuscore or a GPU is missing, construction fails.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        _lib = abi.load()
    return _lib


class GpuScoreError(RuntimeError):
    pass


class LocalGroup:
    """The in-process device transport's group (gs_local_group): the ranks are threads of this process, each with its
    own Engine; the per-batch all-gathers (score rows, or candidate levels under GS_XCHG=levels) run stream-ordered on
    the device as ncclAllGather does."""

    def __init__(self, nranks: int):
        self._h = C.c_void_p()
        rc = lib().gs_local_group_create(nranks, C.byref(self._h))
        if rc != 0:
            raise GpuScoreError(f"gs_local_group_create: {rc}")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().gs_local_group_destroy(self._h)
            self._h = None


class Engine:
    def __init__(self, cfg: abi.GsConfig):
        self.cfg = cfg
        self.n = cfg.num_nodes
        h = C.c_void_p()
        rc = lib().gs_create(C.byref(cfg), C.byref(h))
        if rc != 0:
            raise GpuScoreError(f"gs_create failed: {rc}")
        self._h = h
        self._cb = None

    def close(self):
        if getattr(self, "_h", None):
            lib().gs_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc: int, what: str):
        if rc != 0:
            msg = lib().gs_last_error(self._h)
            raise GpuScoreError(f"{what}: rc={rc}: {msg.decode() if msg else ''}")

    def set_now(self, now_ns: int):
        self._chk(lib().gs_set_now(self._h, int(now_ns)), "gs_set_now")

    def upsert_nodes(self, nodes, idx=None):
        nodes = np.ascontiguousarray(nodes, dtype=abi.NODE_DTYPE)
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.uint32)
        self._chk(lib().gs_nodes_upsert(self._h, abi.ptr(idx), abi.ptr(nodes), len(nodes)), "gs_nodes_upsert")

    def upsert_metrics(self, metrics, pod_metrics=None, offsets=None, idx=None):
        metrics = np.ascontiguousarray(metrics, dtype=abi.METRIC_DTYPE)
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.uint32)
        if pod_metrics is not None:
            pod_metrics = np.ascontiguousarray(pod_metrics, dtype=abi.POD_METRIC_DTYPE)
            offsets = np.ascontiguousarray(offsets, dtype=np.uint32)
        self._chk(lib().gs_node_metrics_upsert(self._h, abi.ptr(idx), abi.ptr(metrics), len(metrics),
                                               abi.ptr(pod_metrics), abi.ptr(offsets)), "gs_node_metrics_upsert")

    def assign(self, node_idx, pods, ts):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        self._chk(lib().gs_pods_assign(self._h, abi.ptr(node_idx), abi.ptr(pods), abi.ptr(ts), len(pods)),
                  "gs_pods_assign")

    def unassign(self, node_idx, pods):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        self._chk(lib().gs_pods_unassign(self._h, abi.ptr(node_idx), abi.ptr(pods), len(pods)), "gs_pods_unassign")

    def forget(self, node_idx, pods):
        """gs_pods_forget: ForgetPod of assumed pods after Unreserve (NodeInfo, podAssignCache, NUMA allocation)."""
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        self._chk(lib().gs_pods_forget(self._h, abi.ptr(node_idx), abi.ptr(pods), len(pods)), "gs_pods_forget")

    def evaluate(self, pods):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        P, N = len(pods), self.n
        scores = np.empty((P, N), np.int16)
        codes = np.empty((P, N), np.uint16)
        plugin = np.empty((P, N, abi.GS_NUM_PLUGINS), np.int16)
        self._chk(lib().gs_evaluate(self._h, abi.ptr(pods), P, abi.ptr(scores), abi.ptr(codes), abi.ptr(plugin)),
                  "gs_evaluate")
        return scores, codes, plugin

    def schedule(self, pods, seq=None):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        if seq is None:
            seq = np.arange(len(pods), dtype=np.uint64)
        seq = np.ascontiguousarray(seq, dtype=np.uint64)
        out = np.zeros(len(pods), abi.PLACEMENT_DTYPE)
        self._chk(lib().gs_schedule(self._h, abi.ptr(pods), len(pods), abi.ptr(seq), abi.ptr(out)), "gs_schedule")
        return out

    def schedule_submit(self, pods, seq=None):
        """gs_schedule_submit: returns a handle for schedule_wait (the placements array, filled once it completes)."""
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        if seq is None:
            seq = np.arange(len(pods), dtype=np.uint64)
        seq = np.ascontiguousarray(seq, dtype=np.uint64)
        out = np.zeros(len(pods), abi.PLACEMENT_DTYPE)
        t = C.c_uint64(0)
        self._chk(lib().gs_schedule_submit(self._h, abi.ptr(pods), len(pods), abi.ptr(seq), abi.ptr(out), C.byref(t)),
                  "gs_schedule_submit")
        return (t.value, out)

    def schedule_wait(self, handle):
        t, out = handle
        self._chk(lib().gs_schedule_wait(self._h, t), "gs_schedule_wait")
        return out

    def pod_event(self, event: int, node_idx, pods):
        """podAssignCache OnAdd / OnUpdate / OnDelete (node_idx -1 = pod.Spec.NodeName == "")."""
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        idx = np.ascontiguousarray(node_idx, dtype=np.int32)
        self._chk(lib().gs_pods_on_event(self._h, event, abi.ptr(idx), abi.ptr(pods), len(pods)), "gs_pods_on_event")

    def assign_cache(self, node: int) -> list[tuple[int, int]]:
        u = np.zeros(256, np.uint64)
        t = np.zeros(256, np.int64)
        n = lib().gs_assign_cache_get(self._h, node, abi.ptr(u), abi.ptr(t), 256)
        self._chk(min(n, 0), "gs_assign_cache_get")
        return list(zip(u[:n].tolist(), t[:n].tolist()))

    # ---- Reservation + DeviceShare
    def ext_configure(self, args: abi.GsExtArgs):
        self._chk(lib().gs_ext_configure(self._h, C.byref(args)), "gs_ext_configure")

    def upsert_devices(self, devs, idx=None):
        devs = np.ascontiguousarray(devs, dtype=abi.NODE_DEVICES_DTYPE)
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.uint32)
        self._chk(lib().gs_node_devices_upsert(self._h, abi.ptr(idx), abi.ptr(devs), len(devs)), "gs_node_devices_upsert")

    def devices(self, node: int):
        out = abi.GsNodeDevices()
        self._chk(lib().gs_node_devices_get(self._h, node, C.byref(out)), "gs_node_devices_get")
        return np.frombuffer(bytes(out), dtype=abi.NODE_DEVICES_DTYPE)[0]

    def upsert_reservations(self, rsv):
        rsv = np.ascontiguousarray(rsv, dtype=abi.RESERVATION_DTYPE)
        self._chk(lib().gs_reservations_upsert(self._h, abi.ptr(rsv), len(rsv)), "gs_reservations_upsert")

    def remove_reservations(self, uids):
        uids = np.ascontiguousarray(uids, dtype=np.uint64)
        self._chk(lib().gs_reservations_remove(self._h, abi.ptr(uids), len(uids)), "gs_reservations_remove")

    def reservation(self, uid: int):
        out = abi.GsReservation()
        rc = lib().gs_reservation_get(self._h, uid, C.byref(out))
        self._chk(min(rc, 0), "gs_reservation_get")
        return np.frombuffer(bytes(out), dtype=abi.RESERVATION_DTYPE)[0] if rc == 1 else None

    def schedule_ext(self, pods, ext, seq=None):
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        ext = np.ascontiguousarray(ext, dtype=abi.POD_EXT_DTYPE)
        assert len(ext) == len(pods)
        if seq is None:
            seq = np.arange(len(pods), dtype=np.uint64)
        seq = np.ascontiguousarray(seq, dtype=np.uint64)
        out = np.zeros(len(pods), abi.PLACEMENT_DTYPE)
        eo = np.zeros(len(pods), abi.EXT_PLACEMENT_DTYPE)
        self._chk(lib().gs_schedule_ext(self._h, abi.ptr(pods), abi.ptr(ext), len(pods), abi.ptr(seq), abi.ptr(out),
                                        abi.ptr(eo)), "gs_schedule_ext")
        return out, eo

    # ---- NodeNUMAResource state
    def register_topology(self, topo) -> int:
        t = abi.GsCpuTopology.from_buffer_copy(np.ascontiguousarray(np.atleast_1d(topo), abi.TOPOLOGY_DTYPE).tobytes())
        out = C.c_int32()
        self._chk(lib().gs_topology_register(self._h, C.byref(t), C.byref(out)), "gs_topology_register")
        return out.value

    def upsert_numa(self, numa, idx=None):
        numa = np.ascontiguousarray(numa, dtype=abi.NODE_NUMA_DTYPE)
        if idx is not None:
            idx = np.ascontiguousarray(idx, dtype=np.uint32)
        self._chk(lib().gs_nodes_numa_upsert(self._h, abi.ptr(idx), abi.ptr(numa), len(numa)), "gs_nodes_numa_upsert")

    def update_allocations(self, node_idx, allocs):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        allocs = np.ascontiguousarray(allocs, dtype=abi.POD_ALLOCATION_DTYPE)
        self._chk(lib().gs_numa_allocations_update(self._h, abi.ptr(node_idx), abi.ptr(allocs), len(allocs)),
                  "gs_numa_allocations_update")

    def release_allocations(self, node_idx, uids):
        node_idx = np.ascontiguousarray(node_idx, dtype=np.uint32)
        uids = np.ascontiguousarray(uids, dtype=np.uint64)
        self._chk(lib().gs_numa_allocations_release(self._h, abi.ptr(node_idx), abi.ptr(uids), len(uids)),
                  "gs_numa_allocations_release")

    def allocation(self, node: int, uid: int):
        out = abi.GsPodAllocation()
        rc = lib().gs_numa_allocation_get(self._h, node, uid, C.byref(out))
        if rc < 0:
            self._chk(rc, "gs_numa_allocation_get")
        return np.frombuffer(bytes(out), abi.POD_ALLOCATION_DTYPE)[0] if rc == 1 else None

    # ---- multi-GPU
    def comm_init_rccl(self, uid: bytes, nranks: int, rank: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._chk(lib().gs_comm_init_rccl(self._h, buf, nranks, rank), "gs_comm_init_rccl")

    def comm_init_callback(self, nranks: int, rank: int, allgather):
        """allgather(send: bytes) -> list[bytes] of every rank's payload (rank order)."""
        def _cb(user, send, recv, nbytes):
            try:
                data = C.string_at(send, nbytes)
                parts = allgather(data)
                blob = b"".join(parts)
                C.memmove(recv, blob, len(blob))
                return 0
            except Exception:
                return -1
        self._cb = abi.ALLGATHER_FN(_cb)
        self._chk(lib().gs_comm_init_callback(self._h, nranks, rank, self._cb, None), "gs_comm_init_callback")

    def comm_init_local(self, group: "LocalGroup", rank: int):
        """In-process device transport: this context is rank `rank` of `group` (ranks as threads of this process)."""
        self._group = group   # the group outlives its contexts
        self._chk(lib().gs_comm_init_local(self._h, group._h, rank), "gs_comm_init_local")

    def stats(self) -> dict:
        s = abi.GsStats()
        self._chk(lib().gs_get_stats(self._h, C.byref(s)), "gs_get_stats")
        return {k: getattr(s, k) for k, _ in abi.GsStats._fields_}

    def reset_stats(self):
        self._chk(lib().gs_reset_stats(self._h), "gs_reset_stats")

    def reset(self):
        """Rebuild the HBM mirror from the host state after a failed call (gs_reset)."""
        self._chk(lib().gs_reset(self._h), "gs_reset")

    def synchronize(self):
        self._chk(lib().gs_synchronize(self._h), "gs_synchronize")

    def mirror_check(self) -> int:
        rc = lib().gs_debug_mirror_check(self._h)
        if rc < 0:
            self._chk(rc, "gs_debug_mirror_check")
        return rc

    def numa_merge(self, cases):
        """Diagnostics: the device's topology-manager Merge on gs_merge_case records (gs_debug_numa_merge)."""
        cases = np.ascontiguousarray(cases, dtype=abi.MERGE_CASE_DTYPE)
        out = np.zeros(len(cases), abi.MERGE_RESULT_DTYPE)
        self._chk(lib().gs_debug_numa_merge(self._h, abi.ptr(cases), len(cases), abi.ptr(out)), "gs_debug_numa_merge")
        return out

    def pair_probe(self, pods, nodes, pod_of, mode: int):
        """Diagnostics: (scores, cycles) of the commit kernel's pair evaluation on mirror rows (gs_debug_pair_probe)."""
        pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        pod_of = np.ascontiguousarray(pod_of, dtype=np.int32)
        n = len(nodes)
        scores = np.zeros(n * (64 if mode == 1 else 1), np.int32)
        cycles = np.zeros(10 * n, np.uint64)
        self._chk(lib().gs_debug_pair_probe(self._h, abi.ptr(pods), len(pods), abi.ptr(nodes), abi.ptr(pod_of), n, mode,
                                            abi.ptr(scores), abi.ptr(cycles)), "gs_debug_pair_probe")
        self.last_probe_stamps = cycles[2 * n:].reshape(n, 8).astype(np.int64)
        return (scores.reshape(n, 64) if mode == 1 else scores), cycles[:n], cycles[n:2 * n]

    def verify_cpusets(self, on: bool = True):
        """Re-run the host takeCPUs for every cpuset the commit kernel selects (schedule fails on a difference)."""
        self._chk(lib().gs_debug_verify_cpuset(self._h, int(on)), "gs_debug_verify_cpuset")


def unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    rc = lib().gs_comm_unique_id(buf)
    if rc != 0:
        raise GpuScoreError(f"gs_comm_unique_id failed: {rc}")
    return bytes(buf)
