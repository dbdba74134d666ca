"""Coscheduling gangs in front of the batched engine: the C-ABI gang manager (gs_gang_*, koordinator_amd/csrc/gs_gang.cpp,
the PodGroupManager of pkg/scheduler/plugins/coscheduling/core/core.go) and `schedule_with_gangs`, which gives the
reference's per-pod order of PreFilter -> node loop -> Reserve -> Permit (PostFilter on a failure, Unreserve of rejected
waiting pods) over batched gs_schedule calls.

Batching is speculative, like the quota gate: the gang transitions of a run of pods are computed in the library
(gs_gang_walk) assuming every pod that passes PreFilter finds a node; the engine then schedules the run's pods in one
call. The gang state is
then restored from the run's snapshot and the run replayed pod by pod with the real outcomes, checking the walk's
assumptions: the run stands while every pod's real PreFilter verdict is the walk's and no transition forgets an
assumed pod (a PostFilter or Unreserve rejecting waiting siblings, a Permit 'Gang not found'), since a forget changes
the node state under the run's later pods. At the first break the rest of the run is withdrawn (gs_pods_forget:
NodeInfo, podAssignCache and NUMA state exactly as before those pods) and the next run starts after that pod, so every
engine call sees the state the sequential order would. Pods left waiting at Permit can be carried to the next call
(WaitingPods)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi

STRICT, NONSTRICT = 0, 1
ONCE_SATISFIED, ONLY_WAITING, WAITING_AND_RUNNING = 0, 1, 2
PF_OK, PF_NOT_FOUND, PF_NOT_INIT, PF_NOT_ENOUGH, PF_CYCLE_INVALID, PF_CYCLE_TOO_LARGE = range(6)
PERMIT_SUCCESS, PERMIT_WAIT, PERMIT_NOT_FOUND = 0, 1, 2
# outcome of each pod of a scheduling pass
ST_UNSCHEDULABLE, ST_WAITING, ST_BOUND, ST_REJECTED = 0, 1, 2, 3

PREFILTER_MESSAGES = {   # core.go:221-272 (gang / pod names as GetId(namespace, name))
    PF_NOT_FOUND: "can't find gang, gangName: {gang}, podName: {pod}",
    PF_NOT_INIT: "gang has not init, gangName: {gang}, podName: {pod}",
    PF_NOT_ENOUGH: "gang child pod not collect enough, gangName: {gang}, podName: {pod}",
    PF_CYCLE_INVALID: "gang scheduleCycle not valid, gangName: {gang}, podName: {pod}",
    PF_CYCLE_TOO_LARGE: "pod's schedule cycle too large, gangName: {gang}, podName: {pod}, podCycle: {pcycle}, "
                        "gangCycle: {gcycle}",
}


def lib():
    return abi.load()


def spec(gang_id: int, min_member: int, total_children: int = -1, mode: int = -1, match_policy: int = -1,
         wait_time_ns: int = -1, group=(), create_time_ns: int = 0) -> abi.GsGangSpec:
    s = abi.GsGangSpec()
    s.gang_id, s.min_member, s.total_children, s.mode, s.match_policy = gang_id, min_member, total_children, mode, match_policy
    s.wait_time_ns, s.create_time_ns = wait_time_ns, create_time_ns
    s.group_n = len(group)
    for k, g in enumerate(group):
        s.group[k] = g
    return s


class GangManager:
    """ctypes handle of a gs_gang_mgr."""

    def __init__(self, default_timeout_ns: int | None = None, skip_check_schedule_cycle: bool = False, _h=None):
        if _h is not None:
            self._h = _h
            return
        a = abi.GsGangArgs()
        lib().gs_gang_args_default(C.byref(a))
        if default_timeout_ns is not None:
            a.default_timeout_ns = default_timeout_ns
        a.skip_check_schedule_cycle = int(skip_check_schedule_cycle)
        h = C.c_void_p()
        self._chk(lib().gs_gang_mgr_create(C.byref(a), C.byref(h)), "gs_gang_mgr_create")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib().gs_gang_mgr_destroy(self._h)
            self._h = None

    @staticmethod
    def _chk(rc, what):
        if rc < 0:
            raise RuntimeError(f"{what}: rc={rc}")
        return rc

    def clone(self) -> "GangManager":
        h = C.c_void_p()
        self._chk(lib().gs_gang_mgr_clone(self._h, C.byref(h)), "gs_gang_mgr_clone")
        return GangManager(_h=h)

    def assign(self, other: "GangManager"):
        self._chk(lib().gs_gang_mgr_assign(self._h, other._h), "gs_gang_mgr_assign")

    def podgroup_upsert(self, s: abi.GsGangSpec):
        self._chk(lib().gs_gang_podgroup_upsert(self._h, C.byref(s)), "gs_gang_podgroup_upsert")

    def podgroup_delete(self, gang_id: int):
        self._chk(lib().gs_gang_podgroup_delete(self._h, gang_id), "gs_gang_podgroup_delete")

    def pod_add(self, gang_id: int, uid: int, assigned: bool = False, annot: abi.GsGangSpec | None = None):
        self._chk(lib().gs_gang_pod_add(self._h, gang_id, uid, int(assigned), C.byref(annot) if annot else None),
                  "gs_gang_pod_add")

    def pod_delete(self, gang_id: int, uid: int):
        self._chk(lib().gs_gang_pod_delete(self._h, gang_id, uid), "gs_gang_pod_delete")

    def prefilter(self, gang_id: int, uid: int, nominated: bool = False) -> int:
        return self._chk(lib().gs_gang_prefilter(self._h, gang_id, uid, int(nominated)), "gs_gang_prefilter")

    def _list_call(self, fn, *args):
        cap = 64
        while True:
            buf = np.zeros(cap, np.uint64)
            n = C.c_uint32(0)
            rc = fn(self._h, *args, abi.ptr(buf), cap, C.byref(n))
            if rc == abi.GS_EINVAL and n.value > cap:
                cap = n.value
                continue
            self._chk(rc, fn.__name__)
            return rc, [int(x) for x in buf[:n.value]]

    def permit(self, gang_id: int, uid: int, now_ns: int):
        w = C.c_int64(0)
        rc, allowed = self._list_call(lambda h, *a: lib().gs_gang_permit(h, gang_id, uid, now_ns, C.byref(w), *a))
        return rc, int(w.value), allowed

    def post_bind(self, gang_id: int, uid: int):
        self._chk(lib().gs_gang_post_bind(self._h, gang_id, uid), "gs_gang_post_bind")

    def post_filter(self, gang_id: int, uid: int) -> list[int]:
        return self._list_call(lambda h, *a: lib().gs_gang_post_filter(h, gang_id, uid, *a))[1]

    def unreserve(self, gang_id: int, uid: int) -> list[int]:
        return self._list_call(lambda h, *a: lib().gs_gang_unreserve(h, gang_id, uid, *a))[1]

    def expire(self, now_ns: int) -> list[int]:
        return self._list_call(lambda h, *a: lib().gs_gang_expire(h, now_ns, *a))[1]

    def waiting_pods(self) -> list[int]:
        return self._list_call(lambda h, *a: lib().gs_gang_waiting_pods(h, *a))[1]

    def info(self, gang_id: int):
        out = abi.GsGangInfo()
        rc = self._chk(lib().gs_gang_get(self._h, gang_id, C.byref(out)), "gs_gang_get")
        return {f: getattr(out, f) for f, _ in abi.GsGangInfo._fields_ if f != "pad"} if rc == 1 else None

    def debug_set(self, gang_id: int, uid: int, what: int, value: int):
        self._chk(lib().gs_gang_debug_set(self._h, gang_id, uid, what, value), "gs_gang_debug_set")

    def child_cycle(self, gang_id: int, uid: int) -> int:
        return lib().gs_gang_child_cycle(self._h, gang_id, uid)


class WaitingPods:
    """Pods left waiting at Permit by earlier passes (the framework's waiting pods): uid -> (gang, node, pod record).
    Pass the same object to consecutive schedule_with_gangs calls so that a gang spanning several calls is allowed,
    rejected or forgotten exactly as in one long queue."""

    def __init__(self):
        self.pods: dict[int, tuple[int, int, np.void]] = {}


class _Pass:
    """The per-pod transitions of one scheduling pass (shared by the speculative walk and the replay)."""

    def __init__(self, engine, mgr, pods, gang_ids, nominated, now_ns, waiting=None):
        self.engine, self.mgr, self.pods, self.gang, self.nom, self.now = engine, mgr, pods, gang_ids, nominated, now_ns
        n = len(pods)
        self.uid_index = {int(u): k for k, u in enumerate(pods["uid"])}
        self.node = np.full(n, -1, np.int32)           # the node a pod is assumed / bound on
        self.state = np.full(n, ST_UNSCHEDULABLE, np.int8)
        self.prefilter = np.zeros(n, np.int8)
        self.permit = np.full(n, -1, np.int8)
        self.waiting = waiting if waiting is not None else WaitingPods()   # pods waiting from earlier passes
        self.carried = {}                                                    # their uid -> new state

    def gang_of(self, uid: int) -> int:
        k = self.uid_index.get(uid)
        return int(self.gang[k]) if k is not None else self.waiting.pods[uid][0]

    def bind(self, uid: int):
        """PostBind of a pod Permit allowed (this pass's, or one waiting from an earlier pass)."""
        k = self.uid_index.get(uid)
        if k is not None:
            self.state[k] = ST_BOUND
        else:
            self.carried[uid] = ST_BOUND
        self.mgr.post_bind(self.gang_of(uid), uid)

    def unreserve_chain(self, rejected, forget: bool):
        """Rejected waiting pods: Unreserve (gang) + ForgetPod on the engine, and the rejections that follow."""
        queue = list(rejected)
        nodes, recs = [], []   # one ForgetPod call for the whole chain (nothing is scheduled in between)
        while queue:
            uid = queue.pop(0)
            k = self.uid_index.get(uid)
            if k is not None:
                nodes.append(int(self.node[k]))
                recs.append(self.pods[k])
                self.state[k] = ST_REJECTED
            else:
                g, node, rec = self.waiting.pods[uid]
                nodes.append(node)
                recs.append(rec)
                self.carried[uid] = ST_REJECTED
            queue.extend(self.mgr.unreserve(self.gang_of(uid), uid))
        if forget and nodes:
            self.engine.forget(np.array(nodes, np.uint32), np.array(recs, abi.POD_DTYPE))

    def before_node_loop(self, k) -> tuple[bool, list[int]]:
        """PreFilter; on a rejection its PostFilter. (passes, waiting pods the PostFilter rejected)"""
        g, uid = int(self.gang[k]), int(self.pods["uid"][k])
        code = self.mgr.prefilter(g, uid, bool(self.nom[k]))
        self.prefilter[k] = code
        if code == PF_OK:
            return True, []
        return False, self.mgr.post_filter(g, uid)

    def after_node_loop(self, k, node) -> list[int]:
        """A FitError's PostFilter, or Reserve + Permit (+ the binds Permit allows); returns pods to Unreserve."""
        g, uid = int(self.gang[k]), int(self.pods["uid"][k])
        if node < 0:
            return self.mgr.post_filter(g, uid)
        self.node[k] = node
        st, _, allowed = self.mgr.permit(g, uid, self.now)
        self.permit[k] = st
        if st == PERMIT_SUCCESS:
            self.state[k] = ST_BOUND
            self.mgr.post_bind(g, uid)
            for a in allowed:
                self.bind(a)
            return []
        if st == PERMIT_WAIT:
            self.state[k] = ST_WAITING
            return []
        # "Gang not found": the pod's Permit fails, its Reserve is undone (it is not a waiting pod)
        self.state[k] = ST_REJECTED
        return [uid]


def schedule_with_gangs(engine, mgr: GangManager, pods, gang_ids, seq=None, nominated=None, now_ns: int = 0,
                        run_cap: int = 192, waiting: WaitingPods | None = None):
    """Schedules `pods` in queue order with Coscheduling's PreFilter / Permit / PostFilter / Unreserve around every pod,
    through batched engine calls (engine: Engine or the oracle's Oracle: schedule(pods, seq), forget(nodes, pods)).
    gang_ids[i]: the pod's gang key (0: no gang). Returns (placements, result) where result holds per pod the gang
    PreFilter code, the Permit status (-1: none), the final state (ST_*) and the node it is assumed / bound on.

    The per-pod gate loop runs in the library (gs_gang_walk / gs_gang_replay over a gs_gang_pass): one walk and one
    replay call per engine call; this function only moves the runs through the engine and forgets withdrawn pods.

    run_cap bounds a run (pods per engine call). A run that breaks (a gang verdict the walk could not foresee) withdraws
    every pod after the break, so long runs schedule and forget many pods twice: on the C3 bench queue (a break every
    ~370 pods) 192 gives 82k decided pods/s against 23k at 4096 (scripts/bench_gang.py --run-cap)."""
    pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
    n = len(pods)
    gang_ids = np.ascontiguousarray(gang_ids, np.uint64)
    seq = np.arange(n, dtype=np.uint64) if seq is None else np.ascontiguousarray(seq, dtype=np.uint64)
    nom = np.zeros(n, np.uint8) if nominated is None else np.ascontiguousarray(nominated, np.uint8)
    waiting = waiting if waiting is not None else WaitingPods()
    uids = np.ascontiguousarray(pods["uid"], np.uint64)
    prefilter = np.zeros(n, np.int8)
    permit = np.full(n, -1, np.int8)
    state = np.zeros(n, np.int8)
    node = np.full(n, -1, np.int32)
    L = lib()
    h = C.c_void_p()
    GangManager._chk(L.gs_gang_pass_create(mgr._h, n, abi.ptr(gang_ids), abi.ptr(uids), abi.ptr(nom), now_ns,
                                           abi.ptr(prefilter), abi.ptr(permit), abi.ptr(state), abi.ptr(node),
                                           C.byref(h)), "gs_gang_pass_create")
    out = np.zeros(n, abi.PLACEMENT_DTYPE)
    out["node"] = -1
    run = np.zeros(max(1, min(run_cap, n)), np.uint32)
    fbuf = np.zeros(n + len(waiting.pods) + 1, np.uint64)
    index = {}

    def where(uid: int):
        """the node and pod record of a pod to forget: this queue's, or one waiting from an earlier pass"""
        if not index:
            index.update((int(u), k) for k, u in enumerate(uids))
        k = index.get(uid)
        if k is not None:
            return int(node[k]), pods[k]
        _, nd, rec = waiting.pods[uid]
        return nd, rec

    def forget(nodes, recs):
        """ForgetPod of the withdrawn run pods (node array / pod records given) and of the pods the Unreserve chains
        rejected"""
        cnt = C.c_uint32(0)
        GangManager._chk(L.gs_gang_pass_forgets(h, abi.ptr(fbuf), len(fbuf), C.byref(cnt)), "gs_gang_pass_forgets")
        if cnt.value:
            more = [where(int(u)) for u in fbuf[:cnt.value]]
            nodes = np.concatenate([nodes, np.array([x[0] for x in more], np.uint32)])
            recs = np.concatenate([recs, np.array([x[1] for x in more], abi.POD_DTYPE)])
        if len(nodes):
            engine.forget(np.ascontiguousarray(nodes, np.uint32), np.ascontiguousarray(recs, abi.POD_DTYPE))

    try:
        i = 0
        rn, j, r_stop, j_next, single = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_int32()
        while i < n:
            GangManager._chk(L.gs_gang_walk(h, i, run_cap, abi.ptr(run), C.byref(rn), C.byref(j)), "gs_gang_walk")
            r = run[:rn.value].astype(np.int64)
            got = engine.schedule(pods[r], seq[r]) if len(r) else np.zeros(0, abi.PLACEMENT_DTYPE)
            got_node = np.ascontiguousarray(got["node"], np.int32)
            GangManager._chk(L.gs_gang_replay(h, i, j.value, abi.ptr(run), rn.value, abi.ptr(got_node),
                                              C.byref(r_stop), C.byref(j_next), C.byref(single)), "gs_gang_replay")
            kept = r_stop.value
            out[r[:kept]] = got[:kept]
            later = kept + np.flatnonzero(got_node[kept:] >= 0)   # the run's withdrawn placements
            forget(got_node[later].astype(np.uint32), pods[r[later]])
            if single.value >= 0:   # the walk's PreFilter failed where the real one passes: this pod alone
                k = single.value
                one = engine.schedule(pods[k:k + 1], seq[k:k + 1])
                out[k] = one[0]
                GangManager._chk(L.gs_gang_pass_after_single(h, k, int(one["node"][0])), "gs_gang_pass_after_single")
                forget(np.zeros(0, np.uint32), np.zeros(0, abi.POD_DTYPE))
            i = j_next.value
        cnt = C.c_uint32(0)
        cu = np.zeros(max(1, 2 * (n + len(waiting.pods))), np.uint64)
        cs = np.zeros(len(cu), np.int8)
        GangManager._chk(L.gs_gang_pass_carried(h, abi.ptr(cu), abi.ptr(cs), len(cu), C.byref(cnt)),
                         "gs_gang_pass_carried")
        carried = {int(u): int(x) for u, x in zip(cu[:cnt.value], cs[:cnt.value])}
    finally:
        L.gs_gang_pass_destroy(h)
    # the waiting set after this pass: earlier pods that were allowed or rejected leave it, this pass's waiting join
    for uid in carried:
        waiting.pods.pop(uid, None)
    for k in np.flatnonzero(state == ST_WAITING):
        waiting.pods[int(uids[k])] = (int(gang_ids[k]), int(node[k]), pods[k].copy())
    return out, {"prefilter": prefilter, "permit": permit, "state": state, "node": node, "carried": carried}


def expire(engine, mgr: GangManager, pods, gang_ids, node, state, now_ns: int, waiting: WaitingPods | None = None):
    """The framework's Permit timeout at now_ns after a pass: waiting pods past their deadline are rejected, their
    Unreserve and ForgetPod run (and the rejections Strict gangs add). Updates state in place; returns the new states
    of pods waiting from earlier passes (`waiting`, which is updated too)."""
    pods = np.ascontiguousarray(pods, dtype=abi.POD_DTYPE)
    P = _Pass(engine, mgr, pods, np.asarray(gang_ids, np.uint64), np.zeros(len(pods), bool), now_ns, waiting)
    P.node[:], P.state[:] = node, state
    P.unreserve_chain(mgr.expire(now_ns), forget=True)
    state[:] = P.state
    for uid in P.carried:
        P.waiting.pods.pop(uid, None)
    for k in np.flatnonzero(P.state == ST_REJECTED):
        P.waiting.pods.pop(int(pods["uid"][k]), None)
    return dict(P.carried)
