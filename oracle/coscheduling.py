"""TEST INFRASTRUCTURE (the checker, never the product): a Python restatement of Coscheduling's PodGroupManager and its
gang cache (pkg/scheduler/plugins/coscheduling/core/core.go, gang.go, gang_cache.go) and the reference's per-pod order
around one scheduling cycle, over the oracle engine one pod at a time. Used by tests/ to check the library's gs_gang_*
manager and koordinator_amd/gang.py's batched driver.

Pinned by the reference's own vectors (tests/test_gang.py: core_test.go TestPlugin_PreFilter and TestPermit)."""
from __future__ import annotations

import numpy as np

STRICT, NONSTRICT = 0, 1
ONCE_SATISFIED, ONLY_WAITING, WAITING_AND_RUNNING = 0, 1, 2
PF_OK, PF_NOT_FOUND, PF_NOT_INIT, PF_NOT_ENOUGH, PF_CYCLE_INVALID, PF_CYCLE_TOO_LARGE = range(6)
PERMIT_SUCCESS, PERMIT_WAIT, PERMIT_NOT_FOUND = 0, 1, 2
ST_UNSCHEDULABLE, ST_WAITING, ST_BOUND, ST_REJECTED = 0, 1, 2, 3


class Gang:
    """gang.go:44-110 (NewGang's defaults)."""

    def __init__(self, gid):
        self.id = gid
        self.wait_time = 0
        self.mode = STRICT
        self.min = 0
        self.total = 0
        self.group = [gid]
        self.children = set()
        self.waiting = set()          # WaitingForBindChildren
        self.bound = set()            # BoundChildren
        self.once = False             # OnceResourceSatisfied
        self.policy = ONCE_SATISFIED
        self.cycle_valid = True
        self.cycle = 1
        self.child_cycle = {}         # ChildrenScheduleRoundMap
        self.from_annotation = True
        self.has_init = False

    def init(self, s: dict, from_podgroup: bool, default_timeout: int):
        """tryInitByPodGroup (gang.go:180-232) / tryInitByPodConfig (gang.go:112-178) on decoded fields."""
        self.min = s["min_member"]
        total = s.get("total_children", -1)
        if total < 0:   # strconv.ParseInt error
            total = self.min
        elif total != 0 and total < self.min:
            total = self.min
        self.total = total
        mode = s.get("mode", -1)
        self.mode = mode if mode in (STRICT, NONSTRICT) else STRICT
        pol = s.get("match_policy", -1)
        self.policy = pol if pol in (ONLY_WAITING, WAITING_AND_RUNNING, ONCE_SATISFIED) else ONCE_SATISFIED
        w = s.get("wait_time_ns", -1)
        # GetWaitTimeDuration: ScheduleTimeoutSeconds >= 0; time.ParseDuration(annotation) > 0
        self.wait_time = w if (w >= 0 if from_podgroup else w > 0) else default_timeout
        self.group = list(s.get("group", ())) or [s["gang_id"]]
        self.from_annotation = not from_podgroup
        self.has_init = True

    def valid_for_permit(self):   # isGangValidForPermit (gang.go:480-496)
        if not self.has_init:
            return False
        if self.policy == ONLY_WAITING:
            return len(self.waiting) >= self.min
        if self.policy == WAITING_AND_RUNNING:
            return len(self.waiting) + len(self.bound) >= self.min
        return len(self.waiting) >= self.min or self.once

    def add_bound(self, uid):     # addBoundPod (gang.go:466-477)
        self.waiting.discard(uid)
        self.bound.add(uid)
        if len(self.bound) >= self.min:
            self.once = True


class PodGroupManager:
    def __init__(self, default_timeout_ns=600 * 10**9, skip_check_schedule_cycle=False):
        self.default_timeout = default_timeout_ns
        self.skip = skip_check_schedule_cycle
        self.gangs: dict[int, Gang] = {}
        self.fw_waiting: dict[int, tuple[int, int]] = {}   # the framework's waiting pods: uid -> (gang, deadline)

    def gang(self, gid, create=False):
        if gid not in self.gangs and create:
            self.gangs[gid] = Gang(gid)
        return self.gangs.get(gid)

    # ---- gang cache event handlers (gang_cache.go)
    def podgroup_upsert(self, s: dict):
        self.gang(s["gang_id"], True).init(s, True, self.default_timeout)

    def podgroup_delete(self, gid):
        self.gangs.pop(gid, None)

    def pod_add(self, gid, uid, assigned=False, annot: dict | None = None):
        g = self.gang(gid, True)
        if annot is not None and not g.has_init and annot["min_member"] >= 0:
            g.init(annot, False, self.default_timeout)
        g.children.add(uid)
        if assigned:
            g.add_bound(uid)
            g.once = True

    def pod_delete(self, gid, uid):
        g = self.gang(gid)
        if g is None:
            return
        for s in (g.children, g.waiting, g.bound):
            s.discard(uid)
        g.child_cycle.pop(uid, None)
        self.fw_waiting.pop(uid, None)
        if g.from_annotation and not g.children:
            del self.gangs[gid]

    # ---- PodGroupManager (core.go)
    def prefilter(self, gid, uid, nominated=False):
        if not gid:
            return PF_OK
        g = self.gang(gid)
        if g is None:
            return PF_NOT_FOUND
        if not g.has_init:
            return PF_NOT_INIT
        if g.policy == ONCE_SATISFIED and g.once:
            return PF_OK
        if len(g.children) < g.min:
            return PF_NOT_ENOUGH
        if self.skip:
            return PF_OK
        if sum(1 for c in g.child_cycle.values() if c == g.cycle) == g.total:   # trySetScheduleCycleValid
            g.cycle_valid = True
            g.cycle += 1
        gcycle = g.cycle
        try:
            if g.mode == STRICT:
                if nominated:
                    return PF_OK
                if not g.cycle_valid:
                    return PF_CYCLE_INVALID
                if g.child_cycle.get(uid, 0) >= gcycle:
                    return PF_CYCLE_TOO_LARGE
            return PF_OK
        finally:
            g.child_cycle[uid] = gcycle   # defer setChildScheduleCycle

    def _reject_group(self, gid):
        g = self.gang(gid)
        if g is None:
            return []
        grp = set(g.group)
        rej = sorted(u for u, (pg, _) in self.fw_waiting.items() if pg in grp)
        for u in rej:
            del self.fw_waiting[u]
        if rej:
            for x in grp:
                if x in self.gangs:
                    self.gangs[x].cycle_valid = False
        return rej

    def permit(self, gid, uid, now):
        if not gid:
            return PERMIT_SUCCESS, 0, []
        g = self.gang(gid)
        if g is None:
            return PERMIT_NOT_FOUND, 0, []
        g.waiting.add(uid)
        for x in g.group:
            gx = self.gang(x)
            if gx is None or not gx.valid_for_permit():
                self.fw_waiting[uid] = (gid, now + g.wait_time)
                return PERMIT_WAIT, g.wait_time, []
        grp = set(g.group)
        allowed = sorted(u for u, (pg, _) in self.fw_waiting.items() if pg in grp)
        for u in allowed:
            del self.fw_waiting[u]
        return PERMIT_SUCCESS, 0, allowed

    def post_bind(self, gid, uid):
        g = self.gang(gid) if gid else None
        if g is not None:
            g.add_bound(uid)

    def post_filter(self, gid, uid):
        g = self.gang(gid) if gid else None
        if g is None or (g.policy == ONCE_SATISFIED and g.once):
            return []
        return self._reject_group(gid) if g.mode == STRICT else []

    def unreserve(self, gid, uid):
        g = self.gang(gid) if gid else None
        if g is None:
            return []
        g.waiting.discard(uid)
        self.fw_waiting.pop(uid, None)
        if not (g.policy == ONCE_SATISFIED and g.once) and g.mode == STRICT:
            return self._reject_group(gid)
        return []

    def expire(self, now):
        rej = sorted(u for u, (_, d) in self.fw_waiting.items() if d <= now)
        for u in rej:
            del self.fw_waiting[u]
        return rej


def schedule_sequential(engine, mgr: PodGroupManager, pods, gang_ids, seq=None, nominated=None, now_ns=0):
    """The reference's order, one pod at a time: PreFilter (gang) -> the node loop on the oracle engine -> Reserve ->
    Permit, PostFilter after a failure, Unreserve + ForgetPod of every rejected waiting pod."""
    n = len(pods)
    seq = np.arange(n, dtype=np.uint64) if seq is None else np.asarray(seq, np.uint64)
    nominated = np.zeros(n, bool) if nominated is None else np.asarray(nominated, bool)
    from koordinator_amd import abi
    out = np.zeros(n, abi.PLACEMENT_DTYPE)
    out["node"] = -1
    res = {"prefilter": np.zeros(n, np.int8), "permit": np.full(n, -1, np.int8),
           "state": np.full(n, ST_UNSCHEDULABLE, np.int8), "node": np.full(n, -1, np.int32)}
    idx = {int(u): k for k, u in enumerate(pods["uid"])}

    def unreserve_all(rej):
        q = list(rej)
        while q:
            u = q.pop(0)
            k = idx[u]
            engine.forget([res["node"][k]], pods[k:k + 1])
            res["state"][k] = ST_REJECTED
            q.extend(mgr.unreserve(int(gang_ids[k]), u))

    for k in range(n):
        g, uid = int(gang_ids[k]), int(pods["uid"][k])
        code = mgr.prefilter(g, uid, bool(nominated[k]))
        res["prefilter"][k] = code
        if code != PF_OK:
            unreserve_all(mgr.post_filter(g, uid))
            continue
        r = engine.schedule(pods[k:k + 1], seq[k:k + 1])
        out[k] = r[0]
        node = int(r["node"][0])
        if node < 0:
            unreserve_all(mgr.post_filter(g, uid))
            continue
        res["node"][k] = node
        st, _, allowed = mgr.permit(g, uid, now_ns)
        res["permit"][k] = st
        if st == PERMIT_SUCCESS:
            res["state"][k] = ST_BOUND
            mgr.post_bind(g, uid)
            for a in allowed:
                res["state"][idx[a]] = ST_BOUND
                mgr.post_bind(int(gang_ids[idx[a]]), a)
        elif st == PERMIT_WAIT:
            res["state"][k] = ST_WAITING
        else:
            unreserve_all([uid])
    return out, res
