// gs_gang.cpp — Coscheduling's gang state: the PodGroupManager of
// pkg/scheduler/plugins/coscheduling/core/core.go over the gang cache (gang.go, gang_cache.go), as host state of the
// library. It touches no node: PreFilter is a per-pod gate in front of gs_schedule, Permit / PostFilter / Unreserve
// decide which assumed pods wait, bind or are rejected, and the caller undoes a rejected pod's Reserve with
// gs_pods_forget (koordinator_amd/gang.py drives both in the reference's per-pod order over batched gs_schedule calls).
//
// Keys: a gang is GetId(namespace, name) and a pod its UID, both as the caller's 64-bit keys. The framework's waiting
// pods (framework.WaitingPod, the pods that got Wait at Permit) of gang pods are tracked here with their Permit deadline.
// Where the reference iterates a Go map (IterateOverWaitingPods), pods are visited in UID order; no result depends on it.
#include <algorithm>
#include <cstring>
#include <deque>
#include <map>
#include <optional>
#include <memory>
#include <set>
#include <unordered_map>
#include <vector>

#include "../../include/gpuscore.h"

namespace {

struct Gang {
  bool has_init = false;
  int min = 0, total = 0;
  int mode = GS_GANG_STRICT;
  int policy = GS_GANG_ONCE_SATISFIED;
  int64_t wait_ns = 0;
  int64_t create_ns = 0;
  std::vector<uint64_t> group;
  bool from_annotation = true;   // GangFromPodAnnotation (NewGang's default)
  std::set<uint64_t> children, waiting, bound;   // Children, WaitingForBindChildren, BoundChildren
  bool once = false;             // OnceResourceSatisfied
  bool cycle_valid = true;       // ScheduleCycleValid
  int cycle = 1;                 // ScheduleCycle
  std::unordered_map<uint64_t, int> child_cycle;   // ChildrenScheduleRoundMap

  bool valid_for_permit() const {   // isGangValidForPermit (gang.go:480-496)
    if (!has_init) return false;
    const int w = (int)waiting.size(), b = (int)bound.size();
    if (policy == GS_GANG_ONLY_WAITING) return w >= min;
    if (policy == GS_GANG_WAITING_AND_RUNNING) return w + b >= min;
    return w >= min || once;
  }
  void add_bound(uint64_t uid) {    // addBoundPod (gang.go:466-477)
    waiting.erase(uid);
    bound.insert(uid);
    if ((int)bound.size() >= min) once = true;
  }
};

}  // namespace

struct gs_gang_mgr {
  gs_gang_args args{};
  std::map<uint64_t, Gang> gangs;
  std::map<uint64_t, std::pair<uint64_t, int64_t>> fw_waiting;   // pod uid -> (gang id, Permit deadline)

  Gang* get(uint64_t id, bool create) {   // getGangFromCacheByGangId (gang_cache.go:48-63) + NewGang (gang.go:92-110)
    if (snap_on) snap_touch(id);   // a speculative walk: the gang's state before its first access is kept
    auto it = gangs.find(id);
    if (it != gangs.end()) return &it->second;
    if (!create) return nullptr;
    Gang& g = gangs[id];
    g.group = {id};
    return &g;
  }
  // The framework's waiting pods of the gang group of `id` (uid order), with their gangs
  void group_waiting(const Gang& g, std::vector<std::pair<uint64_t, uint64_t>>* out) const {
    const std::set<uint64_t> grp(g.group.begin(), g.group.end());
    for (const auto& kv : fw_waiting)
      if (grp.count(kv.second.first)) out->push_back({kv.first, kv.second.first});
  }
  // rejectGangGroupById (core.go:363-394): the waiting pods of the gang group are rejected (their Unreserve follows)
  void reject_group(uint64_t id, std::vector<std::pair<uint64_t, uint64_t>>* out) {
    Gang* g = get(id, false);
    if (!g) return;
    const size_t n0 = out->size();
    group_waiting(*g, out);
    if (out->size() == n0) return;
    for (size_t k = n0; k < out->size(); ++k) fw_waiting.erase((*out)[k].first);
    for (uint64_t gid : g->group)
      if (Gang* x = get(gid, false)) x->cycle_valid = false;
  }
  // (uid, gang) lists of the operations below: the pods Permit allows / a rejection lists
  using List = std::vector<std::pair<uint64_t, uint64_t>>;
  int prefilter(uint64_t gang_id, uint64_t uid, bool nominated);
  int permit(uint64_t gang_id, uint64_t uid, int64_t now_ns, int64_t* wait_ns, List* allowed);
  void post_bind(uint64_t gang_id, uint64_t uid) {
    if (!gang_id) return;
    if (Gang* g = get(gang_id, false)) g->add_bound(uid);
  }
  void post_filter(uint64_t gang_id, List* rejected);
  void unreserve(uint64_t gang_id, uint64_t uid, List* rejected);
  // sizes of the lists these would return, without changing anything
  size_t permit_allows(uint64_t gang_id, uint64_t uid) const;
  size_t post_filter_rejects(uint64_t gang_id) const;
  size_t unreserve_rejects(uint64_t gang_id, uint64_t uid) const;
  // gs_gang_pass: the state a speculative walk is replayed from, copied on first access per gang (every mutation goes
  // through get()) instead of the whole cache per walk, and the framework's waiting pods (a short map)
  bool snap_on = false;
  std::unordered_map<uint64_t, std::optional<Gang>> snap_gangs;   // nullopt: the gang did not exist
  std::map<uint64_t, std::pair<uint64_t, int64_t>> snap_fw;
  void snap_touch(uint64_t id) {
    if (snap_gangs.count(id)) return;
    auto it = gangs.find(id);
    snap_gangs.emplace(id, it == gangs.end() ? std::nullopt : std::optional<Gang>(it->second));
  }
  void snap_begin() {
    snap_gangs.clear();
    snap_fw = fw_waiting;
    snap_on = true;
  }
  void snap_restore() {
    for (auto& kv : snap_gangs) {
      if (kv.second) gangs[kv.first] = std::move(*kv.second);
      else gangs.erase(kv.first);
    }
    fw_waiting = std::move(snap_fw);
    snap_gangs.clear();
    snap_on = false;
  }
};

namespace {

int copy_out(const std::vector<uint64_t>& v, uint64_t* out, uint32_t cap, uint32_t* n) {
  if (n) *n = (uint32_t)v.size();
  if (v.size() > cap) return GS_EINVAL;
  if (out)
    for (size_t k = 0; k < v.size(); ++k) out[k] = v[k];
  return GS_OK;
}

// tryInitByPodGroup (gang.go:180-232) / tryInitByPodConfig (gang.go:112-178) on a decoded spec
void init_gang(Gang& g, const gs_gang_spec& s, bool from_podgroup, int64_t default_timeout) {
  g.min = s.min_member;
  int64_t total = s.total_children;
  if (total < 0 || (total != 0 && total < g.min)) total = g.min;   // unparsable, or below the minimum
  g.total = (int)total;
  g.mode = (s.mode == GS_GANG_NONSTRICT) ? GS_GANG_NONSTRICT : GS_GANG_STRICT;
  g.policy = (s.match_policy == GS_GANG_ONLY_WAITING || s.match_policy == GS_GANG_WAITING_AND_RUNNING)
                 ? s.match_policy
                 : GS_GANG_ONCE_SATISFIED;
  g.create_ns = s.create_time_ns;
  // GetWaitTimeDuration: ScheduleTimeoutSeconds >= 0 (PodGroup); the annotation's duration when > 0
  const bool ok_wait = from_podgroup ? s.wait_time_ns >= 0 : s.wait_time_ns > 0;
  g.wait_ns = ok_wait ? s.wait_time_ns : default_timeout;
  g.group.clear();
  for (uint32_t k = 0; k < s.group_n && k < GS_GANG_GROUP_MAX; ++k) g.group.push_back(s.group[k]);
  if (g.group.empty()) g.group.push_back(s.gang_id);
  g.from_annotation = !from_podgroup;
  g.has_init = true;
}

}  // namespace

int gs_gang_mgr::prefilter(uint64_t gang_id, uint64_t uid, bool nominated) {   // core.go:221-272
  if (!gang_id) return GS_GANG_PREFILTER_OK;
  Gang* g = get(gang_id, false);
  if (!g) return GS_GANG_PREFILTER_NOT_FOUND;
  if (!g->has_init) return GS_GANG_PREFILTER_NOT_INIT;
  if (g->policy == GS_GANG_ONCE_SATISFIED && g->once) return GS_GANG_PREFILTER_OK;
  if ((int)g->children.size() < g->min) return GS_GANG_PREFILTER_NOT_ENOUGH_CHILDREN;
  if (args.skip_check_schedule_cycle) return GS_GANG_PREFILTER_OK;
  {   // trySetScheduleCycleValid (gang.go:435-452)
    int num = 0;
    for (const auto& kv : g->child_cycle) num += kv.second == g->cycle;
    if (num == g->total) {
      g->cycle_valid = true;
      g->cycle += 1;
    }
  }
  const int gcycle = g->cycle;
  int rc = GS_GANG_PREFILTER_OK;
  if (g->mode == GS_GANG_STRICT && !nominated) {
    auto it = g->child_cycle.find(uid);
    const int pcycle = it == g->child_cycle.end() ? 0 : it->second;
    if (!g->cycle_valid) rc = GS_GANG_PREFILTER_CYCLE_INVALID;
    else if (pcycle >= gcycle) rc = GS_GANG_PREFILTER_CYCLE_TOO_LARGE;
  }
  g->child_cycle[uid] = gcycle;   // the deferred setChildScheduleCycle
  return rc;
}

// core.go:312-339 + AllowGangGroup (core.go:488-508)
int gs_gang_mgr::permit(uint64_t gang_id, uint64_t uid, int64_t now_ns, int64_t* wait_ns, List* allowed) {
  if (!gang_id) return GS_GANG_PERMIT_SUCCESS;
  Gang* g = get(gang_id, false);
  if (!g) return GS_GANG_PERMIT_NOT_FOUND;
  g->waiting.insert(uid);   // addAssumedPod
  for (uint64_t gid : g->group) {
    const Gang* x = get(gid, false);
    if (!x || !x->valid_for_permit()) {
      if (wait_ns) *wait_ns = g->wait_ns;
      fw_waiting[uid] = {gang_id, now_ns + g->wait_ns};
      return GS_GANG_PERMIT_WAIT;
    }
  }
  const size_t n0 = allowed->size();
  group_waiting(*g, allowed);
  for (size_t k = n0; k < allowed->size(); ++k) fw_waiting.erase((*allowed)[k].first);
  return GS_GANG_PERMIT_SUCCESS;
}

size_t gs_gang_mgr::permit_allows(uint64_t gang_id, uint64_t uid) const {
  if (!gang_id) return 0;
  auto it = gangs.find(gang_id);
  if (it == gangs.end()) return 0;
  Gang g = it->second;   // the permit's own addAssumedPod, on a copy
  g.waiting.insert(uid);
  for (uint64_t gid : g.group) {
    const Gang* x = nullptr;
    if (gid == gang_id) x = &g;
    else if (auto jt = gangs.find(gid); jt != gangs.end()) x = &jt->second;
    if (!x || !x->valid_for_permit()) return 0;
  }
  List l;
  group_waiting(g, &l);
  return l.size();
}

void gs_gang_mgr::post_filter(uint64_t gang_id, List* rejected) {   // core.go:277-307
  if (!gang_id) return;
  Gang* g = get(gang_id, false);
  if (!g) return;
  if (g->policy == GS_GANG_ONCE_SATISFIED && g->once) return;
  if (g->mode == GS_GANG_STRICT) reject_group(gang_id, rejected);
}

size_t gs_gang_mgr::post_filter_rejects(uint64_t gang_id) const {
  if (!gang_id) return 0;
  auto it = gangs.find(gang_id);
  if (it == gangs.end()) return 0;
  const Gang& g = it->second;
  if ((g.policy == GS_GANG_ONCE_SATISFIED && g.once) || g.mode != GS_GANG_STRICT) return 0;
  List l;
  group_waiting(g, &l);
  return l.size();
}

void gs_gang_mgr::unreserve(uint64_t gang_id, uint64_t uid, List* rejected) {   // core.go:344-361
  if (!gang_id) return;
  Gang* g = get(gang_id, false);
  if (!g) return;
  g->waiting.erase(uid);   // delAssumedPod
  fw_waiting.erase(uid);
  if (!(g->policy == GS_GANG_ONCE_SATISFIED && g->once) && g->mode == GS_GANG_STRICT) reject_group(gang_id, rejected);
}

size_t gs_gang_mgr::unreserve_rejects(uint64_t gang_id, uint64_t uid) const {
  if (!gang_id) return 0;
  auto it = gangs.find(gang_id);
  if (it == gangs.end()) return 0;
  const Gang& g = it->second;
  if ((g.policy == GS_GANG_ONCE_SATISFIED && g.once) || g.mode != GS_GANG_STRICT) return 0;
  List l;
  group_waiting(g, &l);
  size_t n = 0;
  for (const auto& e : l) n += e.first != uid;
  return n;
}

extern "C" {

void gs_gang_args_default(gs_gang_args* a) {
  if (!a) return;
  std::memset(a, 0, sizeof(*a));
  a->default_timeout_ns = 600LL * 1000000000LL;   // CoschedulingArgs.DefaultTimeout (config/v1beta2/defaults.go: 600 s)
}

int gs_gang_mgr_create(const gs_gang_args* args, gs_gang_mgr** out) {
  if (!out) return GS_EINVAL;
  auto* m = new gs_gang_mgr();
  if (args) m->args = *args;
  else gs_gang_args_default(&m->args);
  *out = m;
  return GS_OK;
}

int gs_gang_mgr_destroy(gs_gang_mgr* m) {
  delete m;
  return GS_OK;
}

int gs_gang_mgr_clone(const gs_gang_mgr* m, gs_gang_mgr** out) {
  if (!m || !out) return GS_EINVAL;
  *out = new gs_gang_mgr(*m);
  return GS_OK;
}

int gs_gang_mgr_assign(gs_gang_mgr* dst, const gs_gang_mgr* src) {
  if (!dst || !src) return GS_EINVAL;
  *dst = *src;
  return GS_OK;
}

// onPodGroupAdd / onPodGroupUpdate (gang_cache.go:150-182)
int gs_gang_podgroup_upsert(gs_gang_mgr* m, const gs_gang_spec* s) {
  if (!m || !s || !s->gang_id || s->group_n > GS_GANG_GROUP_MAX) return GS_EINVAL;
  init_gang(*m->get(s->gang_id, true), *s, true, m->args.default_timeout_ns);
  return GS_OK;
}

// onPodGroupDelete (gang_cache.go:184-197)
int gs_gang_podgroup_delete(gs_gang_mgr* m, uint64_t gang_id) {
  if (!m) return GS_EINVAL;
  m->gangs.erase(gang_id);
  return GS_OK;
}

// onPodAdd / onPodUpdate of a gang pod (gang_cache.go:85-120). annot: the pod's gang annotations when the pod has no
// PodGroup label (the gang is then initialized from the first pod carrying a legal min number); assigned: Spec.NodeName
// is set (an already bound member).
int gs_gang_pod_add(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, int assigned, const gs_gang_spec* annot) {
  if (!m || !gang_id || (annot && annot->group_n > GS_GANG_GROUP_MAX)) return GS_EINVAL;
  Gang& g = *m->get(gang_id, true);
  if (annot && !g.has_init && annot->min_member >= 0) init_gang(g, *annot, false, m->args.default_timeout_ns);
  g.children.insert(uid);
  if (assigned) {
    g.add_bound(uid);
    g.once = true;   // setResourceSatisfied
  }
  return GS_OK;
}

// onPodDelete (gang_cache.go:122-148, gang.deletePod)
int gs_gang_pod_delete(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid) {
  if (!m) return GS_EINVAL;
  Gang* g = m->get(gang_id, false);
  if (!g) return GS_OK;
  g->children.erase(uid);
  g->waiting.erase(uid);
  g->bound.erase(uid);
  g->child_cycle.erase(uid);
  m->fw_waiting.erase(uid);
  if (g->from_annotation && g->children.empty()) m->gangs.erase(gang_id);
  return GS_OK;
}

// PodGroupManager.PreFilter (core.go:221-272); gang_id 0: the pod needs no gang. Returns the GS_GANG_PREFILTER_* code
// (the reference's error message for each is rendered by koordinator_amd/gang.py).
int gs_gang_prefilter(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, int nominated) {
  if (!m) return GS_EINVAL;
  return m->prefilter(gang_id, uid, nominated != 0);
}

// PodGroupManager.Permit (core.go:312-339) + Coscheduling.Permit (coscheduling.go:190-210): GS_GANG_PERMIT_SUCCESS (the
// gang group's waiting pods are allowed: allowed[]), _WAIT (the pod waits until wait_ns after now_ns, *wait_ns), or
// _NOT_FOUND (Unschedulable "Gang not found"). gang_id 0: success, nothing else. The allowed list is sized against the
// caller's buffer before any state changes: GS_EINVAL leaves the manager as it was (*n_allowed = the count needed).
int gs_gang_permit(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, int64_t now_ns, int64_t* wait_ns, uint64_t* allowed,
                   uint32_t cap, uint32_t* n_allowed) {
  if (!m) return GS_EINVAL;
  if (n_allowed) *n_allowed = 0;
  if (wait_ns) *wait_ns = 0;
  const size_t need = m->permit_allows(gang_id, uid);
  if (need > cap) {
    if (n_allowed) *n_allowed = (uint32_t)need;
    return GS_EINVAL;
  }
  gs_gang_mgr::List out;
  const int rc = m->permit(gang_id, uid, now_ns, wait_ns, &out);
  if (n_allowed) *n_allowed = (uint32_t)out.size();
  for (size_t k = 0; k < out.size(); ++k)
    if (allowed) allowed[k] = out[k].first;
  return rc;
}

// PodGroupManager.PostBind (core.go:397-447): the gang's bound children (the PodGroup status patch is the caller's)
int gs_gang_post_bind(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid) {
  if (!m) return GS_EINVAL;
  m->post_bind(gang_id, uid);
  return GS_OK;
}

// PodGroupManager.PostFilter (core.go:277-307) after a gang pod found no node (or failed PreFilter): Strict mode rejects
// the gang group's waiting pods (rejected[]; the caller runs their Unreserve) and invalidates its schedule cycle.
// GS_EINVAL when they do not fit the buffer: nothing changed, *n_rejected = the count needed.
int gs_gang_post_filter(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, uint64_t* rejected, uint32_t cap,
                        uint32_t* n_rejected) {
  if (!m) return GS_EINVAL;
  (void)uid;
  const size_t need = m->post_filter_rejects(gang_id);
  if (n_rejected) *n_rejected = (uint32_t)need;
  if (need > cap) return GS_EINVAL;
  gs_gang_mgr::List out;
  m->post_filter(gang_id, &out);
  for (size_t k = 0; k < out.size(); ++k)
    if (rejected) rejected[k] = out[k].first;
  return GS_OK;
}

// PodGroupManager.Unreserve (core.go:344-361) of an assumed gang pod (a rejected waiting pod, or one whose binding
// cycle failed): it leaves the gang's assumed pods; Strict mode rejects the rest of the gang group's waiting pods.
// GS_EINVAL when they do not fit the buffer: nothing changed, *n_rejected = the count needed.
int gs_gang_unreserve(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, uint64_t* rejected, uint32_t cap,
                      uint32_t* n_rejected) {
  if (!m) return GS_EINVAL;
  const size_t need = m->unreserve_rejects(gang_id, uid);
  if (n_rejected) *n_rejected = (uint32_t)need;
  if (need > cap) return GS_EINVAL;
  gs_gang_mgr::List out;
  m->unreserve(gang_id, uid, &out);
  for (size_t k = 0; k < out.size(); ++k)
    if (rejected) rejected[k] = out[k].first;
  return GS_OK;
}

// The framework's Permit timeout: waiting pods whose deadline is <= now_ns are rejected (their Unreserve follows).
int gs_gang_expire(gs_gang_mgr* m, int64_t now_ns, uint64_t* rejected, uint32_t cap, uint32_t* n_rejected) {
  if (!m) return GS_EINVAL;
  std::vector<uint64_t> out;
  for (const auto& kv : m->fw_waiting)
    if (kv.second.second <= now_ns) out.push_back(kv.first);
  if (n_rejected) *n_rejected = (uint32_t)out.size();
  if (out.size() > cap) return GS_EINVAL;   // sized before any change
  for (size_t k = 0; k < out.size(); ++k) {
    if (rejected) rejected[k] = out[k];
    m->fw_waiting.erase(out[k]);
  }
  return GS_OK;
}

int gs_gang_get(const gs_gang_mgr* m, uint64_t gang_id, gs_gang_info* out) {
  if (!m || !out) return GS_EINVAL;
  auto it = m->gangs.find(gang_id);
  if (it == m->gangs.end()) return 0;
  const Gang& g = it->second;
  std::memset(out, 0, sizeof(*out));
  out->has_init = g.has_init;
  out->min_member = g.min;
  out->total_children = g.total;
  out->mode = g.mode;
  out->match_policy = g.policy;
  out->schedule_cycle = g.cycle;
  out->schedule_cycle_valid = g.cycle_valid;
  out->once_resource_satisfied = g.once;
  out->children = (int32_t)g.children.size();
  out->waiting = (int32_t)g.waiting.size();
  out->bound = (int32_t)g.bound.size();
  out->wait_time_ns = g.wait_ns;
  return 1;
}

// ChildrenScheduleRoundMap[uid] (GetChildScheduleCycle); -1: no entry
int gs_gang_child_cycle(const gs_gang_mgr* m, uint64_t gang_id, uint64_t uid) {
  if (!m) return GS_EINVAL;
  auto it = m->gangs.find(gang_id);
  if (it == m->gangs.end()) return -1;
  auto c = it->second.child_cycle.find(uid);
  return c == it->second.child_cycle.end() ? -1 : c->second;
}

// Test hook (the reference's tests set these fields directly): what 0 ScheduleCycleValid, 1 ChildrenScheduleRoundMap[uid],
// 2 OnceResourceSatisfied, 3 GangMatchPolicy (3: a value outside the three policies), 4 args.SkipCheckScheduleCycle
int gs_gang_debug_set(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, int what, int value) {
  if (!m) return GS_EINVAL;
  if (what == 4) { m->args.skip_check_schedule_cycle = value; return GS_OK; }
  Gang* g = m->get(gang_id, false);
  if (!g) return GS_EINVAL;
  switch (what) {
    case 0: g->cycle_valid = value != 0; break;
    case 1: g->child_cycle[uid] = value; break;
    case 2: g->once = value != 0; break;
    case 3: g->policy = value; break;
    default: return GS_EINVAL;
  }
  return GS_OK;
}

// The framework's waiting pods of gangs (uids ascending)
int gs_gang_waiting_pods(const gs_gang_mgr* m, uint64_t* uids, uint32_t cap, uint32_t* n) {
  if (!m) return GS_EINVAL;
  std::vector<uint64_t> v;
  for (const auto& kv : m->fw_waiting) v.push_back(kv.first);
  return copy_out(v, uids, cap, n);
}

// ---- a scheduling pass: the per-pod gang transitions of koordinator_amd/gang.py schedule_with_gangs, natively
struct gs_gang_pass {
  gs_gang_mgr* m;
  uint32_t n;
  const uint64_t* gang;
  const uint64_t* uid;
  const uint8_t* nom;
  int64_t now;
  int8_t* prefilter;
  int8_t* permit;
  int8_t* state;
  int32_t* node;
  std::unordered_map<uint64_t, uint32_t> index;               // uid -> pod index of this queue
  std::unordered_map<uint64_t, uint64_t> carried_gang;        // uid -> gang of a pod waiting from an earlier pass
  std::vector<std::pair<uint64_t, int8_t>> carried;           // their new states, in order
  std::vector<uint64_t> forgets;                              // rejected pods to forget (ForgetPod), in order

  uint64_t gang_of(uint64_t u) const {
    auto it = index.find(u);
    if (it != index.end()) return gang[it->second];
    auto jt = carried_gang.find(u);
    return jt == carried_gang.end() ? 0 : jt->second;
  }
  void set_state(uint64_t u, int8_t st) {
    auto it = index.find(u);
    if (it != index.end()) state[it->second] = st;
    else carried.push_back({u, st});
  }
  // PostBind of a pod Permit allowed (this queue's, or one waiting from an earlier pass)
  void bind(uint64_t u, uint64_t g) {
    set_state(u, GS_GANG_ST_BOUND);
    m->post_bind(g, u);
  }
  // rejected waiting pods: Unreserve (gang) + ForgetPod, and the rejections that follow (one chain, queue order)
  void unreserve_chain(const gs_gang_mgr::List& rejected) {
    std::deque<std::pair<uint64_t, uint64_t>> q(rejected.begin(), rejected.end());
    while (!q.empty()) {
      const auto [u, g] = q.front();
      q.pop_front();
      carried_gang.emplace(u, g);   // (its gang, once fw_waiting no longer holds it)
      forgets.push_back(u);
      set_state(u, GS_GANG_ST_REJECTED);
      gs_gang_mgr::List more;
      m->unreserve(g, u, &more);
      q.insert(q.end(), more.begin(), more.end());
    }
  }
  // PreFilter; on a rejection its PostFilter (the waiting pods it rejects go to *rej)
  bool before_node_loop(uint32_t k, gs_gang_mgr::List* rej) {
    const int code = m->prefilter(gang[k], uid[k], nom && nom[k]);
    prefilter[k] = (int8_t)code;
    if (code == GS_GANG_PREFILTER_OK) return true;
    m->post_filter(gang[k], rej);
    return false;
  }
  // a FitError's PostFilter, or Reserve + Permit (+ the binds Permit allows); the pods to Unreserve go to *rej
  void after_node_loop(uint32_t k, int32_t nd, gs_gang_mgr::List* rej) {
    if (nd < 0) {
      m->post_filter(gang[k], rej);
      return;
    }
    node[k] = nd;
    gs_gang_mgr::List allowed;
    const int st = m->permit(gang[k], uid[k], now, nullptr, &allowed);
    permit[k] = (int8_t)st;
    if (st == GS_GANG_PERMIT_SUCCESS) {
      state[k] = GS_GANG_ST_BOUND;
      m->post_bind(gang[k], uid[k]);
      for (const auto& a : allowed) bind(a.first, a.second);
    } else if (st == GS_GANG_PERMIT_WAIT) {
      state[k] = GS_GANG_ST_WAITING;
    } else {   // "Gang not found": the pod's Permit fails, its Reserve is undone (it is not a waiting pod)
      state[k] = GS_GANG_ST_REJECTED;
      rej->push_back({uid[k], gang[k]});
    }
  }
};

int gs_gang_pass_create(gs_gang_mgr* m, uint32_t n, const uint64_t* gang_ids, const uint64_t* uids,
                        const uint8_t* nominated, int64_t now_ns, int8_t* prefilter, int8_t* permit, int8_t* state,
                        int32_t* node, gs_gang_pass** out) {
  if (!m || !out || (n && (!gang_ids || !uids || !prefilter || !permit || !state || !node))) return GS_EINVAL;
  auto* p = new gs_gang_pass();
  p->m = m;
  p->n = n;
  p->gang = gang_ids;
  p->uid = uids;
  p->nom = nominated;
  p->now = now_ns;
  p->prefilter = prefilter;
  p->permit = permit;
  p->state = state;
  p->node = node;
  p->index.reserve(2 * (size_t)n);
  for (uint32_t k = 0; k < n; ++k) {
    p->index.emplace(uids[k], k);
    prefilter[k] = 0;
    permit[k] = -1;
    state[k] = GS_GANG_ST_UNSCHEDULABLE;
    node[k] = -1;
  }
  for (const auto& kv : m->fw_waiting)   // pods waiting from earlier passes
    if (!p->index.count(kv.first)) p->carried_gang.emplace(kv.first, kv.second.first);
  *out = p;
  return GS_OK;
}

int gs_gang_pass_destroy(gs_gang_pass* p) {
  // a pass aborted between gs_gang_walk and gs_gang_replay (the engine call failed): roll its speculative walk back,
  // so the manager is left as before the walk (and no stray replay can restore a stale snapshot later)
  if (p && p->m && p->m->snap_on) p->m->snap_restore();
  delete p;
  return GS_OK;
}

// the speculative walk (gang.py schedule_with_gangs): every pod that passes PreFilter is assumed to find a node
int gs_gang_walk(gs_gang_pass* p, uint32_t i, uint32_t run_cap, uint32_t* run, uint32_t* run_n, uint32_t* j_out) {
  if (!p || !run || !run_n || !j_out || i > p->n) return GS_EINVAL;
  gs_gang_mgr& m = *p->m;
  m.snap_begin();
  uint32_t j = i, nr = 0;
  while (j < p->n && nr < run_cap) {
    gs_gang_mgr::List rej;
    if (!p->before_node_loop(j, &rej)) {
      ++j;
      if (!rej.empty()) break;   // Unreserves: the engine state changes after this pod
      continue;
    }
    run[nr++] = j;
    gs_gang_mgr::List allowed;
    const int st = m.permit(p->gang[j], p->uid[j], p->now, nullptr, &allowed);
    ++j;
    if (st == GS_GANG_PERMIT_SUCCESS) {
      m.post_bind(p->gang[j - 1], p->uid[j - 1]);
      for (const auto& a : allowed) m.post_bind(a.second, a.first);
    } else if (st == GS_GANG_PERMIT_NOT_FOUND) {
      break;   // its Reserve is undone after the run
    }
  }
  *run_n = nr;
  *j_out = j;
  return GS_OK;
}

// the replay of [i, j) from the walk's snapshot with the run's true nodes
int gs_gang_replay(gs_gang_pass* p, uint32_t i, uint32_t j, const uint32_t* run, uint32_t run_n,
                   const int32_t* got_node, uint32_t* r_stop, uint32_t* j_next, int32_t* single) {
  if (!p || !r_stop || !j_next || !single || j > p->n || i > j || (run_n && (!run || !got_node))) return GS_EINVAL;
  gs_gang_mgr& m = *p->m;
  if (!m.snap_on) return GS_ESTATE;
  m.snap_restore();
  *single = -1;
  uint32_t r = 0, k = i;
  for (; k < j; ++k) {
    gs_gang_mgr::List rej;
    const bool ok = p->before_node_loop(k, &rej);
    const bool in_run = r < run_n && run[r] == k;
    if (ok != in_run) {   // the walk's PreFilter verdict was wrong here: the rest of the run is withdrawn
      if (ok) {
        *single = (int32_t)k;   // it passes: the caller schedules it alone (gs_gang_pass_after_single)
      } else {
        p->unreserve_chain(rej);
      }
      *r_stop = r;
      *j_next = k + 1;
      return GS_OK;
    }
    if (ok) {
      p->after_node_loop(k, got_node[r], &rej);
      ++r;
    }
    if (!rej.empty()) {
      p->unreserve_chain(rej);
      if (r < run_n) {   // a forget changes the node state under the run's later pods
        *r_stop = r;
        *j_next = k + 1;
        return GS_OK;
      }
    }
  }
  *r_stop = r;
  *j_next = j;
  return GS_OK;
}

int gs_gang_pass_after_single(gs_gang_pass* p, uint32_t k, int32_t nd) {
  if (!p || k >= p->n) return GS_EINVAL;
  gs_gang_mgr::List rej;
  p->after_node_loop(k, nd, &rej);
  p->unreserve_chain(rej);
  return GS_OK;
}

int gs_gang_pass_forgets(gs_gang_pass* p, uint64_t* uids, uint32_t cap, uint32_t* n) {
  if (!p) return GS_EINVAL;
  if (n) *n = (uint32_t)p->forgets.size();
  if (p->forgets.size() > cap) return GS_EINVAL;
  for (size_t k = 0; k < p->forgets.size(); ++k)
    if (uids) uids[k] = p->forgets[k];
  p->forgets.clear();
  return GS_OK;
}

int gs_gang_pass_carried(gs_gang_pass* p, uint64_t* uids, int8_t* states, uint32_t cap, uint32_t* n) {
  if (!p) return GS_EINVAL;
  if (n) *n = (uint32_t)p->carried.size();
  if (p->carried.size() > cap) return GS_EINVAL;
  for (size_t k = 0; k < p->carried.size(); ++k) {
    if (uids) uids[k] = p->carried[k].first;
    if (states) states[k] = p->carried[k].second;
  }
  return GS_OK;
}

}  // extern "C"
