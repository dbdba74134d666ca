// gs_quota.cpp — ElasticQuota admission: the per-pod quota gate that runs in PreFilter,
// before the node loop. It reads the quota forest (O(depth) groups per pod, nothing per node), so it is host
// code next to the engine, not a device kernel. Restates:
//   * quotaTree.redistribution / iterationForRedistribution (elasticquota/core/runtime_quota_calculator.go:106-166)
//     — the min-then-shared-weight water filling of one parent's runtime over its children, per dimension;
//   * the request tree (group_quota_manager.go:184-224 recursiveUpdateGroupTreeWithDeltaRequest, quota_info.go:
//     201-212 getLimitRequestNoLock) and the top-down runtime refresh (group_quota_manager.go:264-321), computed
//     for every group at once from a settled tree;
//   * Plugin.PreFilter (plugin.go:210-254) and checkQuotaRecursive (plugin_helper.go:281-297).
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/gpuscore.h"

namespace {

constexpr int D = GS_QUOTA_DIMS;

// iterationForRedistribution (runtime_quota_calculator.go:140-166), as a loop instead of tail recursion. Each
// node's share depends only on (totalRes, totalSharedWeight), so the Go map's iteration order cannot change the
// result; the share is int64(float64(w)*float64(total)/float64(totalW) + 0.5) — the same three IEEE double
// operations, truncated toward zero like Go's conversion.
void iterate(int64_t total, int64_t total_w, std::vector<uint32_t>& nodes, std::vector<uint32_t>& next,
             const int64_t* request, const int64_t* weight, int64_t* rt) {
  while (total_w > 0) {
    next.clear();
    int64_t part = 0, next_w = 0;
    for (uint32_t i : nodes) {
      const int64_t delta = (int64_t)((double)weight[i] * (double)total / (double)total_w + 0.5);
      rt[i] += delta;
      if (rt[i] < request[i]) {
        next.push_back(i);
        next_w += weight[i];
      } else {
        part += rt[i] - request[i];
        rt[i] = request[i];
      }
    }
    if (part <= 0 || next.empty()) return;
    total = part;
    total_w = next_w;
    nodes.swap(next);
  }
}

// quotaTree.redistribution (runtime_quota_calculator.go:106-138).
void redistribute(uint32_t n, const int64_t* request, const int64_t* min, const int64_t* guaranteed,
                  const int64_t* weight, const uint8_t* lent, int64_t total, int64_t* rt) {
  int64_t to_part = total, total_w = 0;
  thread_local std::vector<uint32_t> adjust, next;   // scratch reused across calls (no per-parent allocation)
  adjust.clear();
  for (uint32_t i = 0; i < n; ++i) {
    const int64_t m = guaranteed[i] > min[i] ? guaranteed[i] : min[i];   // guarantee above min replaces it
    if (request[i] > m) {
      adjust.push_back(i);
      total_w += weight[i];
      rt[i] = m;
    } else {
      rt[i] = lent[i] ? request[i] : m;   // a quota that does not lend keeps its min
    }
    to_part -= rt[i];
  }
  if (to_part > 0) iterate(to_part, total_w, adjust, next, request, weight, rt);
}

// quotav1.LessThanOrEqual(Mask(Add(podRequest, used), names(podRequest)), limit): only keys of the limit that the
// pod requests are compared (a key missing from `used` is zero). Returns the exceeding dimensions.
uint32_t exceeds(const int64_t* used, const int64_t* req, uint32_t req_mask, const int64_t* limit,
                 uint32_t limit_mask) {
  uint32_t m = 0;
  for (int d = 0; d < D; ++d)
    if ((limit_mask >> d & 1u) && (req_mask >> d & 1u) && used[d] + req[d] > limit[d]) m |= 1u << d;
  return m;
}

}  // namespace

extern "C" int gs_quota_redistribute(const int64_t* request, const int64_t* min, const int64_t* guaranteed,
                                     const int64_t* shared_weight, const uint8_t* allow_lent, uint32_t n,
                                     int64_t total, int64_t* runtime) {
  if (n == 0) return GS_OK;
  if (!request || !min || !guaranteed || !shared_weight || !allow_lent || !runtime) return GS_EINVAL;
  redistribute(n, request, min, guaranteed, shared_weight, allow_lent, total, runtime);
  return GS_OK;
}

extern "C" int gs_quota_refresh_runtime(const gs_quota_group* g, uint32_t n, const int64_t total[GS_QUOTA_DIMS],
                                        int64_t* runtime, int64_t* limit_request, uint32_t* runtime_mask) {
  if (n && (!g || !total)) return GS_EINVAL;
  // children in CSR form (slot n = the root), then a BFS from the root: parents before children. A group the
  // BFS does not reach sits on a cycle.
  std::vector<uint32_t> off(n + 2, 0), kid(n), order;
  order.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    const int32_t p = g[i].parent;
    if (p < -1 || p >= (int32_t)n) return GS_EINVAL;
    ++off[(p < 0 ? n : (uint32_t)p) + 1];
  }
  for (uint32_t i = 0; i <= n; ++i) off[i + 1] += off[i];
  {
    std::vector<uint32_t> fill(off.begin(), off.end() - 1);
    for (uint32_t i = 0; i < n; ++i) kid[fill[g[i].parent < 0 ? n : (uint32_t)g[i].parent]++] = i;
  }
  for (uint32_t k = off[n]; k < off[n + 1]; ++k) order.push_back(kid[k]);
  for (size_t h = 0; h < order.size(); ++h)
    for (uint32_t k = off[order[h]]; k < off[order[h] + 1]; ++k) order.push_back(kid[k]);
  if (order.size() != n) return GS_EINVAL;

  uint32_t keys = 0;   // updateResourceKeyNoLock: the union of every quota's Max keys
  for (uint32_t i = 0; i < n; ++i) keys |= g[i].max_mask;
  keys &= (1u << D) - 1;
  if (runtime_mask)
    for (uint32_t i = 0; i < n; ++i) runtime_mask[i] = keys;

  // bottom-up (reverse BFS): ChildRequest = own pods + the children's limited requests; Request = ChildRequest,
  // raised to Min when the quota does not lend; limited request = min(Request, Max) on Max's keys.
  std::vector<int64_t> child(size_t(n) * D), limit(size_t(n) * D);
  for (uint32_t i = 0; i < n; ++i)
    for (int d = 0; d < D; ++d) child[size_t(i) * D + d] = g[i].request[d];
  for (uint32_t h = n; h-- > 0;) {
    const uint32_t i = order[h];
    for (int d = 0; d < D; ++d) {
      int64_t r = child[size_t(i) * D + d];
      if (r < 0) r = 0;   // addChildRequestNonNegativeNoLock
      if (!g[i].allow_lent && (g[i].min_mask >> d & 1u) && g[i].min[d] > r) r = g[i].min[d];
      if ((g[i].max_mask >> d & 1u) && r > g[i].max[d]) r = g[i].max[d];
      limit[size_t(i) * D + d] = r;
      if (g[i].parent >= 0) child[size_t(g[i].parent) * D + d] += r;
    }
  }

  // top-down (root, then BFS order): each parent's runtime (the root's: total) is redistributed over its
  // children, per key.
  std::vector<int64_t> rt(size_t(n) * D, 0);
  std::vector<int64_t> req, mn, gu, w, out;
  std::vector<uint8_t> lent;
  for (uint32_t h = 0; h <= n; ++h) {
    const uint32_t p = h == 0 ? n : order[h - 1];
    const uint32_t k0 = off[p], m = off[p + 1] - k0;
    if (m == 0) continue;
    req.resize(m); mn.resize(m); gu.resize(m); w.resize(m); lent.resize(m); out.resize(m);
    for (int d = 0; d < D; ++d) {
      if (!(keys >> d & 1u)) continue;
      for (uint32_t j = 0; j < m; ++j) {
        const uint32_t c = kid[k0 + j];
        req[j] = limit[size_t(c) * D + d];
        mn[j] = (g[c].min_mask >> d & 1u) ? g[c].min[d] : 0;
        gu[j] = g[c].guaranteed[d];
        w[j] = g[c].shared_weight[d];
        lent[j] = g[c].allow_lent ? 1 : 0;
      }
      const int64_t tot = p == n ? total[d] : rt[size_t(p) * D + d];
      redistribute(m, req.data(), mn.data(), gu.data(), w.data(), lent.data(), tot, out.data());
      for (uint32_t j = 0; j < m; ++j) rt[size_t(kid[k0 + j]) * D + d] = out[j];
    }
  }
  if (runtime) std::memcpy(runtime, rt.data(), rt.size() * sizeof(int64_t));
  if (limit_request) std::memcpy(limit_request, limit.data(), limit.size() * sizeof(int64_t));
  return GS_OK;
}

extern "C" int gs_quota_prefilter(const gs_quota_group* g, uint32_t n, const int64_t* runtime,
                                  const uint32_t* runtime_mask, int32_t quota, const int64_t pod_request[GS_QUOTA_DIMS],
                                  uint32_t pod_request_mask, uint32_t flags, gs_quota_status* out) {
  if (!out) return GS_EINVAL;
  out->code = GS_QUOTA_ADMIT;
  out->group = -1;
  out->exceed_mask = 0;
  out->depth = 0;
  std::memset(out->used, 0, sizeof(out->used));
  if (quota < 0) return GS_OK;   // no quota label: PreFilter skips (plugin.go:211-215)
  if ((uint32_t)quota >= n || !g || !pod_request) return GS_EINVAL;
  const bool use_runtime = flags & GS_QUOTA_RUNTIME;
  if (use_runtime && (!runtime || !runtime_mask)) return GS_EINVAL;
  // validate only this pod's ancestor chain (O(depth) per pod, not the forest)
  uint32_t hops = 0;
  for (int32_t p = g[quota].parent; p != -1; p = g[p].parent)
    if (p < -1 || (uint32_t)p >= n || ++hops > n) return GS_EINVAL;

  // getQuotaInfoUsedLimit (plugin_helper.go:314-319): Runtime when runtime quota is on, else Max
  auto check = [&](uint32_t q) {
    return use_runtime ? exceeds(g[q].used, pod_request, pod_request_mask, runtime + size_t(q) * D,
                                   runtime_mask[q])
                       : exceeds(g[q].used, pod_request, pod_request_mask, g[q].max, g[q].max_mask);
  };
  uint32_t m = check((uint32_t)quota);
  if (m) {
    out->code = GS_QUOTA_INSUFFICIENT;
    out->group = quota;
    out->exceed_mask = m;
    std::memcpy(out->used, g[quota].used, sizeof(out->used));
    return GS_OK;
  }
  if (flags & GS_QUOTA_NON_PREEMPTIBLE) {   // nonPreemptibleUsed + request within Min (plugin.go:235-244)
    m = exceeds(g[quota].non_preemptible_used, pod_request, pod_request_mask, g[quota].min, g[quota].min_mask);
    if (m) {
      out->code = GS_QUOTA_INSUFFICIENT_NON_PREEMPTIBLE;
      out->group = quota;
      out->exceed_mask = m;
      std::memcpy(out->used, g[quota].non_preemptible_used, sizeof(out->used));
      return GS_OK;
    }
  }
  if (flags & GS_QUOTA_CHECK_PARENT) {   // checkQuotaRecursive: this quota, then every ancestor below the root
    uint32_t hops = 0;
    for (int32_t q = quota; q >= 0; q = g[q].parent, ++hops) {
      m = check((uint32_t)q);
      if (m) {
        out->code = GS_QUOTA_INSUFFICIENT;
        out->group = q;
        out->exceed_mask = m;
        out->depth = hops;
        std::memcpy(out->used, g[q].used, sizeof(out->used));
        return GS_OK;
      }
    }
  }
  return GS_OK;
}

// GroupQuotaManager.ReservePod / UnreservePod (group_quota_manager.go:791-805 -> updatePodUsedNoLock): the pod's
// request joins (sign -1: leaves) used — and non-preemptible used — of its quota and every ancestor, each clamped
// at zero. A speculative Reserve withdrawn by gs_quota_settle_batch cancels exactly (used never goes below zero).
extern "C" int gs_quota_reserve(gs_quota_group* g, uint32_t n, int32_t quota, const int64_t request[GS_QUOTA_DIMS],
                                uint32_t flags, int32_t sign) {
  if (quota < 0) return GS_OK;
  if (!g || !request || (uint32_t)quota >= n || (sign != 1 && sign != -1)) return GS_EINVAL;
  uint32_t hops = 0;
  for (int32_t q = quota; q != -1; q = g[q].parent) {
    if (q < -1 || (uint32_t)q >= n || ++hops > n) return GS_EINVAL;
    for (int d = 0; d < D; ++d) {   // addUsedNonNegativeNoLock (quota_info.go:252-261): negatives clamp to 0
      g[q].used[d] = std::max<int64_t>(0, g[q].used[d] + sign * request[d]);
      if (flags & GS_QUOTA_NON_PREEMPTIBLE)
        g[q].non_preemptible_used[d] = std::max<int64_t>(0, g[q].non_preemptible_used[d] + sign * request[d]);
    }
  }
  return GS_OK;
}

// The admission loop of a quota-gated batch (koordinator_amd/quota.py schedule_with_quota): PreFilter each pod
// in order and Reserve every admitted pod speculatively (as if placed). Admission is monotone in used, so an
// admitted verdict stands whatever the speculative pods' outcomes. A rejection is final when it also holds
// against the certain used (used minus this call's speculative Reserves on the pod's chain, the least the true
// used can be); otherwise the loop stops before that pod, to be re-checked once the batch's true placements
// are reserved. *consumed = the pods decided.
extern "C" int gs_quota_admit_batch(gs_quota_group* g, uint32_t n, const int64_t* runtime,
                                    const uint32_t* runtime_mask, const int32_t* quota, const int64_t* requests,
                                    const uint32_t* request_mask, const uint32_t* flags, uint32_t count,
                                    gs_quota_status* status, uint32_t* consumed) {
  if (!consumed || (count && (!quota || !requests || !request_mask || !flags || !status))) return GS_EINVAL;
  *consumed = 0;
  std::vector<int64_t> spec(size_t(n) * 2 * D, 0);   // per group: speculative used, non-preemptible used
  std::vector<uint8_t> touched(n, 0);
  auto shift = [&](int32_t q0, int64_t sign) {        // remove (-1) / restore (+1) the speculation on a chain
    for (int32_t q = q0; q != -1; q = g[q].parent)
      if (touched[q])
        for (int d = 0; d < D; ++d) {
          g[q].used[d] += sign * spec[size_t(q) * 2 * D + d];
          g[q].non_preemptible_used[d] += sign * spec[size_t(q) * 2 * D + D + d];
        }
  };
  // on an error, every speculative Reserve of this call is withdrawn before returning (used as on entry)
  auto undo = [&](int rc) {
    for (uint32_t q = 0; q < n; ++q)
      if (touched[q])
        for (int d = 0; d < D; ++d) {
          g[q].used[d] -= spec[size_t(q) * 2 * D + d];
          g[q].non_preemptible_used[d] -= spec[size_t(q) * 2 * D + D + d];
        }
    *consumed = 0;
    return rc;
  };
  for (uint32_t j = 0; j < count; ++j) {
    const int64_t* req = requests + size_t(j) * D;
    gs_quota_status st;
    int rc = gs_quota_prefilter(g, n, runtime, runtime_mask, quota[j], req, request_mask[j], flags[j], &st);
    if (rc != GS_OK) return undo(rc);
    if (st.code != GS_QUOTA_ADMIT) {
      bool overlap = false;
      for (int32_t q = quota[j]; q != -1 && !overlap; q = g[q].parent) overlap = touched[q];
      if (overlap) {
        gs_quota_status certain;
        shift(quota[j], -1);
        rc = gs_quota_prefilter(g, n, runtime, runtime_mask, quota[j], req, request_mask[j], flags[j], &certain);
        shift(quota[j], +1);
        if (rc != GS_OK) return undo(rc);
        if (certain.code == GS_QUOTA_ADMIT) return GS_OK;   // depends on the speculation: cut here
        st = certain;                                       // rejected at the least possible used: final
      }
    } else if (quota[j] >= 0) {
      rc = gs_quota_reserve(g, n, quota[j], req, flags[j], 1);
      if (rc != GS_OK) return undo(rc);
      for (int32_t q = quota[j]; q != -1; q = g[q].parent) {
        touched[q] = 1;
        for (int d = 0; d < D; ++d) {
          spec[size_t(q) * 2 * D + d] += req[d];
          if (flags[j] & GS_QUOTA_NON_PREEMPTIBLE) spec[size_t(q) * 2 * D + D + d] += req[d];
        }
      }
    }
    status[j] = st;
    *consumed = j + 1;
  }
  return GS_OK;
}

// Settles a run decided by gs_quota_admit_batch once the engine's placements are known: the speculative Reserves
// are withdrawn and the run is replayed in order — a placed pod is reserved, an admitted pod with no node is not,
// and every rejected pod's status is recomputed against the used it would have seen in the one-pod-at-a-time
// order (a final rejection decided against the certain used keeps its verdict, its detail may change).
// GS_ESTATE if a replayed verdict differs from the one admit_batch gave (it cannot, by monotonicity).
extern "C" int gs_quota_settle_batch(gs_quota_group* g, uint32_t n, const int64_t* runtime,
                                     const uint32_t* runtime_mask, const int32_t* quota, const int64_t* requests,
                                     const uint32_t* request_mask, const uint32_t* flags, uint32_t count,
                                     const int32_t* placed_node, gs_quota_status* status) {
  if (count && (!quota || !requests || !request_mask || !flags || !status || !placed_node)) return GS_EINVAL;
  for (uint32_t j = 0; j < count; ++j)
    if (status[j].code == GS_QUOTA_ADMIT && quota[j] >= 0) {
      int rc = gs_quota_reserve(g, n, quota[j], requests + size_t(j) * D, flags[j], -1);
      if (rc != GS_OK) return rc;
    }
  for (uint32_t j = 0; j < count; ++j) {
    const int64_t* req = requests + size_t(j) * D;
    gs_quota_status st;
    int rc = gs_quota_prefilter(g, n, runtime, runtime_mask, quota[j], req, request_mask[j], flags[j], &st);
    if (rc != GS_OK) return rc;
    if ((st.code == GS_QUOTA_ADMIT) != (status[j].code == GS_QUOTA_ADMIT)) return GS_ESTATE;
    status[j] = st;
    if (st.code == GS_QUOTA_ADMIT && quota[j] >= 0 && placed_node[j] >= 0) {
      rc = gs_quota_reserve(g, n, quota[j], req, flags[j], 1);
      if (rc != GS_OK) return rc;
    }
  }
  return GS_OK;
}
