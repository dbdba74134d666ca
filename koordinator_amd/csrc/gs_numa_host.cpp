// gs_numa_host.cpp — NodeNUMAResource host state of libgpuscore (see gs_numa_host.h).
// Reference paths are relative to pkg/scheduler/plugins/nodenumaresource/.
#include "gs_numa_host.h"

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>

#include "gs_layout.h"

namespace gs {

namespace {

int64_t amplify(int64_t origin, double ratio) {   // apis/extension/node_resource_amplification.go:170-175
  if (ratio <= 1) return origin;
  return (int64_t)std::ceil((double)origin * ratio);
}

// Go 1.18 sort.Slice for <= 12 elements: gap-6 shell pass + insertion sort (ties keep input order
// except for the gap-6 swaps). Used where the reference comparator has ties (cpu_accumulator.go:142,161).
template <class T, class Less>
void go_sort_small(std::vector<T>& v, Less less) {
  int n = (int)v.size();
  if (n > 12) { std::stable_sort(v.begin(), v.end(), less); return; }
  for (int i = 6; i < n; ++i)
    if (less(v[i], v[i - 6])) std::swap(v[i], v[i - 6]);
  for (int i = 1; i < n; ++i)
    for (int j = i; j > 0 && less(v[j], v[j - 1]); --j) std::swap(v[j], v[j - 1]);
}

struct Counts {
  int raw = 0, full = 0, spread = 0;
  int64_t packed() const { return (int64_t)raw | ((int64_t)full << 9) | ((int64_t)spread << 18); }
};

// available CPUs restricted to `numa` (-1: all): raw count, CPUs in fully available cores, cores with one
// available CPU (filterCPUsByRequiredCPUBindPolicy, resource_manager.go:534-566, counted)
Counts count_available(const TopoClass& t, const CpuMask& avail, int numa) {
  Counts c;
  std::map<int, int> per_core;
  for (int cpu = 0; cpu < t.num_cpus; ++cpu) {
    if (!avail.has(cpu) || (numa >= 0 && t.node[cpu] != numa)) continue;
    ++c.raw;
    per_core[t.core[cpu]]++;
  }
  for (auto& kv : per_core) {
    if (kv.second == t.cpc) c.full += kv.second;
    ++c.spread;
  }
  return c;
}

CpuMask filter_required(const TopoClass& t, int policy, const CpuMask& avail) {
  if (policy != GS_CPU_BIND_FULL_PCPUS && policy != GS_CPU_BIND_SPREAD_BY_PCPUS) return avail;
  std::map<int, std::vector<int>> per_core;
  for (int cpu = 0; cpu < t.num_cpus; ++cpu)
    if (avail.has(cpu)) per_core[t.core[cpu]].push_back(cpu);
  CpuMask out;
  for (auto& kv : per_core) {
    if (policy == GS_CPU_BIND_FULL_PCPUS) {
      if ((int)kv.second.size() == t.cpc)
        for (int c : kv.second) out.set(c);
    } else {
      out.set(kv.second[0]);
    }
  }
  return out;
}

bool satisfied_required(const TopoClass& t, int policy, const CpuMask& cpus) {   // resource_manager.go:568-589
  std::set<int> cores;
  for (int c = 0; c < t.num_cpus; ++c)
    if (cpus.has(c)) cores.insert(t.core[c]);
  if (policy == GS_CPU_BIND_FULL_PCPUS) return (int)cores.size() * t.cpc == cpus.count();
  if (policy == GS_CPU_BIND_SPREAD_BY_PCPUS) return (int)cores.size() == cpus.count();
  return true;
}

// cpuAccumulator (cpu_accumulator.go:249-822) over the topology arrays
struct Acc {
  const TopoClass& t;
  int max_ref;
  bool allocatable[GS_MAX_CPUS];
  int aref[GS_MAX_CPUS];
  int nalloc = 0;
  int needed;
  bool exclusive;
  int ep, strategy;
  std::set<int> excl_cores, excl_nodes;
  CpuMask result;

  Acc(const TopoClass& tc, int mr, const CpuMask& available, const uint16_t* ref, const uint8_t* ex, int n, int e, int st)
      : t(tc), max_ref(mr), needed(n), ep(e), strategy(st) {
    for (int c = 0; c < GS_MAX_CPUS; ++c) {
      if (ref[c] == 0) continue;
      int core = c < t.num_cpus ? t.core[c] : 0, node = c < t.num_cpus ? t.node[c] : 0;
      if (ex[c] == GS_CPU_EXCLUSIVE_PCPU_LEVEL) excl_cores.insert(core);
      else if (ex[c] == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL) excl_nodes.insert(node);
    }
    exclusive = e == GS_CPU_EXCLUSIVE_PCPU_LEVEL || e == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL;
    for (int c = 0; c < GS_MAX_CPUS; ++c) {
      allocatable[c] = c < t.num_cpus && available.has(c);
      aref[c] = (max_ref > 1 && allocatable[c]) ? ref[c] : 0;
      nalloc += allocatable[c];
    }
  }
  bool most() const { return strategy == GS_NUMA_ALLOC_MOST_ALLOCATED; }
  bool sless(int a, int b) const { return most() ? a < b : a > b; }
  void take(const std::vector<int>& cpus) {
    for (int c : cpus) {
      result.set(c);
      if (allocatable[c]) { allocatable[c] = false; --nalloc; }
      if (exclusive) {
        if (ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL) excl_cores.insert(t.core[c]);
        else excl_nodes.insert(t.node[c]);
      }
    }
    needed -= (int)cpus.size();
  }
  bool needs(int n) const { return needed >= n; }
  bool satisfied() const { return needed < 1; }
  bool failed() const { return needed > nalloc; }
  bool xp(int c) const { return ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL && excl_cores.count(t.core[c]); }
  bool xn(int c) const { return ep == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL && excl_nodes.count(t.node[c]); }
  int core_ref(int core) const {
    int r = 0;
    for (int c = 0; c < t.num_cpus; ++c)
      if (allocatable[c] && t.core[c] == core) r += aref[c];
    return r;
  }
  void sort_cores(std::vector<int>& cores, std::map<int, std::vector<int>>& cic) const {
    if (cores.size() <= 1) return;
    std::sort(cores.begin(), cores.end(), [&](int i, int j) {
      if (cic[i].size() != cic[j].size()) return cic[i].size() > cic[j].size();
      if (max_ref > 1) {
        int a = core_ref(i), b = core_ref(j);
        if (a != b) return a < b;
      }
      return i < j;
    });
  }
  void sort_by_ref(std::vector<int>& cpus) const {
    std::sort(cpus.begin(), cpus.end(), [&](int i, int j) {
      if (aref[i] != aref[j]) return aref[i] < aref[j];
      return i < j;
    });
  }
  std::vector<int> extract(const std::vector<int>& cpus) const {
    std::vector<int> out;
    std::set<int> seen;
    for (int c : cpus)
      if (seen.insert(t.core[c]).second) out.push_back(c);
    return out;
  }
  std::vector<std::vector<int>> cores_in_node(bool full, bool fe) const {   // freeCoresInNode
    std::map<int, int> sfree;
    std::map<int, std::vector<int>> cic;
    for (int c = 0; c < t.num_cpus; ++c) {
      if (!allocatable[c] || (fe && xn(c))) continue;
      cic[t.core[c]].push_back(c);
      sfree[t.socket[c]]++;
    }
    std::map<int, std::vector<int>> by_node;
    for (auto& kv : cic) {
      if (full && (int)kv.second.size() != t.cpc) continue;
      by_node[t.node[kv.second[0]]].push_back(kv.first);
    }
    std::vector<int> ids;
    std::map<int, std::vector<int>> lists;
    for (auto& kv : by_node) {
      ids.push_back(kv.first);
      std::vector<int> cores = kv.second;
      sort_cores(cores, cic);
      std::vector<int>& out = lists[kv.first];
      for (int core : cores) out.insert(out.end(), cic[core].begin(), cic[core].end());
    }
    std::sort(ids.begin(), ids.end(), [&](int i, int j) {
      int a = (int)lists[i].size(), b = (int)lists[j].size();
      if (a != b) return sless(a, b);
      int sa = sfree[t.socket[lists[i][0]]], sb = sfree[t.socket[lists[j][0]]];
      if (sa != sb) return sless(sa, sb);
      return i < j;
    });
    std::vector<std::vector<int>> res;
    for (int id : ids) res.push_back(lists[id]);
    return res;
  }
  std::vector<std::vector<int>> cores_in_socket(bool full) const {   // freeCoresInSocket
    std::map<int, std::vector<int>> cic;
    for (int c = 0; c < t.num_cpus; ++c)
      if (allocatable[c]) cic[t.core[c]].push_back(c);
    std::map<int, std::vector<int>> by_socket;
    for (auto& kv : cic) {
      if (full && (int)kv.second.size() != t.cpc) continue;
      by_socket[t.socket[kv.second[0]]].push_back(kv.first);
    }
    std::vector<int> ids;
    std::map<int, std::vector<int>> lists;
    for (auto& kv : by_socket) {
      ids.push_back(kv.first);
      std::vector<int> cores = kv.second;
      sort_cores(cores, cic);
      std::vector<int>& out = lists[kv.first];
      for (int core : cores) out.insert(out.end(), cic[core].begin(), cic[core].end());
    }
    std::sort(ids.begin(), ids.end(), [&](int i, int j) {
      int a = (int)lists[i].size(), b = (int)lists[j].size();
      if (a != b) return sless(a, b);
      return i < j;
    });
    std::vector<std::vector<int>> res;
    for (int id : ids) res.push_back(lists[id]);
    return res;
  }
  std::vector<std::vector<int>> cpus_in_node(bool fe) const {   // freeCPUsInNode
    std::map<int, std::vector<int>> lists;
    std::map<int, int> nfree, sfree;
    for (int c = 0; c < t.num_cpus; ++c) {
      if (!allocatable[c] || (fe && (xp(c) || xn(c)))) continue;
      lists[t.node[c]].push_back(c);
      nfree[t.node[c]]++;
      sfree[t.socket[c]]++;
    }
    std::vector<int> ids;
    for (auto& kv : lists) {
      ids.push_back(kv.first);
      if (max_ref > 1) sort_by_ref(kv.second);
      if (fe) kv.second = extract(kv.second);
    }
    std::sort(ids.begin(), ids.end(), [&](int i, int j) {
      int a = nfree[i], b = nfree[j];
      if (a != b) return sless(a, b);
      int sa = sfree[t.socket[lists[i][0]]], sb = sfree[t.socket[lists[j][0]]];
      if (sa != sb) return sless(sa, sb);
      return i < j;
    });
    std::vector<std::vector<int>> res;
    for (int id : ids) res.push_back(lists[id]);
    return res;
  }
  std::vector<std::vector<int>> cpus_in_socket(bool fe) const {   // freeCPUsInSocket
    std::map<int, std::vector<int>> lists;
    for (int c = 0; c < t.num_cpus; ++c) {
      if (!allocatable[c] || (fe && xp(c))) continue;
      lists[t.socket[c]].push_back(c);
    }
    std::vector<int> ids;
    for (auto& kv : lists) {
      ids.push_back(kv.first);
      if (max_ref > 1) sort_by_ref(kv.second);
      if (fe) kv.second = extract(kv.second);
    }
    std::sort(ids.begin(), ids.end(), [&](int i, int j) {
      int a = (int)lists[i].size(), b = (int)lists[j].size();
      if (a != b) return sless(a, b);
      return i < j;
    });
    std::vector<std::vector<int>> res;
    for (int id : ids) res.push_back(lists[id]);
    return res;
  }
  std::vector<int> free_cpus(bool fe) const {   // freeCPUs
    std::map<int, std::vector<int>> cic;
    std::map<int, int> csock, cnode, nfree, sfree, colo;
    for (int c = 0; c < t.num_cpus; ++c) {
      if (!allocatable[c] || (fe && (xp(c) || xn(c)))) continue;
      cic[t.core[c]].push_back(c);
      csock[t.core[c]] = t.socket[c];
      cnode[t.core[c]] = t.node[c];
      nfree[t.node[c]]++;
      sfree[t.socket[c]]++;
    }
    for (auto& kv : sfree) {
      int n = 0;
      for (int c = 0; c < t.num_cpus; ++c)
        if (t.socket[c] == kv.first && result.has(c)) ++n;
      colo[kv.first] = n;
    }
    std::vector<int> cores;
    for (auto& kv : cic) cores.push_back(kv.first);
    std::sort(cores.begin(), cores.end(), [&](int i, int j) {
      int si = csock[i], sj = csock[j];
      if (colo[si] != colo[sj]) return colo[si] > colo[sj];
      if (sfree[si] != sfree[sj]) return sless(sfree[si], sfree[sj]);
      int ni = cnode[i], nj = cnode[j];
      if (nfree[ni] != nfree[nj]) return sless(nfree[ni], nfree[nj]);
      if (cic[i].size() != cic[j].size()) return cic[i].size() < cic[j].size();
      if (si != sj) return si < sj;
      if (max_ref > 1) {
        int a = core_ref(i), b = core_ref(j);
        if (a != b) return a < b;
      }
      return i < j;
    });
    std::vector<int> out;
    for (int core : cores) {
      std::vector<int> cpus = cic[core];
      if (max_ref > 1) sort_by_ref(cpus);
      out.insert(out.end(), cpus.begin(), cpus.end());
    }
    return out;
  }
  std::vector<int> spread(const std::vector<int>& cpus) const {   // spreadCPUs
    if ((int)cpus.size() <= t.cpc) return cpus;
    std::vector<int> prep = cpus, out;
    while (!prep.empty()) {
      std::vector<int> rest;
      std::set<int> seen;
      for (int c : prep) {
        if (!seen.insert(t.core[c]).second) { rest.push_back(c); continue; }
        out.push_back(c);
      }
      prep = rest;
    }
    return out;
  }
};

std::vector<int> head(const std::vector<int>& v, int n) { return std::vector<int>(v.begin(), v.begin() + n); }

bool take_preferred(const TopoClass& t, int max_ref, const CpuMask& available, const uint16_t* ref,
                    const uint8_t* ex, int needed, int bind, int excl, int strategy, CpuMask* out) {
  // takePreferredCPUs (cpu_accumulator.go:29-81) with preferredCPUs = {} (no reservations on this path)
  if (needed <= 0) { *out = CpuMask{}; return true; }
  return take_cpus(t, max_ref, available, ref, ex, needed, bind, excl, strategy, out);
}

// TopoDev (gs_cpuset_dev.h) of a topology; leaves ok = 0 outside the device scope
void make_topo_dev(const TopoClass& t, TopoDev* d) {
  std::memset(d, 0, sizeof(*d));
  if (!t.valid || t.num_cpus <= 0) return;
  std::vector<int> cores, nodes, socks;
  for (int c = 0; c < t.num_cpus; ++c) {
    cores.push_back(t.core[c]);
    nodes.push_back(t.node[c]);
    socks.push_back(t.socket[c]);
  }
  auto uniq = [](std::vector<int>& v) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
  };
  uniq(cores);
  uniq(nodes);
  uniq(socks);
  if ((int)cores.size() > TD_CORES || (int)nodes.size() > TD_NODES || (int)socks.size() > TD_SOCKETS) return;
  if (t.cpc < 1 || t.cpc > TD_POS || (int)nodes.size() != t.num_nodes) return;   // a NUMA node id in two sockets
  const bool wide = cores.size() > 64;
  auto idx = [](const std::vector<int>& v, int x) { return (int)(std::lower_bound(v.begin(), v.end(), x) - v.begin()); };
  int core_sock[TD_CORES], core_node[TD_CORES], node_sock[TD_NODES], npos[TD_CORES] = {0};
  std::fill(core_sock, core_sock + TD_CORES, -1);
  std::fill(core_node, core_node + TD_CORES, -1);
  std::fill(node_sock, node_sock + TD_NODES, -1);
  std::memset(d->core_cpu, 0xff, sizeof(d->core_cpu));
  std::memset(d->cpu_core, 0xff, sizeof(d->cpu_core));
  std::memset(d->cpu_pos, 0xff, sizeof(d->cpu_pos));
  cm_t node_m[TD_NODES] = {}, sock_m[TD_SOCKETS] = {}, pos_m[TD_POS] = {};
  for (int c = 0; c < t.num_cpus; ++c) {   // ascending CPU id: position j = rank of the CPU inside its core
    const int k = idx(cores, t.core[c]), n = idx(nodes, t.node[c]), s = idx(socks, t.socket[c]);
    if ((core_sock[k] >= 0 && core_sock[k] != s) || (core_node[k] >= 0 && core_node[k] != n) ||
        (node_sock[n] >= 0 && node_sock[n] != s))
      { std::memset(d, 0, sizeof(*d)); return; }
    core_sock[k] = s;
    core_node[k] = n;
    node_sock[n] = s;
    const int j = npos[k]++;
    // beyond 64 cores the 256 bits of a plane set hold two planes of 128 cores: <= 2 CPUs per core
    if (j >= TD_POS || (wide && j >= 2)) { std::memset(d, 0, sizeof(*d)); return; }
    const cm_t b = (cm_t)1 << k;
    d->core_cpu[k][j] = (uint8_t)c;
    d->cpu_core[c] = (uint8_t)k;
    d->cpu_pos[c] = (uint8_t)j;
    pos_m[j] |= b;
    node_m[n] |= b;
    sock_m[s] |= b;
    d->core_node[k] = (uint8_t)n;
  }
  auto put = [](uint64_t* w, cm_t m) { w[0] = cm_lo(m); w[1] = cm_hi(m); };
  for (int n = 0; n < TD_NODES; ++n) put(d->node_cores[n], node_m[n]);
  for (int s = 0; s < TD_SOCKETS; ++s) put(d->sock_cores[s], sock_m[s]);
  for (int j = 0; j < TD_POS; ++j) put(d->pos_cores[j], pos_m[j]);
  for (int n = 0; n < (int)nodes.size(); ++n) d->node_sock[n] = (uint8_t)node_sock[n];
  d->num_cpus = t.num_cpus;
  d->ncores = (int)cores.size();
  d->nnodes = (int)nodes.size();
  d->nsockets = (int)socks.size();
  d->cpc = t.cpc;
  d->cpn = t.cpn;
  d->cps = t.cps;
  d->wide = wide ? 1 : 0;
  d->ok = 1;
}

// node index (TopoDev order) of a NUMA node id, TD_NODES if the topology has no such node
int dev_node_index(const TopoClass& t, int node_id) {
  for (int c = 0; c < t.num_cpus; ++c)
    if (t.node[c] == node_id) return t.dev.core_node[t.dev.cpu_core[c]];
  return TD_NODES;
}

}  // namespace

static_assert(C_CPU_XC1 - C_CPU_UN0 == 10 && offsetof(CpuStateDev, xc1) == 80 && offsetof(CpuStateDev, rc) == 48,
              "the CPU state columns are CpuStateDev's first 11 words");

void numa_cpu_state(const NumaNode& n, bool default_most, CpuStateDev* cs) {
  std::memset(cs, 0, sizeof(*cs));
  cs->topo = -1;
  const TopoClass* t = n.topo.get();
  if (!t || !t->dev.ok) return;
  const TopoDev& d = t->dev;
  const int mr = n.max_ref();
  // the plane sets as CPU-indexed packed words: word / bit of CPU (core rank k, position j)
  auto set_cpu = [&](uint64_t* w, int c) {
    const int k = d.cpu_core[c], j = d.cpu_pos[c];
    const int bit = d.wide ? j * 128 + k : j * 64 + k;
    w[bit >> 6] |= 1ull << (bit & 63);
  };
  cm_t xc = 0;
  for (int c = 0; c < t->num_cpus; ++c) {   // getAvailableCPUs (node_allocation.go:142-162)
    const bool taken = n.ref[c] > 0 && n.ref[c] >= mr;
    const bool reserved = (n.cfg.reserved_cpus[c >> 6] >> (c & 63)) & 1;
    if (taken || reserved) set_cpu(cs->un, c);
    else if (mr == 2 && n.ref[c] == 1) set_cpu(cs->rc, c);   // the accumulator's RefCount
  }
  // exclusiveInCores / exclusiveInNUMANodes of newCPUAccumulator (cpu_accumulator.go:256-264): the CoreID /
  // NodeID of every allocated CPU (zero values for CPUs outside the topology)
  uint32_t xn = 0;
  for (int c = 0; c < GS_MAX_CPUS; ++c) {
    if (n.ref[c] == 0) continue;
    const int core = c < t->num_cpus ? t->core[c] : 0, node = c < t->num_cpus ? t->node[c] : 0;
    if (n.excl[c] == GS_CPU_EXCLUSIVE_PCPU_LEVEL) {
      for (int c2 = 0; c2 < t->num_cpus; ++c2)
        if (t->core[c2] == core) { xc |= (cm_t)1 << d.cpu_core[c2]; break; }
    } else if (n.excl[c] == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL) {
      const int ni = dev_node_index(*t, node);
      if (ni < TD_NODES) xn |= 1u << ni;
    }
  }
  cs->xc = cm_lo(xc);
  cs->xc1 = cm_hi(xc);
  const int nz = n.cfg.has_options ? n.cfg.num_zones : 0;
  uint32_t zidx = 0;
  for (int z = 0; z < GS_MAX_NUMA; ++z) {
    int ni = TD_NODES;
    if (z < nz) {
      const int id = n.cfg.zones[z].node_id;
      ni = dev_node_index(*t, id);
      uint64_t cnt = 0;
      for (int c = 0; c < t->num_cpus; ++c)
        if (n.ref[c] > 0 && t->node[c] == id) ++cnt;
      cs->zal |= cnt << (16 * z);
    }
    zidx |= (uint32_t)(ni < TD_NODES ? ni : 15) << (4 * z);
  }
  int strategy = n.cfg.numa_allocate_strategy;
  if (strategy == GS_NUMA_ALLOC_UNSET) strategy = default_most ? GS_NUMA_ALLOC_MOST_ALLOCATED : GS_NUMA_ALLOC_LEAST_ALLOCATED;
  cs->meta = xn | (zidx << CM_ZIDX_SHIFT) | (strategy == GS_NUMA_ALLOC_MOST_ALLOCATED ? CM_MOST : 0u) |
             (mr == 2 ? CM_MR2 : 0u);
  cs->topo = mr <= 2 ? n.cfg.topology : -1;
}

bool take_cpus(const TopoClass& t, int max_ref, const CpuMask& available, const uint16_t* ref, const uint8_t* ex,
               int needed, int bind, int excl, int strategy, CpuMask* out) {
  Acc a(t, max_ref, available, ref, ex, needed, excl, strategy);
  auto done = [&] { *out = a.result; return true; };
  if (a.satisfied()) return done();
  if (a.failed()) { *out = CpuMask{}; return false; }
  const bool full = bind == GS_CPU_BIND_FULL_PCPUS;
  if (full || t.cpc == 1) {
    if (a.needed <= t.cpn)
      for (bool fe : {true, false})
        for (auto& l : a.cores_in_node(true, fe))
          if ((int)l.size() >= a.needed) { a.take(head(l, a.needed)); return done(); }
    if (a.needed <= t.cps)
      for (auto& l : a.cores_in_socket(true))
        if ((int)l.size() >= a.needed) { a.take(head(l, a.needed)); return done(); }
    auto fr = a.cores_in_socket(true);
    go_sort_small(fr, [](const std::vector<int>& x, const std::vector<int>& y) { return x.size() > y.size(); });
    std::vector<std::vector<int>> unsat;
    for (auto& l : fr) {
      if (!a.needs((int)l.size())) unsat.push_back(l);
      else { a.take(l); if (a.satisfied()) return done(); }
    }
    if (a.needs(t.cpc)) {
      go_sort_small(unsat, [](const std::vector<int>& x, const std::vector<int>& y) { return x.size() < y.size(); });
      for (auto& l : unsat)
        for (int i = 0; i + t.cpc <= (int)l.size(); i += t.cpc) {
          a.take(std::vector<int>(l.begin() + i, l.begin() + i + t.cpc));
          if (a.satisfied()) return done();
          if (!a.needs(t.cpc)) break;
        }
    }
  }
  if (!full) {
    if (a.needed <= t.cpn)
      for (bool fe : {true, false})
        for (auto& l : a.cpus_in_node(fe))
          if ((int)l.size() >= a.needed) { a.take(head(a.spread(l), a.needed)); return done(); }
    if (a.needed <= t.cps)
      for (bool fe : {true, false})
        for (auto& l : a.cpus_in_socket(fe))
          if ((int)l.size() >= a.needed) { a.take(head(a.spread(l), a.needed)); return done(); }
  }
  for (bool fe : {true, false})
    for (int c : a.spread(a.free_cpus(fe))) {
      if (a.needs(1)) a.take({c});
      if (a.satisfied()) return done();
    }
  *out = CpuMask{};
  return false;
}

std::shared_ptr<TopoClass> make_topo(const gs_cpu_topology& in, const char** err) {
  auto t = std::make_shared<TopoClass>();
  if (in.num_cpus < 0 || in.num_cpus > GS_MAX_CPUS) { *err = "num_cpus outside [0, GS_MAX_CPUS]"; return nullptr; }
  t->num_cpus = in.num_cpus;
  std::set<int> sockets;
  std::set<std::pair<int, int>> nodes;
  std::set<std::tuple<int, int, int>> cores;
  std::map<int, int> core_node;
  for (int c = 0; c < in.num_cpus; ++c) {
    t->core[c] = in.core_id[c];
    t->socket[c] = in.socket_id[c];
    t->node[c] = in.node_id[c];
    sockets.insert(in.socket_id[c]);
    nodes.insert({in.socket_id[c], in.node_id[c]});
    cores.insert({in.socket_id[c], in.node_id[c], in.core_id[c]});
    auto it = core_node.find(in.core_id[c]);
    if (it != core_node.end() && it->second != in.node_id[c]) { *err = "a core spans NUMA nodes"; return nullptr; }
    core_node[in.core_id[c]] = in.node_id[c];
    if (in.node_id[c] >= 64) { *err = "NUMA node id >= 64"; return nullptr; }
  }
  if (sockets.size() > 12) { *err = "more than 12 sockets"; return nullptr; }
  t->num_sockets = (int)sockets.size();   // CPUTopologyBuilder counts (socket), (socket,node), (socket,node,core)
  t->num_nodes = (int)nodes.size();
  t->num_cores = (int)cores.size();
  t->valid = t->num_sockets && t->num_nodes && t->num_cores && t->num_cpus;
  t->cpc = t->num_cores ? t->num_cpus / t->num_cores : 0;
  t->cpn = t->num_nodes ? t->num_cpus / t->num_nodes : 0;
  t->cps = t->num_sockets ? t->num_cpus / t->num_sockets : 0;
  if (t->cpc > 255) { *err = "CPUsPerCore > 255"; return nullptr; }
  make_topo_dev(*t, &t->dev);
  return t;
}

void numa_add(NumaNode& n, const PodAllocRec& a) {
  if (n.pods.count(a.uid)) return;
  n.pods[a.uid] = a;
  for (int c = 0; c < GS_MAX_CPUS; ++c)
    if (a.cpus.has(c)) {
      n.excl[c] = (uint8_t)a.excl;
      n.ref[c]++;
    }
  for (const auto& z : a.numa) {
    ZoneAlloc& r = n.ares[z.node_id];
    if (z.mask & GS_USAGE_CPU) { r.cpu += z.cpu_milli; r.keys |= GS_USAGE_CPU; }
    if (z.mask & GS_USAGE_MEMORY) { r.mem += z.memory; r.keys |= GS_USAGE_MEMORY; }
  }
}

void numa_release(NumaNode& n, uint64_t uid) {
  auto it = n.pods.find(uid);
  if (it == n.pods.end()) return;
  PodAllocRec a = it->second;
  n.pods.erase(it);
  for (int c = 0; c < GS_MAX_CPUS; ++c)
    if (a.cpus.has(c) && n.ref[c] > 0 && --n.ref[c] == 0) n.excl[c] = 0;
  for (const auto& z : a.numa) {   // quotav1.SubtractWithNonNegativeResult
    auto r = n.ares.find(z.node_id);
    if (r == n.ares.end()) continue;
    if (r->second.keys & GS_USAGE_CPU) r->second.cpu = std::max<int64_t>(0, r->second.cpu - ((z.mask & GS_USAGE_CPU) ? z.cpu_milli : 0));
    if (r->second.keys & GS_USAGE_MEMORY) r->second.mem = std::max<int64_t>(0, r->second.mem - ((z.mask & GS_USAGE_MEMORY) ? z.memory : 0));
    if (z.mask & GS_USAGE_CPU) r->second.keys |= GS_USAGE_CPU;
    if (z.mask & GS_USAGE_MEMORY) r->second.keys |= GS_USAGE_MEMORY;
  }
}

CpuMask numa_available(const NumaNode& n) {
  CpuMask m;
  if (!n.topo) return m;
  int mr = n.max_ref();
  for (int c = 0; c < n.topo->num_cpus; ++c) {
    bool taken = n.ref[c] > 0 && n.ref[c] >= mr;
    bool reserved = (n.cfg.reserved_cpus[c >> 6] >> (c & 63)) & 1;
    if (!taken && !reserved) m.set(c);
  }
  return m;
}

void numa_derive(const NumaNode& n, bool default_most, int64_t* i64, int64_t* i32) {
  CpuStateDev cs;
  numa_cpu_state(n, default_most, &cs);
  for (int j = 0; j < 11; ++j) i64[C_CPU_UN0 + j] = reinterpret_cast<const int64_t*>(&cs)[j];
  i32[C_CPU_META] = (int32_t)cs.meta;
  i32[C_TOPO_DEV] = cs.topo;
  const gs_node_numa& g = n.cfg;
  const TopoClass* t = n.topo.get();
  uint32_t f = 0;
  if (g.has_options) f |= NF_HAS_OPTIONS;
  if (t) f |= NF_TOPO;
  if (t && t->valid) f |= NF_TOPO_VALID;
  if (g.node_amplification_invalid) f |= NF_AMP_INVALID;
  f |= (uint32_t)(g.numa_topology_policy & 3) << NF_POLICY_SHIFT;
  f |= (uint32_t)(g.node_cpu_bind_policy & 3) << NF_BIND_SHIFT;
  int nz = g.has_options ? g.num_zones : 0;
  f |= (uint32_t)nz << NF_ZONES_SHIFT;
  uint32_t f2 = 0;
  for (int z = 0; z < GS_MAX_NUMA; ++z) {
    i64[C_ZCAP_CPU0 + z] = i64[C_ZCAP_MEM0 + z] = i64[C_ZRAW_CPU0 + z] = i64[C_ZRAW_MEM0 + z] = 0;
    i32[C_ZFREE0 + z] = 0;
    i32[C_ZADJ0 + z] = 0;
    if (z >= nz) continue;
    const gs_numa_zone& zz = g.zones[z];
    if (zz.mask & GS_USAGE_CPU) { f |= 1u << (NF_ZCPU_SHIFT + z); i64[C_ZCAP_CPU0 + z] = zz.cpu_milli; }
    if (zz.mask & GS_USAGE_MEMORY) { f |= 1u << (NF_ZMEM_SHIFT + z); i64[C_ZCAP_MEM0 + z] = zz.memory; }
    auto it = n.ares.find(zz.node_id);
    if (it != n.ares.end()) {
      f2 |= 1u << (NF2_ENTRY_SHIFT + z);
      if (it->second.keys & GS_USAGE_CPU) f2 |= 1u << (NF2_ACPU_SHIFT + z);
      if (it->second.keys & GS_USAGE_MEMORY) f2 |= 1u << (NF2_AMEM_SHIFT + z);
      i64[C_ZRAW_CPU0 + z] = it->second.cpu;
      i64[C_ZRAW_MEM0 + z] = it->second.mem;
    }
  }
  if (t) f |= (uint32_t)(t->cpc & 255) << NF_CPC_SHIFT;
  double amp = g.cpu_amplification_ratio, namp = g.node_cpu_amplification_ratio;
  std::memcpy(&i64[C_AMP], &amp, 8);
  std::memcpy(&i64[C_NAMP], &namp, 8);
  int alloc_cpus = 0;
  if (t)
    for (int c = 0; c < GS_MAX_CPUS; ++c) alloc_cpus += n.ref[c] > 0;
  i32[C_NFLAGS] = (int32_t)f;
  i32[C_NFLAGS2] = (int32_t)f2;
  i32[C_ALLOC_CPUS] = alloc_cpus;
  i32[C_TFREE] = 0;
  if (t && t->valid) {
    CpuMask avail = numa_available(n);
    i32[C_TFREE] = count_available(*t, avail, -1).packed();
    for (int z = 0; z < nz; ++z) i32[C_ZFREE0 + z] = count_available(*t, avail, g.zones[z].node_id).packed();
  }
  if (t && amp > 1) {
    for (int z = 0; z < nz; ++z) {
      int64_t cs = 0;
      for (int c = 0; c < t->num_cpus; ++c)
        if (n.ref[c] > 0 && t->node[c] == g.zones[z].node_id) ++cs;
      cs *= 1000;
      i32[C_ZADJ0 + z] = (int32_t)(amplify(cs, amp) - cs);
    }
  }
}

bool numa_allocate_cpuset(const NumaNode& n, int num_cpus, int bind, bool required, int excl, int strategy,
                          const std::vector<gs_numa_zone>& split, CpuMask* out) {
  if (!n.topo_valid()) return false;
  const TopoClass& t = *n.topo;
  CpuMask available = numa_available(n);
  if (required) available = filter_required(t, bind, available);
  if (available.count() < num_cpus) return false;
  CpuMask result;
  int needed = num_cpus;
  if (!split.empty()) {
    for (const auto& z : split) {
      CpuMask in;
      for (int c = 0; c < t.num_cpus; ++c)
        if (available.has(c) && t.node[c] == z.node_id) in.set(c);
      int num = in.count();
      int node_needed = (int)(((z.mask & GS_USAGE_CPU) ? z.cpu_milli : 0) / 1000);
      if (node_needed < num) num = node_needed;
      CpuMask got;
      if (!take_preferred(t, n.max_ref(), in, n.ref, n.excl, num, bind, excl, strategy, &got)) return false;
      for (int w = 0; w < GS_CPU_WORDS; ++w) result.w[w] |= got.w[w];
    }
    needed -= result.count();
    if (needed != 0) return false;
  }
  if (needed > 0) {
    CpuMask rest = available;
    for (int w = 0; w < GS_CPU_WORDS; ++w) rest.w[w] &= ~result.w[w];
    CpuMask got;
    if (!take_preferred(t, n.max_ref(), rest, n.ref, n.excl, needed, bind, excl, strategy, &got)) return false;
    for (int w = 0; w < GS_CPU_WORDS; ++w) result.w[w] |= got.w[w];
  }
  if (required && !satisfied_required(t, bind, result)) return false;
  *out = result;
  return true;
}

}  // namespace gs

// Self-test of the bit-plane cpuset selection (gs_cpuset_dev.h, the code the commit kernel runs) against the
// host restatement on random compact topologies (core-major and sibling-interleaved CPU numbering, SMT 1/2/4,
// 1-2 sockets x 1-4 NUMA nodes; a third of them wide: up to 128 cores of SMT 1/2), random allocations with
// maxRefCount 1 or 2 (RefCounts 0-2), exclusivity and reservations, and random requests (bind and exclusive
// policies, strategies, NUMA splits); after each selection the device state update (td_reserve_update) is compared
// with the host's re-derivation of the node after addPodAllocation. Returns the number of mismatches; `msg`
// describes the first one. Test hook, not part of include/gpuscore.h.
extern "C" int gsx_cpuset_selftest(uint64_t seed, int iters, char* msg, size_t len) {
  using namespace gs;
  uint64_t s = seed;
  auto rnd = [&](int n) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (int)(z % (uint64_t)n);
  };
  int bad = 0;
  if (msg && len) msg[0] = 0;
  auto report = [&](int it, const char* what) {
    if (!bad && msg && len) snprintf(msg, len, "iteration %d: %s", it, what);
    ++bad;
  };
  static const int kCpc[] = {1, 2, 2, 4};
  for (int it = 0; it < iters; ++it) {
    const bool wide = rnd(3) == 0;
    int sockets = 1 + rnd(2), nps = 1 + rnd(4), cores_pn = 1 + rnd(6), cpc = kCpc[rnd(4)];
    if (wide) {   // 65-128 cores, SMT 1 / 2 (the C3 shapes: 2 sockets, 2 or 4 NUMA nodes, 32-128 cores)
      sockets = 2;
      nps = 1 + rnd(2);
      cpc = 1 + rnd(2);
      const int per = 128 / (sockets * nps);
      cores_pn = per / 2 + 1 + rnd(per / 2);
    }
    const bool interleave = rnd(2);
    const int ncores = sockets * nps * cores_pn;
    gs_cpu_topology in;
    std::memset(&in, 0, sizeof(in));
    in.num_cpus = ncores * cpc;
    for (int sk = 0; sk < sockets; ++sk)
      for (int nn = 0; nn < nps; ++nn)
        for (int co = 0; co < cores_pn; ++co)
          for (int th = 0; th < cpc; ++th) {
            const int gcore = (sk * nps + nn) * cores_pn + co;
            const int cpu = interleave ? th * ncores + gcore : gcore * cpc + th;
            in.core_id[cpu] = (sk << 16) | (nn * cores_pn + co);
            in.socket_id[cpu] = sk;
            in.node_id[cpu] = 2 * (sk * nps + nn);   // sparse ids
          }
    const char* err = nullptr;
    auto t = make_topo(in, &err);
    if (!t || !t->dev.ok) { report(it, "topology outside the device scope"); continue; }
    NumaNode n;
    n.cfg.has_options = 1;
    const int mr = 1 + rnd(2);
    n.cfg.max_ref_count = mr;
    n.cfg.topology = 0;
    n.topo = t;
    const int nnodes = sockets * nps, nz = nnodes < GS_MAX_NUMA ? nnodes : GS_MAX_NUMA;
    n.cfg.num_zones = nz;
    for (int z = 0; z < nz; ++z) {
      n.cfg.zones[z].node_id = 2 * z + (rnd(8) == 0 ? 1 : 0);   // now and then a zone the topology lacks
      n.cfg.zones[z].mask = GS_USAGE_CPU | GS_USAGE_MEMORY;
    }
    const int density = 1 + rnd(4);
    const bool some_excl = rnd(2);
    for (int c = 0; c < in.num_cpus; ++c) {
      if (rnd(density + 1) == 0) {
        n.ref[c] = (uint16_t)(1 + (mr == 2 ? rnd(2) : 0));
        const int e = some_excl ? rnd(6) : 5;
        n.excl[c] = (uint8_t)(e == 0 ? GS_CPU_EXCLUSIVE_PCPU_LEVEL : e == 1 ? GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL
                                                                    : GS_CPU_EXCLUSIVE_NONE);
      }
      if (rnd(24) == 0) n.cfg.reserved_cpus[c >> 6] |= 1ull << (c & 63);
    }
    n.cfg.numa_allocate_strategy = rnd(3);
    const bool dmost = rnd(2);
    int strategy = n.cfg.numa_allocate_strategy;
    if (strategy == GS_NUMA_ALLOC_UNSET) strategy = dmost ? GS_NUMA_ALLOC_MOST_ALLOCATED : GS_NUMA_ALLOC_LEAST_ALLOCATED;
    CpuStateDev cs;
    numa_cpu_state(n, dmost, &cs);
    if (cs.topo != 0) { report(it, "cpu state not device-eligible"); continue; }
    const CpuMask avail = numa_available(n);
    const int na = avail.count();
    const int needed = 1 + rnd(std::max(1, std::min(na + 2, 48)));
    const int bind = rnd(4), ep = rnd(3);
    const char* shape = wide ? "wide" : "compact";
    // takeCPUs over the whole available set
    CpuMask h;
    const bool hok = take_cpus(*t, mr, avail, n.ref, n.excl, needed, bind, ep, strategy, &h);
    uint64_t R[4], w[4];
    const bool dok = td_take_cpus(t->dev, cs, needed, bind, ep, strategy == GS_NUMA_ALLOC_MOST_ALLOCATED, R);
    td_to_cpus(t->dev, R, w);
    if (hok != dok || (hok && std::memcmp(w, h.w, sizeof(w)) != 0)) {
      char b[400];
      snprintf(b, sizeof b, "takeCPUs differs (host ok=%d dev ok=%d, need %d bind %d excl %d strategy %d, cpc %d, "
               "interleave %d, %s, %d cores, maxRefCount %d) host %llx %llx dev %llx %llx", hok, dok, needed, bind, ep,
               strategy, cpc, interleave, shape, ncores, mr, (unsigned long long)h.w[0], (unsigned long long)h.w[1],
               (unsigned long long)w[0], (unsigned long long)w[1]);
      if (getenv("GSX_SELFTEST_DUMP")) {
        fprintf(stderr, "cpu core node ref excl avail:\n");
        for (int c = 0; c < in.num_cpus; ++c)
          fprintf(stderr, "  %d %d %d %d %d %d\n", c, in.core_id[c], in.node_id[c], n.ref[c], n.excl[c], avail.has(c));
      }
      report(it, b);
      continue;
    }
    // allocateCPUSet with an optional NUMA split
    const bool required = rnd(2);
    std::vector<gs_numa_zone> split;
    uint32_t zkeys = 0;
    int64_t zcpu[4] = {0, 0, 0, 0};
    if (rnd(2)) {
      for (int z = 0; z < nz; ++z) {
        const int k = rnd(4);
        if (k == 0) continue;
        gs_numa_zone a{};
        a.node_id = n.cfg.zones[z].node_id;
        if (k != 2) { a.mask |= GS_USAGE_CPU; a.cpu_milli = 1000LL * rnd(needed + 1); zkeys |= 1u << z; zcpu[z] = a.cpu_milli; }
        if (k != 1) { a.mask |= GS_USAGE_MEMORY; a.memory = 1 << 20; zkeys |= 1u << (4 + z); }
        split.push_back(a);
      }
    }
    CpuMask h2;
    const bool hok2 = numa_allocate_cpuset(n, needed, bind, required, ep, strategy, split, &h2);
    const bool dok2 = td_allocate_cpuset(t->dev, cs, needed, bind, required, ep, zkeys, zcpu, R);
    td_to_cpus(t->dev, R, w);
    if (hok2 != dok2 || (hok2 && std::memcmp(w, h2.w, sizeof(w)) != 0)) {
      char b[256];
      snprintf(b, sizeof b, "allocateCPUSet differs (host ok=%d dev ok=%d, need %d bind %d required %d excl %d, "
               "%zu zones, %s, %d cores, maxRefCount %d)", hok2, dok2, needed, bind, required, ep, split.size(), shape,
               ncores, mr);
      report(it, b);
      continue;
    }
    // the device state update against the host's re-derivation after addPodAllocation
    if (hok2) {
      PodAllocRec rec;
      rec.uid = 1;
      rec.cpus = h2;
      rec.excl = ep;
      NumaNode n2 = n;
      numa_add(n2, rec);
      CpuStateDev cs2 = cs, want;
      const int added = td_reserve_update(t->dev, cs2, R, ep, nz);
      numa_cpu_state(n2, dmost, &want);
      int64_t i64[NUM_I64_COLS] = {0}, i32[NUM_I32_COLS] = {0};
      numa_derive(n2, dmost, i64, i32);
      int64_t b64[NUM_I64_COLS] = {0}, b32[NUM_I32_COLS] = {0};
      numa_derive(n, dmost, b64, b32);
      const bool stale = cs2.meta & CM_XSTALE;
      const bool same_x = stale || (cs2.xc == want.xc && cs2.xc1 == want.xc1 &&
                                    (cs2.meta & CM_XN_MASK) == (want.meta & CM_XN_MASK));
      if (td_counts(t->dev, cs2, -1) != (int32_t)i32[C_TFREE] ||
          std::memcmp(cs2.un, want.un, sizeof(want.un)) != 0 || std::memcmp(cs2.rc, want.rc, sizeof(want.rc)) != 0 ||
          cs2.zal != want.zal || !same_x || added != (int)(i32[C_ALLOC_CPUS] - b32[C_ALLOC_CPUS]) ||
          (cs2.meta & ~(CM_XN_MASK | CM_XSTALE)) != (want.meta & ~CM_XN_MASK)) {
        char b[200];
        snprintf(b, sizeof b, "post-Reserve CPU state differs (%s, %d cores, maxRefCount %d, excl %d)", shape, ncores,
                 mr, ep);
        report(it, b);
        continue;
      }
    }
  }
  return bad;
}
