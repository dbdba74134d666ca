// gs_numa_host.cpp — NodeNUMAResource host state of libgpuscore (see gs_numa_host.h).
// Reference paths are relative to pkg/scheduler/plugins/nodenumaresource/.
#include "gs_numa_host.h"

#include <algorithm>
#include <cmath>
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

}  // namespace

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

void numa_derive(const NumaNode& n, int64_t* i64, int64_t* i32) {
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
