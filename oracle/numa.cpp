// numa.cpp — CPU restatement of NodeNUMAResource + the NUMA topology manager. TEST INFRASTRUCTURE ONLY
// (see oracle.h / numa.h). Every function cites the reference file:line it restates; paths are relative to
// pkg/scheduler/plugins/nodenumaresource/ unless given in full.
#include "numa.h"

#include <algorithm>
#include <cmath>
#include <functional>

namespace orn {

namespace {

constexpr int64_t kMaxNodeScore = 100;

// extension.Amplify (apis/extension/node_resource_amplification.go:170-175)
int64_t amplify(int64_t origin, double ratio) {
  if (ratio <= 1) return origin;
  return (int64_t)std::ceil((double)origin * ratio);
}

int popcount(uint64_t m) { return __builtin_popcountll(m); }

bool scalar_slot(int r) { return (GS_SCALAR_RES_MASK >> r) & 1u; }

// Go 1.18 sort.Slice for n <= 12 (sort/zfuncversion.go quickSort_func: one ShellSort pass with gap 6, then
// insertionSort_func). Only the socket-list sorts of takeCPUs have ties (cpu_accumulator.go:142-144,161-163).
template <class T, class Less>
void go_sort_slice(std::vector<T>& v, Less less) {
  int n = (int)v.size();
  if (n > 12) {   // quickSort_func proper: not reachable with <= 12 sockets (enforced by build_topology)
    std::stable_sort(v.begin(), v.end(), less);
    return;
  }
  if (n > 1) {
    for (int i = 6; i < n; ++i)
      if (less(v[i], v[i - 6])) std::swap(v[i], v[i - 6]);
    for (int i = 1; i < n; ++i)
      for (int j = i; j > 0 && less(v[j], v[j - 1]); --j) std::swap(v[j], v[j - 1]);
  }
}

CPUSet cpus_of(const CPUDetails& d) {
  CPUSet s;
  for (auto& kv : d) s.insert(kv.first);
  return s;
}
CPUDetails keep_only(const CPUDetails& d, const CPUSet& cpus) {   // cpu_topology.go KeepOnly
  CPUDetails r;
  for (auto& kv : d)
    if (cpus.count(kv.first)) r[kv.first] = kv.second;
  return r;
}
CPUSet cpus_in_numa(const CPUDetails& d, int node) {
  CPUSet s;
  for (auto& kv : d)
    if (kv.second.node == node) s.insert(kv.first);
  return s;
}
CPUSet cpus_in_socket(const CPUDetails& d, int socket) {
  CPUSet s;
  for (auto& kv : d)
    if (kv.second.socket == socket) s.insert(kv.first);
  return s;
}
std::set<int> cores_of(const CPUDetails& d) {
  std::set<int> s;
  for (auto& kv : d) s.insert(kv.second.core);
  return s;
}
std::vector<int> cpus_in_core(const CPUDetails& d, int core) {
  std::vector<int> v;
  for (auto& kv : d)
    if (kv.second.core == core) v.push_back(kv.first);
  return v;   // ascending (map order)
}
CPUSet set_minus(const CPUSet& a, const CPUSet& b) {
  CPUSet r;
  for (int x : a)
    if (!b.count(x)) r.insert(x);
  return r;
}
CPUSet set_and(const CPUSet& a, const CPUSet& b) {
  CPUSet r;
  for (int x : a)
    if (b.count(x)) r.insert(x);
  return r;
}

}  // namespace

RL rl_add(const RL& a, const RL& b) {
  RL r = a;
  for (int k = 0; k < GS_NUM_RES; ++k)
    if (b.has(k)) r.set(k, r.get(k) + b.v[k]);
  return r;
}

RL rl_sub_nonneg(const RL& a, const RL& b) {   // k8s.io/apiserver quota/v1 SubtractWithNonNegativeResult
  RL r;
  for (int k = 0; k < GS_NUM_RES; ++k) {
    if (a.has(k)) {
      int64_t q = a.v[k] - (b.has(k) ? b.v[k] : 0);
      r.set(k, q > 0 ? q : 0);
    } else if (b.has(k)) {
      r.set(k, 0);
    }
  }
  return r;
}

// CPUTopologyBuilder.AddCPUInfo over the reported detail (topology_options.go:167-173, cpu_topology.go:40-68)
std::shared_ptr<CPUTopology> build_topology(const gs_cpu_topology& t) {
  auto topo = std::make_shared<CPUTopology>();
  std::map<int, std::map<int, std::set<int>>> tracker;
  for (int c = 0; c < t.num_cpus && c < GS_MAX_CPUS; ++c) {
    CPUInfo info;
    info.cpu = c;
    info.core = t.core_id[c];
    info.node = t.node_id[c];
    info.socket = t.socket_id[c];
    topo->details[c] = info;
    auto& sk = tracker[info.socket];
    auto& nd = sk[info.node];
    nd.insert(info.core);
  }
  topo->num_sockets = (int)tracker.size();
  for (auto& s : tracker) {
    topo->num_nodes += (int)s.second.size();
    for (auto& n : s.second) topo->num_cores += (int)n.second.size();
  }
  topo->num_cpus = (int)topo->details.size();
  return topo;
}

std::shared_ptr<CPUTopology> build_test_topology(int sockets, int nodes_per_socket, int cores_per_node, int cpc) {
  auto topo = std::make_shared<CPUTopology>();
  topo->num_sockets = sockets;
  topo->num_nodes = nodes_per_socket * sockets;
  topo->num_cores = cores_per_node * nodes_per_socket * sockets;
  topo->num_cpus = cpc * topo->num_cores;
  int node = 0, core = 0, cpu = 0;
  for (int s = 0; s < sockets; ++s)
    for (int n = 0; n < nodes_per_socket; ++n, ++node)
      for (int c = 0; c < cores_per_node; ++c, ++core)
        for (int p = 0; p < cpc; ++p, ++cpu) topo->details[cpu] = CPUInfo{cpu, core, node, s, 0, 0};
  return topo;
}

// ---- NodeAllocation (node_allocation.go:63-177) ---------------------------------------------------
void NodeAllocation::update(const PodAllocation& a, const CPUTopology* topo) {
  release(a.uid);
  add(a, topo);
}

void NodeAllocation::add(const PodAllocation& a, const CPUTopology* topo) {   // addPodAllocation :82-110
  if (pods.count(a.uid)) return;
  pods[a.uid] = a;
  for (int cpu : a.cpus) {
    auto it = allocated_cpus.find(cpu);
    CPUInfo info;
    if (it != allocated_cpus.end()) info = it->second;
    else if (topo && topo->details.count(cpu)) info = topo->details.at(cpu);
    else info.cpu = cpu;
    info.excl = a.excl;
    info.ref++;
    allocated_cpus[cpu] = info;
  }
  for (size_t i = 0; i < a.numa.size(); ++i) {
    const NUMANodeResource& nr = a.numa[i];
    auto it = allocated_res.find(nr.node);
    if (it == allocated_res.end()) it = allocated_res.emplace(nr.node, NUMANodeResource{(int)i, RL{}}).first;
    it->second.res = rl_add(it->second.res, nr.res);
  }
}

void NodeAllocation::release(uint64_t uid) {   // :112-140
  auto pit = pods.find(uid);
  if (pit == pods.end()) return;
  PodAllocation a = pit->second;
  pods.erase(pit);
  for (int cpu : a.cpus) {
    auto it = allocated_cpus.find(cpu);
    if (it == allocated_cpus.end()) continue;
    if (--it->second.ref == 0) allocated_cpus.erase(it);
  }
  for (const auto& nr : a.numa) {
    auto it = allocated_res.find(nr.node);
    if (it != allocated_res.end()) it->second.res = rl_sub_nonneg(it->second.res, nr.res);
  }
}

void NodeAllocation::available_cpus(const CPUTopology& topo, int max_ref, const CPUSet& reserved,
                                    const CPUSet& preferred, CPUSet* avail, CPUDetails* allocated) const {   // :142-162
  CPUDetails info = allocated_cpus;
  for (int cpu : preferred) {
    auto it = info.find(cpu);
    if (it != info.end() && --it->second.ref == 0) info.erase(it);
  }
  CPUSet alloc;
  for (auto& kv : info)
    if (kv.second.ref >= max_ref) alloc.insert(kv.first);
  if (avail) *avail = set_minus(set_minus(cpus_of(topo.details), alloc), reserved);
  if (allocated) *allocated = info;
}

void NodeAllocation::available_numa(const TopologyOptions& o, std::map<int, RL>* total_avail,
                                    std::map<int, RL>* total_alloc) const {   // :164-177
  for (const auto& nr : o.numa) {
    RL allocated_res_l;
    auto it = allocated_res.find(nr.node);
    if (it != allocated_res.end()) {
      allocated_res_l = it->second.res;
      if (o.amp_ratio > 1) {
        int64_t cs = 0;
        for (auto& kv : allocated_cpus)
          if (kv.second.node == nr.node) ++cs;
        cs *= 1000;
        int64_t amplified = amplify(cs, o.amp_ratio);
        int64_t q = allocated_res_l.get(GS_RES_CPU);
        allocated_res_l.set(GS_RES_CPU, q - cs + amplified);
      }
      allocated_res_l = rl_sub_nonneg(allocated_res_l, RL{});   // reusableResources: none without reservations
      if (total_alloc) (*total_alloc)[nr.node] = allocated_res_l;
    }
    if (total_avail) (*total_avail)[nr.node] = rl_sub_nonneg(nr.res, allocated_res_l);
  }
}

// ---- cpuAccumulator (cpu_accumulator.go:249-822) ---------------------------------------------------
namespace {

struct Acc {
  const CPUTopology& topo;
  int max_ref;
  CPUDetails allocatable;
  int needed;
  bool exclusive;
  std::set<int> excl_cores, excl_nodes;
  int excl_policy;
  int strategy;
  CPUSet result;

  Acc(const CPUTopology& t, int mr, const CPUSet& available, const CPUDetails& allocated, int n, int ep, int st)
      : topo(t), max_ref(mr), needed(n), excl_policy(ep), strategy(st) {   // newCPUAccumulator :262-298
    for (auto& kv : allocated) {
      if (kv.second.excl == GS_CPU_EXCLUSIVE_PCPU_LEVEL) excl_cores.insert(kv.second.core);
      else if (kv.second.excl == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL) excl_nodes.insert(kv.second.node);
    }
    exclusive = ep == GS_CPU_EXCLUSIVE_PCPU_LEVEL || ep == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL;
    allocatable = keep_only(t.details, available);
    if (max_ref > 1)
      for (auto& kv : allocatable) {
        auto it = allocated.find(kv.first);
        kv.second.ref = it != allocated.end() ? it->second.ref : 0;
      }
  }
  bool most() const { return strategy == GS_NUMA_ALLOC_MOST_ALLOCATED; }
  void take(const std::vector<int>& cpus) {   // :300-315
    for (int c : cpus) {
      result.insert(c);
      allocatable.erase(c);
      if (exclusive) {
        const CPUInfo& info = topo.details.at(c);
        if (excl_policy == GS_CPU_EXCLUSIVE_PCPU_LEVEL) excl_cores.insert(info.core);
        else if (excl_policy == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL) excl_nodes.insert(info.node);
      }
    }
    needed -= (int)cpus.size();
  }
  bool needs(int n) const { return needed >= n; }
  bool satisfied() const { return needed < 1; }
  bool failed() const { return needed > (int)allocatable.size(); }
  bool excl_pcpu(const CPUInfo& i) const { return excl_policy == GS_CPU_EXCLUSIVE_PCPU_LEVEL && excl_cores.count(i.core); }
  bool excl_numa(const CPUInfo& i) const {
    return excl_policy == GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL && excl_nodes.count(i.node);
  }
  std::vector<int> extract_cpu(const std::vector<int>& cpus) const {   // :343-355
    std::vector<int> sel;
    std::set<int> cores;
    for (int c : cpus) {
      int core = topo.details.at(c).core;
      if (cores.insert(core).second) sel.push_back(c);
    }
    return sel;
  }
  int core_ref(const CPUDetails& d, int core) const {   // getCoreRefCount :791-798
    int r = 0;
    for (auto& kv : d)
      if (kv.second.core == core) r += kv.second.ref;
    return r;
  }
  void sort_cores(const CPUDetails& d, std::vector<int>& cores, std::map<int, std::vector<int>>& cic) const {   // :357-379
    if (cores.size() <= 1) return;
    std::sort(cores.begin(), cores.end(), [&](int i, int j) {
      size_t ic = cic[i].size(), jc = cic[j].size();
      if (ic != jc) return ic > jc;
      if (max_ref > 1) {
        int ir = core_ref(d, i), jr = core_ref(d, j);
        if (ir != jr) return ir < jr;
      }
      return i < j;
    });
  }
  void sort_by_ref(std::vector<int>& cpus) const {   // sortCPUsByRefCount :800-811
    std::sort(cpus.begin(), cpus.end(), [&](int i, int j) {
      int ir = allocatable.at(i).ref, jr = allocatable.at(j).ref;
      if (ir != jr) return ir < jr;
      return i < j;
    });
  }
  bool score_less(int a, int b) const { return most() ? a < b : a > b; }

  // freeCoresInNode :381-461
  std::vector<std::vector<int>> free_cores_in_node(bool full, bool filter_excl) const {
    std::map<int, int> socket_free;
    std::map<int, std::vector<int>> cic;
    for (auto& kv : allocatable) {
      if (filter_excl && excl_numa(kv.second)) continue;
      cic[kv.second.core].push_back(kv.first);
      socket_free[kv.second.socket]++;
    }
    std::map<int, std::vector<int>> cores_in_nodes;
    for (auto& kv : cic) {
      if (full && (int)kv.second.size() != topo.cpus_per_core()) continue;
      const CPUInfo& info = allocatable.at(kv.second[0]);
      cores_in_nodes[info.node].push_back(kv.first);
    }
    std::vector<int> node_ids;
    std::map<int, std::vector<int>> cpus_in_nodes;
    for (auto& kv : cores_in_nodes) {
      node_ids.push_back(kv.first);
      std::vector<int> cores = kv.second;
      sort_cores(allocatable, cores, cic);
      std::vector<int> out;
      for (int c : cores) {
        std::vector<int> cpus = cic[c];
        std::sort(cpus.begin(), cpus.end());
        out.insert(out.end(), cpus.begin(), cpus.end());
      }
      cpus_in_nodes[kv.first] = out;
    }
    std::sort(node_ids.begin(), node_ids.end(), [&](int i, int j) {
      const CPUInfo& ii = allocatable.at(cpus_in_nodes[i][0]);
      const CPUInfo& jj = allocatable.at(cpus_in_nodes[j][0]);
      int inf = (int)cpus_in_nodes[i].size(), jnf = (int)cpus_in_nodes[j].size();
      if (inf != jnf) return score_less(inf, jnf);
      int isf = socket_free.count(ii.socket) ? socket_free.at(ii.socket) : 0;
      int jsf = socket_free.count(jj.socket) ? socket_free.at(jj.socket) : 0;
      if (isf != jsf) return score_less(isf, jsf);
      return i < j;
    });
    std::vector<std::vector<int>> res;
    for (int n : node_ids) res.push_back(cpus_in_nodes[n]);
    return res;
  }

  // freeCoresInSocket :463-525
  std::vector<std::vector<int>> free_cores_in_socket(bool full) const {
    std::map<int, std::vector<int>> cic;
    for (auto& kv : allocatable) cic[kv.second.core].push_back(kv.first);
    std::map<int, std::vector<int>> cores_in_sockets;
    for (auto& kv : cic) {
      if (full && (int)kv.second.size() != topo.cpus_per_core()) continue;
      cores_in_sockets[allocatable.at(kv.second[0]).socket].push_back(kv.first);
    }
    std::vector<int> ids;
    std::map<int, std::vector<int>> cis;
    for (auto& kv : cores_in_sockets) {
      ids.push_back(kv.first);
      std::vector<int> cores = kv.second;
      sort_cores(allocatable, cores, cic);
      std::vector<int> out;
      for (int c : cores) {
        std::vector<int> cpus = cic[c];
        std::sort(cpus.begin(), cpus.end());
        out.insert(out.end(), cpus.begin(), cpus.end());
      }
      cis[kv.first] = out;
    }
    std::sort(ids.begin(), ids.end(), [&](int i, int j) {
      int a = (int)cis[i].size(), b = (int)cis[j].size();
      if (a != b) return score_less(a, b);
      return i < j;
    });
    std::vector<std::vector<int>> res;
    for (int s : ids) res.push_back(cis[s]);
    return res;
  }

  // freeCPUsInNode :527-598
  std::vector<std::vector<int>> free_cpus_in_node(bool filter_excl) const {
    std::map<int, std::vector<int>> cin;
    std::map<int, int> node_free, socket_free;
    for (auto& kv : allocatable) {
      if (filter_excl && (excl_pcpu(kv.second) || excl_numa(kv.second))) continue;
      cin[kv.second.node].push_back(kv.first);
      node_free[kv.second.node]++;
      socket_free[kv.second.socket]++;
    }
    std::vector<int> ids;
    for (auto& kv : cin) {
      ids.push_back(kv.first);
      std::vector<int>& cpus = kv.second;
      std::sort(cpus.begin(), cpus.end());
      if (max_ref > 1) sort_by_ref(cpus);
      if (filter_excl) cpus = extract_cpu(cpus);
    }
    std::sort(ids.begin(), ids.end(), [&](int i, int j) {
      const CPUInfo& ii = allocatable.at(cin[i][0]);
      const CPUInfo& jj = allocatable.at(cin[j][0]);
      int inf = node_free[ii.node], jnf = node_free[jj.node];
      int isf = socket_free[ii.socket], jsf = socket_free[jj.socket];
      if (inf != jnf) return score_less(inf, jnf);
      if (isf != jsf) return score_less(isf, jsf);
      return i < j;
    });
    std::vector<std::vector<int>> res;
    for (int n : ids) res.push_back(cin[n]);
    return res;
  }

  // freeCPUsInSocket :600-647
  std::vector<std::vector<int>> free_cpus_in_socket(bool filter_excl) const {
    std::map<int, std::vector<int>> cis;
    for (auto& kv : allocatable) {
      if (filter_excl && excl_pcpu(kv.second)) continue;
      cis[kv.second.socket].push_back(kv.first);
    }
    std::vector<int> ids;
    for (auto& kv : cis) {
      ids.push_back(kv.first);
      std::vector<int>& cpus = kv.second;
      std::sort(cpus.begin(), cpus.end());
      if (max_ref > 1) sort_by_ref(cpus);
      if (filter_excl) cpus = extract_cpu(cpus);
    }
    std::sort(ids.begin(), ids.end(), [&](int i, int j) {
      int a = (int)cis[i].size(), b = (int)cis[j].size();
      if (a != b) return score_less(a, b);
      return i < j;
    });
    std::vector<std::vector<int>> res;
    for (int s : ids) res.push_back(cis[s]);
    return res;
  }

  // freeCPUs :649-789
  std::vector<int> free_cpus(bool filter_excl) const {
    std::map<int, std::vector<int>> cic;
    std::map<int, int> core_socket, core_node, node_free, socket_free;
    for (auto& kv : allocatable) {
      if (filter_excl && (excl_pcpu(kv.second) || excl_numa(kv.second))) continue;
      cic[kv.second.core].push_back(kv.first);
      core_socket[kv.second.core] = kv.second.socket;
      core_node[kv.second.core] = kv.second.node;
      node_free[kv.second.node]++;
      socket_free[kv.second.socket]++;
    }
    std::map<int, int> colo;
    for (auto& kv : socket_free) colo[kv.first] = (int)set_and(cpus_in_socket(topo.details, kv.first), result).size();
    std::vector<int> cores;
    for (auto& kv : cic) cores.push_back(kv.first);
    std::sort(cores.begin(), cores.end(), [&](int i, int j) {
      int is = core_socket[i], js = core_socket[j];
      if (colo[is] != colo[js]) return colo[is] > colo[js];
      if (socket_free[is] != socket_free[js]) return score_less(socket_free[is], socket_free[js]);
      int in = core_node[i], jn = core_node[j];
      if (node_free[in] != node_free[jn]) return score_less(node_free[in], node_free[jn]);
      if (cic[i].size() != cic[j].size()) return cic[i].size() < cic[j].size();
      if (is != js) return is < js;
      if (max_ref > 1) {
        int ir = core_ref(allocatable, i), jr = core_ref(allocatable, j);
        if (ir != jr) return ir < jr;
      }
      return i < j;
    });
    std::vector<int> res;
    for (int c : cores) {
      std::vector<int> cpus = cic[c];
      std::sort(cpus.begin(), cpus.end());
      if (max_ref > 1) sort_by_ref(cpus);
      res.insert(res.end(), cpus.begin(), cpus.end());
    }
    return res;
  }

  std::vector<int> spread(const std::vector<int>& cpus) const {   // spreadCPUs :813-822
    if ((int)cpus.size() <= topo.cpus_per_core()) return cpus;
    std::vector<int> prepared = cpus, out;
    while (!prepared.empty()) {
      std::vector<int> reserved;
      std::set<int> seen;
      for (int c : prepared) {
        int core = topo.details.at(c).core;
        if (seen.count(core)) { reserved.push_back(c); continue; }
        out.push_back(c);
        seen.insert(core);
      }
      prepared = reserved;
    }
    return out;
  }
};

std::vector<int> prefix(const std::vector<int>& v, int n) { return std::vector<int>(v.begin(), v.begin() + n); }

}  // namespace

// takeCPUs (cpu_accumulator.go:83-247)
bool take_cpus(const CPUTopology& topo, int max_ref, const CPUSet& available, const CPUDetails& allocated, int needed,
               int bind, int excl, int strategy, CPUSet* result) {
  Acc acc(topo, max_ref, available, allocated, needed, excl, strategy);
  if (acc.satisfied()) { *result = acc.result; return true; }
  if (acc.failed()) { result->clear(); return false; }
  const bool full = bind == GS_CPU_BIND_FULL_PCPUS;
  const int cpc = topo.cpus_per_core();
  if (full || cpc == 1) {
    if (acc.needed <= topo.cpus_per_node()) {
      for (bool fe : {true, false})
        for (auto& cpus : acc.free_cores_in_node(true, fe))
          if ((int)cpus.size() >= acc.needed) { acc.take(prefix(cpus, acc.needed)); *result = acc.result; return true; }
    }
    if (acc.needed <= topo.cpus_per_socket()) {
      for (auto& cpus : acc.free_cores_in_socket(true))
        if ((int)cpus.size() >= acc.needed) { acc.take(prefix(cpus, acc.needed)); *result = acc.result; return true; }
    }
    auto free = acc.free_cores_in_socket(true);
    go_sort_slice(free, [](const std::vector<int>& a, const std::vector<int>& b) { return a.size() > b.size(); });
    std::vector<std::vector<int>> unsatisfied;
    for (auto& cpus : free) {
      if (!acc.needs((int)cpus.size())) {
        unsatisfied.push_back(cpus);
      } else {
        acc.take(cpus);
        if (acc.satisfied()) { *result = acc.result; return true; }
      }
    }
    if (acc.needs(cpc)) {
      free = unsatisfied;
      go_sort_slice(free, [](const std::vector<int>& a, const std::vector<int>& b) { return a.size() < b.size(); });
      for (auto& cpus : free) {
        for (int i = 0; i + cpc <= (int)cpus.size(); i += cpc) {
          acc.take(std::vector<int>(cpus.begin() + i, cpus.begin() + i + cpc));
          if (acc.satisfied()) { *result = acc.result; return true; }
          if (!acc.needs(cpc)) break;
        }
      }
    }
  }
  if (!full) {
    if (acc.needed <= topo.cpus_per_node()) {
      for (bool fe : {true, false})
        for (auto& cpus : acc.free_cpus_in_node(fe))
          if ((int)cpus.size() >= acc.needed) {
            acc.take(prefix(acc.spread(cpus), acc.needed));
            *result = acc.result;
            return true;
          }
    }
    if (acc.needed <= topo.cpus_per_socket()) {
      for (bool fe : {true, false})
        for (auto& cpus : acc.free_cpus_in_socket(fe))
          if ((int)cpus.size() >= acc.needed) {
            acc.take(prefix(acc.spread(cpus), acc.needed));
            *result = acc.result;
            return true;
          }
    }
  }
  for (bool fe : {true, false}) {
    for (int c : acc.spread(acc.free_cpus(fe))) {
      if (acc.needs(1)) acc.take({c});
      if (acc.satisfied()) { *result = acc.result; return true; }
    }
  }
  result->clear();
  return false;
}

namespace {

// takePreferredCPUs (cpu_accumulator.go:29-81)
bool take_preferred(const CPUTopology& topo, int max_ref, CPUSet available, const CPUSet& preferred_in,
                    const CPUDetails& allocated, int needed, int bind, int excl, int strategy, CPUSet* out) {
  CPUSet result;
  CPUSet preferred = set_and(available, preferred_in);
  if (!preferred.empty()) {
    int n = std::min<int>(needed, (int)preferred.size());
    if (!take_cpus(topo, max_ref, preferred, allocated, n, bind, excl, strategy, &result)) return false;
    needed -= (int)result.size();
    available = set_minus(available, preferred);
  }
  if (needed > 0) {
    CPUSet cpus;
    if (!take_cpus(topo, max_ref, available, allocated, needed, bind, excl, strategy, &cpus)) return false;
    for (int c : cpus) result.insert(c);
  }
  *out = result;
  return true;
}

// filterCPUsByRequiredCPUBindPolicy (resource_manager.go:534-566)
CPUSet filter_by_required(int policy, const CPUSet& available, const CPUDetails& details_in, int cpc) {
  CPUDetails details = keep_only(details_in, available);
  if (policy == GS_CPU_BIND_FULL_PCPUS) {
    CPUSet r;
    for (int core : cores_of(details)) {
      auto cpus = cpus_in_core(details, core);
      if ((int)cpus.size() == cpc) r.insert(cpus.begin(), cpus.end());
    }
    return r;
  }
  if (policy == GS_CPU_BIND_SPREAD_BY_PCPUS) {
    CPUSet r;
    for (int core : cores_of(details)) r.insert(cpus_in_core(details, core)[0]);
    return r;
  }
  return available;
}

// satisfiedRequiredCPUBindPolicy (resource_manager.go:568-589)
bool satisfied_required(int policy, const CPUSet& cpus, const CPUTopology& topo) {
  CPUDetails d = keep_only(topo.details, cpus);
  if (policy == GS_CPU_BIND_FULL_PCPUS) return (int)cores_of(d).size() * topo.cpus_per_core() == (int)cpus.size();
  if (policy == GS_CPU_BIND_SPREAD_BY_PCPUS) return cores_of(d).size() == cpus.size();
  return true;
}

struct ResourceOptions {   // resource_manager.go:47-60
  int num_cpus = 0;
  bool request_bind = false;
  RL requests, original;
  bool required = false;
  int bind = GS_CPU_BIND_UNSET;
  int excl = GS_CPU_EXCLUSIVE_NONE;
  CPUSet preferred;
  Hint hint;
  bool scorer = false;
};

int64_t least_requested(int64_t req, int64_t cap) {   // least_allocated.go:49-58
  if (cap == 0) return 0;
  if (req > cap) return 0;
  return ((cap - req) * kMaxNodeScore) / cap;
}
int64_t most_requested(int64_t req, int64_t cap) {    // most_allocated.go:45-55
  if (cap == 0) return 0;
  if (req > cap) req = cap;
  return (req * kMaxNodeScore) / cap;
}

// resourceAllocationScorer.score (scoring.go:187-203) over framework.Resource views of ResourceLists:
// allocatable/requested/pod are RLs (absent key = 0; scalar keys must be present in allocatable).
int64_t alloc_score(const NumaArgs& a, int type, const RL& requested, const RL& allocatable, const RL& pod) {
  int64_t node_score = 0, weight_sum = 0;
  for (int r = 0; r < GS_NUM_RES; ++r) {
    int64_t w = a.weights[r];
    if (w == 0) continue;
    int64_t preq = pod.get(r);
    if (preq == 0 && scalar_slot(r)) continue;       // calculateResourceAllocatableRequest :205-226
    int64_t al, rq;
    if (scalar_slot(r)) {
      if (!allocatable.has(r)) continue;
      al = allocatable.v[r];
      rq = requested.get(r) + preq;
    } else {
      al = allocatable.get(r);
      rq = requested.get(r) + preq;
    }
    if (al == 0) continue;
    node_score += (type == GS_SCORING_MOST_ALLOCATED ? most_requested(rq, al) : least_requested(rq, al)) * w;
    weight_sum += w;
  }
  if (weight_sum == 0) return 0;
  return node_score / weight_sum;
}

RL node_rl(const int64_t* v) {   // NodeInfo.Allocatable / Requested as a ResourceList (every slot present)
  RL r;
  for (int k = 0; k < GS_NUM_RES - 1; ++k) r.set(k, v[k]);
  return r;
}

// requestCPUBind (util.go:105-122); returns a reason (0 ok)
int request_cpu_bind(const PreState& st, int node_bind, bool* out) {
  *out = false;
  if (st.request_bind) { *out = true; return 0; }
  int64_t cpu = st.requests.get(GS_RES_CPU);
  if (cpu == 0) return 0;
  if (node_bind != GS_NODE_CPU_BIND_NONE) {
    if (cpu % 1000 != 0) return GS_NUMA_INVALID_REQUESTED_CPUS;
    *out = true;
  }
  return 0;
}

// resourceManager.GetAvailableCPUs (resource_manager.go:391-404): returns false on ErrInvalidCPUTopology
bool get_available_cpus(const NodeNUMA& n, const CPUSet& preferred, CPUSet* avail, CPUDetails* allocated) {
  const TopologyOptions& o = n.opts;
  if (!o.topo) {
    if (avail) avail->clear();
    if (allocated) allocated->clear();
    return true;
  }
  if (!o.topo->valid()) return false;
  n.alloc.available_cpus(*o.topo, o.max_ref, o.reserved, preferred, avail, allocated);
  return true;
}

// getResourceOptions (plugin.go:481-532) without reservations (reservationReservedCPUs empty)
ResourceOptions resource_options(const PreState& st, const NodeNUMA& n, bool rb, const Hint& hint) {
  const TopologyOptions& o = n.opts;
  ResourceOptions ro;
  ro.requests = st.requests;
  if (rb && o.amp_ratio > 1 && ro.requests.get(GS_RES_CPU) != 0)   // AmplifyResourceList(requests, ratios, cpu)
    ro.requests.set(GS_RES_CPU, amplify(ro.requests.v[GS_RES_CPU], o.amp_ratio));
  ro.original = st.requests;
  ro.num_cpus = st.num_cpus;
  ro.request_bind = rb;
  // getCPUBindPolicy (util.go:85-103)
  if (st.required != GS_CPU_BIND_UNSET) {
    ro.bind = st.required;
    ro.required = true;
  } else {
    ro.bind = st.preferred;
    if (o.node_cpu_bind == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS) { ro.bind = GS_CPU_BIND_SPREAD_BY_PCPUS; ro.required = true; }
    else if (o.node_cpu_bind == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY) { ro.bind = GS_CPU_BIND_FULL_PCPUS; ro.required = true; }
  }
  ro.excl = st.excl;
  ro.hint = hint;
  return ro;
}

int numa_strategy(const NumaArgs& a, const TopologyOptions& o) {   // GetNUMAAllocateStrategy (util.go:35-41)
  if (o.numa_alloc_strategy != GS_NUMA_ALLOC_UNSET) return o.numa_alloc_strategy;
  return a.numa_scoring == GS_SCORING_MOST_ALLOCATED ? GS_NUMA_ALLOC_MOST_ALLOCATED : GS_NUMA_ALLOC_LEAST_ALLOCATED;
}

std::vector<int> bits_of(uint64_t m) {
  std::vector<int> v;
  for (int i = 0; i < 64; ++i)
    if (m >> i & 1) v.push_back(i);
  return v;
}

// allocateRes (resource_manager.go:252-271)
void allocate_res(int64_t* avail, int64_t* req, int64_t* allocated) {
  if (*avail > *req) { *avail -= *req; *allocated = *req; *req = 0; }
  else if (*avail < *req) { *req -= *avail; *allocated = *avail; *avail = 0; }
  else { *allocated = *avail; *avail = 0; *req = 0; }
}

// allocateResourcesByHint (resource_manager.go:195-250)
bool allocate_by_hint(const NodeNUMA& n, const ResourceOptions& ro, std::vector<NUMANodeResource>* out) {
  const TopologyOptions& o = n.opts;
  if (o.numa.empty()) return false;
  std::map<int, RL> avail;
  n.alloc.available_numa(o, &avail, nullptr);
  RL req = ro.request_bind ? ro.original : ro.requests;
  uint32_t inter = 0;
  std::vector<NUMANodeResource> result;
  for (int id : bits_of(ro.hint.mask)) {
    RL& al = avail[id];
    NUMANodeResource r{id, RL{}};
    for (int k = 0; k < GS_NUM_RES; ++k) {
      if (!req.has(k) || !al.has(k)) continue;
      inter |= 1u << k;
      int64_t got = 0;
      allocate_res(&al.v[k], &req.v[k], &got);
      if (got != 0) r.res.set(k, got);
    }
    if (!r.res.is_zero()) result.push_back(r);
    if (req.is_zero()) break;
  }
  for (int k = 0; k < GS_NUM_RES; ++k)
    if ((inter >> k & 1) && req.get(k) != 0) return false;   // "Insufficient NUMA <resource>"
  *out = result;
  return true;
}

// allocateCPUSet (resource_manager.go:273-360)
bool allocate_cpuset(const NumaArgs& a, const NodeNUMA& n, const std::vector<NUMANodeResource>& numa,
                     const ResourceOptions& ro, CPUSet* out) {
  const TopologyOptions& o = n.opts;
  CPUSet available;
  CPUDetails allocated;
  if (!get_available_cpus(n, ro.preferred, &available, &allocated)) return false;
  if (!o.topo) {   // CPUTopology nil: the reference dereferences it below; nothing can be allocated here
    if (ro.num_cpus > 0) return false;
    out->clear();
    return true;
  }
  const CPUTopology& topo = *o.topo;
  if (ro.required) available = filter_by_required(ro.bind, available, keep_only(topo.details, available), topo.cpus_per_core());
  if ((int)available.size() < ro.num_cpus) return false;
  CPUSet result;
  int strategy = numa_strategy(a, o);
  int needed = ro.num_cpus;
  if (!numa.empty()) {
    for (const auto& nr : numa) {
      CPUSet in_node = set_and(available, cpus_in_numa(topo.details, nr.node));
      int num = (int)in_node.size();
      int node_needed = (int)(nr.res.get(GS_RES_CPU) / 1000);
      if (node_needed < num) num = node_needed;
      CPUSet cpus;
      if (!take_preferred(topo, o.max_ref, in_node, ro.preferred, allocated, num, ro.bind, ro.excl, strategy, &cpus))
        return false;
      result.insert(cpus.begin(), cpus.end());
    }
    needed -= (int)result.size();
    if (needed != 0) return false;
  }
  if (needed > 0) {
    CPUSet rem;
    if (!take_preferred(topo, o.max_ref, set_minus(available, result), ro.preferred, allocated, needed, ro.bind, ro.excl,
                        strategy, &rem))
      return false;
    result.insert(rem.begin(), rem.end());
  }
  if (ro.required && !satisfied_required(ro.bind, result, topo)) return false;
  *out = result;
  return true;
}

// resourceManager.Allocate (resource_manager.go:171-193)
bool allocate(const NumaArgs& a, const NodeNUMA& n, uint64_t uid, const ResourceOptions& ro, PodAllocation* out) {
  PodAllocation pa;
  pa.uid = uid;
  pa.excl = ro.excl;
  if (ro.hint.has_mask) {
    if (!allocate_by_hint(n, ro, &pa.numa)) return false;
  }
  if (ro.request_bind) {
    if (!allocate_cpuset(a, n, pa.numa, ro, &pa.cpus)) return false;
  }
  *out = pa;
  return true;
}

// ---- hints (resource_manager.go:122-169, 418-532) -------------------------------------------------
struct HintsMap {
  bool nil = true;                          // GetPodTopologyHints returned nil (error)
  std::map<int, std::vector<Hint>> hints;   // resource slot -> hints
};

// bitmask.IterateBitMasks (pkg/util/bitmask/bitmask.go:206-222)
void iterate_bitmasks(const std::vector<int>& bits, const std::function<void(uint64_t)>& cb) {
  std::function<void(size_t, uint64_t, int, int)> rec = [&](size_t start, uint64_t accum, int have, int size) {
    if (have == size) { cb(accum); return; }
    for (size_t i = start; i < bits.size(); ++i) rec(i + 1, accum | (1ull << bits[i]), have + 1, size);
  };
  for (int size = 1; size <= (int)bits.size(); ++size) rec(0, 0, 0, size);
}

HintsMap topology_hints(const NumaArgs& a, const NodeNUMA& n, const ResourceOptions& ro) {
  HintsMap hm;
  const TopologyOptions& o = n.opts;
  if (o.numa.empty()) return hm;
  std::map<int, RL> total_avail;
  n.alloc.available_numa(o, &total_avail, nullptr);
  if (ro.required) {   // trimNUMANodeResources :140-169
    CPUSet available;
    if (!get_available_cpus(n, ro.preferred, &available, nullptr)) return hm;
    CPUDetails details = o.topo ? keep_only(o.topo->details, available) : CPUDetails{};
    int cpc = o.topo ? o.topo->cpus_per_core() : 0;
    for (auto& kv : total_avail) {
      int64_t q = kv.second.get(GS_RES_CPU);
      if (q == 0) continue;
      CPUSet in_node = cpus_in_numa(details, kv.first);
      if ((int64_t)in_node.size() * 1000 >= q) in_node = filter_by_required(ro.bind, in_node, details, cpc);
      if ((int64_t)in_node.size() * 1000 < q) kv.second.set(GS_RES_CPU, (int64_t)in_node.size() * 1000);
    }
  }
  // generateResourceHints :418-492
  const RL& pod = ro.requests;
  hm.nil = false;
  std::map<int, int> min_size;
  for (int k = 0; k < GS_NUM_RES; ++k)
    if (pod.has(k)) min_size[k] = (int)o.numa.size();
  std::vector<int> nodes;
  for (auto& nr : o.numa) nodes.push_back(nr.node);
  uint32_t total_names = 0;
  auto gen = [&](uint64_t mask, int64_t score, const RL& total, const RL& free, const std::vector<int>& names) {
    for (int r : names)
      if (total.get(r) < pod.get(r)) return;
    int cnt = popcount(mask);
    for (int r : names)
      if (cnt < min_size[r]) min_size[r] = cnt;
    for (int r : names)
      if (free.get(r) < pod.get(r)) return;
    for (int r : names) hm.hints[r].push_back(Hint{true, mask, false, score});
  };
  std::vector<int> mem_names;
  if (pod.has(GS_RES_MEMORY)) mem_names.push_back(GS_RES_MEMORY);
  iterate_bitmasks(nodes, [&](uint64_t mask) {
    RL available, total;
    for (int id : bits_of(mask)) {
      auto it = total_avail.find(id);
      if (it != total_avail.end()) available = rl_add(available, it->second);
      for (auto& nr : o.numa)
        if (nr.node == id) { total = rl_add(total, nr.res); break; }
    }
    int64_t score = 0;
    if (ro.scorer) score = alloc_score(a, a.numa_scoring, rl_sub_nonneg(total, available), total, pod);
    gen(mask, score, total, available, mem_names);
    for (int k = 0; k < GS_NUM_RES; ++k) {
      if (!pod.has(k)) continue;
      if (total.has(k)) total_names |= 1u << k;
      if (k == GS_RES_MEMORY) continue;
      gen(mask, score, total, available, {k});
    }
  });
  for (auto& kv : hm.hints)
    for (auto& h : kv.second) h.preferred = popcount(h.mask) == min_size[kv.first];
  for (int k = 0; k < GS_NUM_RES; ++k)
    if (pod.has(k) && (total_names >> k & 1) && !hm.hints.count(k)) hm.hints[k] = {};
  return hm;
}

// ---- policies (frameworkext/topologymanager/policy*.go) -------------------------------------------
// Resource iteration order of filterProvidersHints (policy.go:108, a Go map): fixed to sorted resource
// names (cpu < ephemeral-storage < kubernetes.io/* < memory); `reverse` flips it to expose order dependence.
const int kNameOrder[GS_NUM_RES - 1] = {GS_RES_CPU, GS_RES_EPHEMERAL, GS_RES_BATCH_CPU, GS_RES_BATCH_MEMORY,
                                        GS_RES_MID_CPU, GS_RES_MID_MEMORY, GS_RES_MEMORY};

std::vector<std::vector<Hint>> filter_providers(const HintsMap& hm, bool reverse) {   // policy.go:98-126
  std::vector<std::vector<Hint>> all;
  if (hm.nil || hm.hints.empty()) {
    all.push_back({Hint{false, 0, true, 0}});
    return all;
  }
  for (int i = 0; i < GS_NUM_RES - 1; ++i) {
    int k = kNameOrder[reverse ? GS_NUM_RES - 2 - i : i];
    auto it = hm.hints.find(k);
    if (it == hm.hints.end()) continue;
    if (it->second.empty()) all.push_back({Hint{false, 0, false, 0}});
    else all.push_back(it->second);
  }
  return all;
}

bool narrower(uint64_t a, uint64_t b) {   // bitmask.IsNarrowerThan
  if (popcount(a) == popcount(b)) return a < b;
  return popcount(a) < popcount(b);
}

Hint merge_filtered(uint64_t def, const std::vector<std::vector<Hint>>& lists) {   // policy.go:128-186
  Hint best{true, def, false, 0};
  std::vector<Hint> perm;
  std::function<void(size_t)> rec = [&](size_t i) {
    if (i == lists.size()) {
      bool pref = true;
      uint64_t m = def;
      for (const Hint& h : perm) {
        m &= h.has_mask ? h.mask : def;
        if (!h.preferred) pref = false;
      }
      Hint merged{true, m, pref, 0};
      if (popcount(m) == 0) return;
      for (const Hint& v : perm)
        if (v.has_mask && v.mask == m && v.score > merged.score) merged.score = v.score;
      if (merged.preferred && !best.preferred) { best = merged; return; }
      if (!merged.preferred && best.preferred) return;
      if (!narrower(merged.mask, best.mask)) {
        if (popcount(merged.mask) == popcount(best.mask) && merged.score > best.score) best = merged;
        return;
      }
      best = merged;
      return;
    }
    for (const Hint& h : lists[i]) {
      perm.push_back(h);
      rec(i + 1);
      perm.pop_back();
    }
  };
  rec(0);
  return best;
}

// policy.Merge -> (best, admit)
// the policy's Merge over filterProvidersHints' lists (policy_best_effort.go:43-48, policy_restricted.go:42-47,
// policy_single_numa_node.go:48-78): the merged hint; the admit verdict
bool policy_merge_filtered(int policy, uint64_t def, std::vector<std::vector<Hint>> filtered, Hint* best) {
  if (policy == GS_NUMA_POLICY_SINGLE_NUMA_NODE) {   // policy_single_numa_node.go:48-78
    for (auto& l : filtered) {
      std::vector<Hint> keep;
      for (auto& h : l) {
        if (!h.has_mask && h.preferred) keep.push_back(h);
        if (h.has_mask && popcount(h.mask) == 1 && h.preferred) keep.push_back(h);
      }
      l = keep;
    }
    *best = merge_filtered(def, filtered);
    if (best->mask == def) *best = Hint{false, 0, best->preferred, 0};
    return best->preferred;
  }
  *best = merge_filtered(def, filtered);
  if (policy == GS_NUMA_POLICY_RESTRICTED) return best->preferred;   // policy_restricted.go:42-47
  return true;                                                       // policy_best_effort.go:43-48
}

// topologyManager.calculateAffinity (manager.go:82-90): every provider's lists (filterProvidersHints), then Merge
bool policy_merge(int policy, const std::vector<int>& numa_nodes, const HintsMap& hm, bool reverse, Hint* best,
                  const std::vector<std::vector<Hint>>* provider2 = nullptr) {
  uint64_t def = 0;
  for (int id : numa_nodes) def |= 1ull << id;
  std::vector<std::vector<Hint>> lists = filter_providers(hm, reverse);
  if (provider2)
    for (const auto& l : *provider2) lists.push_back(l.empty() ? std::vector<Hint>{Hint{false, 0, false, 0}} : l);
  return policy_merge_filtered(policy, def, lists, best);
}

}  // namespace

// ---- plugin ---------------------------------------------------------------------------------------

// PreFilter (plugin.go:219-269)
PreState prefilter(const NumaArgs& a, const gs_pod& pod) {
  PreState st;
  for (int k = 0; k < GS_NUM_RES - 1; ++k)
    if (pod.request_mask >> k & 1) st.requests.set(k, pod.requests[k]);
  if (st.requests.is_zero()) { st.skip = true; return st; }
  int64_t cpu = st.requests.get(GS_RES_CPU);
  st.num_cpus = (int)(cpu / 1000);
  // AllowUseCPUSet (util.go:43-50)
  bool allow = (pod.qos_class == GS_QOS_LSE || pod.qos_class == GS_QOS_LSR) && pod.priority_class == GS_PRIO_PROD;
  if (allow) {
    int bind = pod.preferred_cpu_bind_policy;
    if (bind == GS_CPU_BIND_UNSET || bind == GS_CPU_BIND_DEFAULT) bind = a.default_bind;
    int required = pod.required_cpu_bind_policy;
    if (required == GS_CPU_BIND_DEFAULT) required = a.default_bind;
    if (required != GS_CPU_BIND_UNSET) bind = required;
    if (bind == GS_CPU_BIND_FULL_PCPUS || bind == GS_CPU_BIND_SPREAD_BY_PCPUS) {
      if (cpu % 1000 != 0) { st.status = GS_NUMA_INVALID_REQUESTED_CPUS; return st; }
      if (cpu > 0) {
        st.request_bind = true;
        st.required = required;
        st.preferred = bind;
        st.excl = pod.preferred_cpu_exclusive_policy;
      }
    }
  }
  return st;
}

namespace {

// filterAmplifiedCPUs (plugin.go:340-373)
int filter_amplified(const NodeNUMA& n, const NodeView& v, int64_t pod_milli, bool rb) {
  if (pod_milli == 0) return 0;
  const TopologyOptions& o = n.opts;
  if (o.node_amp_invalid) return GS_NUMA_INVALID_AMP_RATIO;
  double ratio = o.node_amp_ratio;
  if (ratio <= 1) return 0;
  if (rb) pod_milli = amplify(pod_milli, ratio);
  CPUDetails allocated;
  if (!get_available_cpus(n, CPUSet{}, nullptr, &allocated)) return GS_NUMA_AVAILABLE_CPUS_ERROR;
  int64_t alloc_milli = (int64_t)allocated.size() * 1000;
  int64_t requested = v.req_cpu;
  if (requested >= alloc_milli && alloc_milli > 0) requested = requested - alloc_milli + amplify(alloc_milli, ratio);
  if (pod_milli > v.alloc_cpu - requested) return GS_NUMA_INSUFFICIENT_AMP_CPU;
  return 0;
}

}  // namespace

int filter(const NumaArgs& a, const PreState& st, const NodeNUMA& n, const NodeView& v, Hint* affinity,
           bool* has_affinity, bool reverse, const std::vector<std::vector<Hint>>* provider2) {
  *has_affinity = false;
  if (st.status) return st.status;
  if (st.skip) return 0;
  const TopologyOptions& o = n.opts;
  bool rb = false;
  if (int rc = request_cpu_bind(st, o.node_cpu_bind, &rb)) return rc;
  if (int rc = filter_amplified(n, v, st.requests.get(GS_RES_CPU), rb)) return rc;
  if (rb) {
    if (!(o.topo && o.topo->valid())) return GS_NUMA_INVALID_TOPOLOGY;
    int required = st.required;
    if (o.node_cpu_bind == GS_NODE_CPU_BIND_FULL_PCPUS_ONLY) required = GS_CPU_BIND_FULL_PCPUS;
    else if (o.node_cpu_bind == GS_NODE_CPU_BIND_SPREAD_BY_PCPUS) required = GS_CPU_BIND_SPREAD_BY_PCPUS;
    if (st.required != GS_CPU_BIND_UNSET && st.required != required) return GS_NUMA_BIND_POLICY_CONFLICT;
    if (required == GS_CPU_BIND_FULL_PCPUS && st.num_cpus % o.topo->cpus_per_core() != 0) return GS_NUMA_SMT_ALIGNMENT;
    if (required != GS_CPU_BIND_UNSET && o.numa_policy == GS_NUMA_POLICY_NONE) {
      ResourceOptions ro = resource_options(st, n, rb, Hint{});
      PodAllocation pa;
      if (!allocate(a, n, 0, ro, &pa)) return GS_NUMA_ALLOCATE_FAILED;
    }
  }
  if (o.numa_policy != GS_NUMA_POLICY_NONE) {
    // FilterByNUMANode (topology_hint.go:30-39) -> topologyManager.Admit (manager.go:58-80)
    if (o.numa.empty()) return GS_NUMA_MISSING_NUMA_RESOURCES;
    std::vector<int> ids;
    for (auto& nr : o.numa) ids.push_back(nr.node);
    ResourceOptions ro = resource_options(st, n, rb, Hint{});
    ro.scorer = true;
    HintsMap hm = topology_hints(a, n, ro);   // GetPodTopologyHints (topology_hint.go:41-67); errors -> nil
    Hint best;
    if (!policy_merge(o.numa_policy, ids, hm, reverse, &best, provider2)) return GS_NUMA_AFFINITY_ERROR;
    *affinity = best;
    *has_affinity = true;
    ResourceOptions ro2 = resource_options(st, n, rb, best);   // provider Allocate (topology_hint.go:69-96)
    PodAllocation pa;
    if (!allocate(a, n, 0, ro2, &pa)) return GS_NUMA_ADMIT_ALLOCATE_FAILED;
  }
  return 0;
}

// resourceManager.GetTopologyHints (resource_manager.go:122-137) for the pod PreFilter described, on one node, with the
// options the provider passes (topology_hint.go:41-67). Test hook for resource_manager_test.go
// TestResourceManagerGetTopologyHint: entries (resource slot, mask, preferred) in hint order; an empty list for a
// resource is one entry with preferred = 2. Returns 1 for a nil map (an error), 0 otherwise, or the bind status.
int topology_hints_test(const NumaArgs& a, const PreState& st, const NodeNUMA& n, int32_t* res, uint64_t* masks,
                        uint8_t* preferred, uint32_t cap, uint32_t* count) {
  *count = 0;
  if (st.status) return st.status;
  bool rb = false;
  if (int rc = request_cpu_bind(st, n.opts.node_cpu_bind, &rb)) return rc;
  ResourceOptions ro = resource_options(st, n, rb, Hint{});
  ro.scorer = true;
  HintsMap hm = topology_hints(a, n, ro);
  if (hm.nil) return 1;
  uint32_t k = 0;
  auto put = [&](int r, uint64_t m, uint8_t p) {
    if (k < cap) { res[k] = r; masks[k] = m; preferred[k] = p; }
    ++k;
  };
  for (auto& kv : hm.hints) {
    if (kv.second.empty()) put(kv.first, 0, 2);
    for (const Hint& h : kv.second) put(kv.first, h.mask, h.preferred ? 1 : 0);
  }
  *count = k;
  return 0;
}

int64_t score(const NumaArgs& a, const PreState& st, const NodeNUMA& n, const NodeView& v, const Hint& affinity) {
  if (st.status || st.skip) return 0;
  const TopologyOptions& o = n.opts;
  bool rb = false;
  if (request_cpu_bind(st, o.node_cpu_bind, &rb)) return 0;
  if (rb && !(o.topo && o.topo->valid())) return 0;
  ResourceOptions ro = resource_options(st, n, rb, affinity);
  RL alloc_rl = node_rl(v.alloc), req_rl = node_rl(v.req);
  if (o.numa_policy == GS_NUMA_POLICY_NONE) {   // scoreWithAmplifiedCPUs (scoring.go:99-116)
    int64_t qty = st.requests.get(GS_RES_CPU);
    if (qty == 0 || o.amp_ratio <= 1) return alloc_score(a, a.scoring, req_rl, alloc_rl, ro.requests);
    CPUDetails allocated;
    if (!get_available_cpus(n, ro.preferred, nullptr, &allocated)) return 0;
    int64_t am = (int64_t)allocated.size() * 1000;
    req_rl.set(GS_RES_CPU, req_rl.get(GS_RES_CPU) - am + amplify(am, o.amp_ratio));
    return alloc_score(a, a.scoring, req_rl, alloc_rl, ro.requests);
  }
  PodAllocation pa;
  if (!allocate(a, n, 0, ro, &pa)) return 0;
  // calculateAllocatableAndRequested (scoring.go:118-164)
  RL allocatable, requested;
  if (!pa.numa.empty()) {
    std::map<int, RL> by_node;
    n.alloc.available_numa(o, nullptr, &by_node);
    for (const auto& nr : pa.numa) {
      auto it = by_node.find(nr.node);
      if (it != by_node.end() && it->second.keys) requested = rl_add(requested, it->second);
      for (const auto& z : o.numa)
        if (z.node == nr.node) { allocatable = rl_add(allocatable, z.res); break; }
    }
  } else {
    allocatable = alloc_rl;
    requested = req_rl;
  }
  if (!pa.cpus.empty()) {
    CPUDetails allocated;
    if (o.topo) n.alloc.available_cpus(*o.topo, o.max_ref, o.reserved, set_minus(ro.preferred, pa.cpus), nullptr, &allocated);
    requested.set(GS_RES_CPU, amplify((int64_t)allocated.size() * 1000, o.amp_ratio));
  }
  return alloc_score(a, a.scoring, requested, allocatable, ro.requests);
}

int reserve(const NumaArgs& a, const PreState& st, NodeNUMA& n, const gs_pod& pod, const Hint& affinity,
            PodAllocation* out) {
  if (out) *out = PodAllocation{};
  if (st.status) return -1;
  if (st.skip) return 0;
  const TopologyOptions& o = n.opts;
  bool rb = false;
  if (request_cpu_bind(st, o.node_cpu_bind, &rb)) return -1;
  if (!rb && o.numa_policy == GS_NUMA_POLICY_NONE) return 0;
  if (rb && !(o.topo && o.topo->valid())) return -1;
  ResourceOptions ro = resource_options(st, n, rb, affinity);
  PodAllocation pa;
  if (!allocate(a, n, pod.uid, ro, &pa)) return -1;
  // resourceManager.Update (resource_manager.go:362-373): skipped without a valid CPU topology
  if (o.topo && o.topo->valid()) n.alloc.update(pa, o.topo.get());
  if (out) *out = pa;
  return 0;
}

}  // namespace orn

// ---- test entry: the topology-manager Merge over explicit hint lists (policy_test.go vectors) ----------------
// lists as filterProvidersHints produced them: nlists lists, list i holding lens[i] hints (has_mask, mask,
// preferred) taken in order from the flat arrays. Returns the admit verdict; *out = the merged hint.
extern "C" int or_policy_merge(int policy, uint64_t numa_mask, int nlists, const int32_t* lens, const uint8_t* has_mask,
                               const uint64_t* masks, const uint8_t* preferred, uint8_t* out_has_mask,
                               uint64_t* out_mask, uint8_t* out_preferred) {
  if (policy == GS_NUMA_POLICY_NONE) {   // policy_none.go:40-42: an empty hint, admitted
    *out_has_mask = 0; *out_mask = 0; *out_preferred = 0;
    return 1;
  }
  std::vector<std::vector<orn::Hint>> lists(nlists);
  int k = 0;
  for (int i = 0; i < nlists; ++i)
    for (int j = 0; j < lens[i]; ++j, ++k) lists[i].push_back(orn::Hint{has_mask[k] != 0, masks[k], preferred[k] != 0, 0});
  orn::Hint best;
  const bool admit = orn::policy_merge_filtered(policy, numa_mask, lists, &best);
  *out_has_mask = best.has_mask ? 1 : 0;
  *out_mask = best.has_mask ? best.mask : 0;
  *out_preferred = best.preferred ? 1 : 0;
  return admit ? 1 : 0;
}

// The same with per-hint scores (NUMATopologyHint.Score, which mergeFilteredHints compares between equally wide masks)
extern "C" int or_policy_merge_scored(int policy, uint64_t numa_mask, int nlists, const int32_t* lens,
                                      const uint8_t* has_mask, const uint64_t* masks, const uint8_t* preferred,
                                      const int64_t* scores, uint8_t* out_has_mask, uint64_t* out_mask,
                                      uint8_t* out_preferred) {
  if (policy == GS_NUMA_POLICY_NONE) {
    *out_has_mask = 0; *out_mask = 0; *out_preferred = 0;
    return 1;
  }
  std::vector<std::vector<orn::Hint>> lists(nlists);
  int k = 0;
  for (int i = 0; i < nlists; ++i)
    for (int j = 0; j < lens[i]; ++j, ++k)
      lists[i].push_back(orn::Hint{has_mask[k] != 0, masks[k], preferred[k] != 0, scores[k]});
  orn::Hint best;
  const bool admit = orn::policy_merge_filtered(policy, numa_mask, lists, &best);
  *out_has_mask = best.has_mask ? 1 : 0;
  *out_mask = best.has_mask ? best.mask : 0;
  *out_preferred = best.preferred ? 1 : 0;
  return admit ? 1 : 0;
}

// bitmask.IterateBitMasks (bitmask.go:206-222): the masks of every non-empty subset of `bits` in visit order
extern "C" int or_iterate_bitmasks(const int32_t* bits, int nbits, uint64_t* out, int cap) {
  std::vector<int> b(bits, bits + nbits);
  int n = 0;
  orn::iterate_bitmasks(b, [&](uint64_t m) { if (n < cap) out[n] = m; ++n; });
  return n;
}

