// numa.h — CPU restatement of NodeNUMAResource (pkg/scheduler/plugins/nodenumaresource) and the
// NUMA topology manager (pkg/scheduler/frameworkext/topologymanager). TEST INFRASTRUCTURE ONLY:
// internal to oracle/ (see oracle.h), never linked by koordinator_amd/.
//
// Data structures follow the reference shapes: cpuset.CPUSet = ordered set, CPUDetails = map keyed by
// cpu id, corev1.ResourceList = (slot -> quantity) with an explicit key mask, NodeAllocation with per-pod
// records. Reference paths are relative to hormes/koordinator.
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "../include/gpuscore.h"

namespace orn {

using CPUSet = std::set<int>;

// corev1.ResourceList over the gs_resource slots (cpu in milli, others in units)
struct RL {
  int64_t v[GS_NUM_RES] = {0};
  uint32_t keys = 0;
  bool has(int r) const { return keys & (1u << r); }
  int64_t get(int r) const { return has(r) ? v[r] : 0; }
  void set(int r, int64_t x) { v[r] = x; keys |= 1u << r; }
  bool is_zero() const {   // quotav1.IsZero
    for (int r = 0; r < GS_NUM_RES; ++r)
      if (has(r) && v[r] != 0) return false;
    return true;
  }
};
RL rl_add(const RL& a, const RL& b);                 // quotav1.Add
RL rl_sub_nonneg(const RL& a, const RL& b);          // quotav1.SubtractWithNonNegativeResult

struct CPUInfo {
  int cpu = 0, core = 0, node = 0, socket = 0;
  int ref = 0;
  int excl = GS_CPU_EXCLUSIVE_NONE;
};
using CPUDetails = std::map<int, CPUInfo>;

struct CPUTopology {   // cpu_topology.go:25-31
  int num_cpus = 0, num_cores = 0, num_nodes = 0, num_sockets = 0;
  CPUDetails details;
  bool valid() const { return num_sockets && num_nodes && num_cores && num_cpus; }
  int cpus_per_core() const { return num_cores ? num_cpus / num_cores : 0; }
  int cpus_per_socket() const { return num_sockets ? num_cpus / num_sockets : 0; }
  int cpus_per_node() const { return num_nodes ? num_cpus / num_nodes : 0; }
};
std::shared_ptr<CPUTopology> build_topology(const gs_cpu_topology& t);   // CPUTopologyBuilder
// buildCPUTopologyForTest (cpu_accumulator_test.go:30-57)
std::shared_ptr<CPUTopology> build_test_topology(int sockets, int nodes_per_socket, int cores_per_node, int cpus_per_core);

struct NUMANodeResource {
  int node = 0;
  RL res;
};

struct TopologyOptions {   // topology_options.go:40-50 (+ node labels resolved by the caller)
  bool present = false;
  std::shared_ptr<CPUTopology> topo;    // nullptr: CPUTopology == nil
  CPUSet reserved;
  int max_ref = 0;
  int node_cpu_bind = GS_NODE_CPU_BIND_NONE;
  int numa_policy = GS_NUMA_POLICY_NONE;
  int numa_alloc_strategy = GS_NUMA_ALLOC_UNSET;
  double amp_ratio = 0;                 // AmplificationRatios[cpu]
  double node_amp_ratio = -1;           // node annotation ratio (filterAmplifiedCPUs)
  bool node_amp_invalid = false;
  std::vector<NUMANodeResource> numa;
};

struct PodAllocation {   // node_allocation.go:40-47
  uint64_t uid = 0;
  CPUSet cpus;
  int excl = GS_CPU_EXCLUSIVE_NONE;
  std::vector<NUMANodeResource> numa;
};

struct NodeAllocation {  // node_allocation.go:32-38
  std::map<uint64_t, PodAllocation> pods;
  CPUDetails allocated_cpus;
  std::map<int, NUMANodeResource> allocated_res;
  void update(const PodAllocation& a, const CPUTopology* topo);
  void add(const PodAllocation& a, const CPUTopology* topo);
  void release(uint64_t uid);
  void available_cpus(const CPUTopology& topo, int max_ref, const CPUSet& reserved, const CPUSet& preferred,
                      CPUSet* avail, CPUDetails* allocated) const;
  void available_numa(const TopologyOptions& o, std::map<int, RL>* total_avail, std::map<int, RL>* total_alloc) const;
};

struct Hint {            // topologymanager.NUMATopologyHint
  bool has_mask = false; // NUMANodeAffinity != nil
  uint64_t mask = 0;
  bool preferred = false;
  int64_t score = 0;
};

struct NodeNUMA {
  TopologyOptions opts;
  NodeAllocation alloc;
};

struct NumaArgs {
  int default_bind = GS_CPU_BIND_FULL_PCPUS;
  int scoring = GS_SCORING_LEAST_ALLOCATED;
  int numa_scoring = GS_SCORING_LEAST_ALLOCATED;
  int64_t weights[GS_NUM_RES] = {0};
};

struct PreState {        // preFilterState (plugin.go:172-181)
  int status = 0;        // gs_numa_reason of a PreFilter failure (applies to every node)
  bool skip = false;
  bool request_bind = false;
  RL requests;
  int required = GS_CPU_BIND_UNSET, preferred = GS_CPU_BIND_UNSET, excl = GS_CPU_EXCLUSIVE_NONE;
  int num_cpus = 0;
};

struct NodeView {        // what the plugin reads from NodeInfo
  int64_t alloc_cpu, alloc_mem, req_cpu, req_mem;
  const int64_t* alloc;  // all slots
  const int64_t* req;
};

PreState prefilter(const NumaArgs& a, const gs_pod& pod);
// Filter (plugin.go:275-338); returns gs_numa_reason; *affinity = the store entry the Admit wrote (if any).
// provider2: the hint lists of the second NUMATopologyHintProvider (DeviceShare, after NodeNUMAResource in the
// profile's plugin order, framework_extender.go:138-140), as filterProvidersHints appends them (an empty list = no
// possible affinity; nullptr or no lists = a provider without hints, whose preferred any-numa hint is neutral).
int filter(const NumaArgs& a, const PreState& st, const NodeNUMA& n, const NodeView& v, Hint* affinity,
           bool* has_affinity, bool reverse_resource_order = false,
           const std::vector<std::vector<Hint>>* provider2 = nullptr);
// Score (scoring.go:55-97) with the Filter-time affinity
int64_t score(const NumaArgs& a, const PreState& st, const NodeNUMA& n, const NodeView& v, const Hint& affinity);
int topology_hints_test(const NumaArgs& a, const PreState& st, const NodeNUMA& n, int32_t* res, uint64_t* masks,
                        uint8_t* preferred, uint32_t cap, uint32_t* count);
// Reserve (plugin.go:375-422): Allocate + resourceManager.Update. Returns 0 or a negative error.
int reserve(const NumaArgs& a, const PreState& st, NodeNUMA& n, const gs_pod& pod, const Hint& affinity,
            PodAllocation* out);

// takeCPUs (cpu_accumulator.go:83-247); returns false on error
bool take_cpus(const CPUTopology& topo, int max_ref, const CPUSet& available, const CPUDetails& allocated, int needed,
               int bind_policy, int excl_policy, int strategy, CPUSet* result);

}  // namespace orn
