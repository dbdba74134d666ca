// gs_numa_host.h — host half of the NodeNUMAResource path: the per-node NodeAllocation mirror, the
// derived HBM columns the kernels read, and cpuset selection at Reserve (takeCPUs). The device evaluates
// Filter/Score of every (pod, node) pair from count summaries of this state; which CPUs a cpuset pod gets
// only matters at Reserve and is chosen here.
#pragma once
#include <stdint.h>

#include <map>
#include <memory>
#include <unordered_map>
#include <vector>

#include "../../include/gpuscore.h"
#include "gs_cpuset_dev.h"

namespace gs {

struct CpuMask {
  uint64_t w[GS_CPU_WORDS] = {0, 0, 0, 0};
  bool has(int c) const { return (w[c >> 6] >> (c & 63)) & 1; }
  void set(int c) { w[c >> 6] |= 1ull << (c & 63); }
  void clr(int c) { w[c >> 6] &= ~(1ull << (c & 63)); }
  int count() const { return __builtin_popcountll(w[0]) + __builtin_popcountll(w[1]) + __builtin_popcountll(w[2]) + __builtin_popcountll(w[3]); }
  bool empty() const { return !(w[0] | w[1] | w[2] | w[3]); }
};

// A registered CPUTopology (nodenumaresource/cpu_topology.go:25-31) with the derived per-core / per-NUMA /
// per-socket membership the selection code needs.
struct TopoClass {
  int num_cpus = 0, num_cores = 0, num_nodes = 0, num_sockets = 0;
  bool valid = false;
  int cpc = 0, cpn = 0, cps = 0;    // CPUsPerCore / CPUsPerNode / CPUsPerSocket
  int32_t core[GS_MAX_CPUS] = {0};
  uint8_t socket[GS_MAX_CPUS] = {0}, node[GS_MAX_CPUS] = {0};
  TopoDev dev{};                    // bit-plane form for the device-side cpuset Reserve (dev.ok = 0: host only)
};

struct ZoneAlloc {                  // NodeAllocation.allocatedResources[numa node] (node_allocation.go:37)
  uint32_t keys = 0;                // GS_USAGE_CPU / GS_USAGE_MEMORY
  int64_t cpu = 0, mem = 0;
};

struct PodAllocRec {
  uint64_t uid = 0;
  CpuMask cpus;
  int excl = GS_CPU_EXCLUSIVE_NONE;
  std::vector<gs_numa_zone> numa;
};

struct NumaNode {
  gs_node_numa cfg{};
  std::shared_ptr<const TopoClass> topo;   // nullptr: CPUTopology == nil
  std::unordered_map<uint64_t, PodAllocRec> pods;
  uint16_t ref[GS_MAX_CPUS] = {0};         // allocatedCPUs RefCount (0 = absent)
  uint8_t excl[GS_MAX_CPUS] = {0};         // allocatedCPUs ExclusivePolicy
  std::map<int, ZoneAlloc> ares;
  int max_ref() const { return cfg.has_options ? (cfg.max_ref_count ? cfg.max_ref_count : 1) : 0; }
  bool topo_valid() const { return topo && topo->valid; }
};

std::shared_ptr<TopoClass> make_topo(const gs_cpu_topology& t, const char** err);
void numa_add(NumaNode& n, const PodAllocRec& a);      // addPodAllocation (node_allocation.go:82-110)
void numa_release(NumaNode& n, uint64_t uid);          // release (node_allocation.go:112-140)
// Derived columns: i64 = the row's int64 words, i32 = its int32 words (gs_layout.h order). default_most:
// NUMAScoringStrategy MostAllocated (the NUMAAllocateStrategy of nodes that do not set one).
void numa_derive(const NumaNode& n, bool default_most, int64_t* i64, int64_t* i32_widened);
// CpuStateDev of a node (topo = -1 unless its topology has a TopoDev and maxRefCount <= 1)
void numa_cpu_state(const NumaNode& n, bool default_most, CpuStateDev* cs);
// Available CPUs (getAvailableCPUs, node_allocation.go:142-162, preferred = {})
CpuMask numa_available(const NumaNode& n);
// allocateCPUSet (resource_manager.go:273-360) given the NUMA split Allocate produced on the device.
// bind/required from getCPUBindPolicy; strategy resolved. Returns false when the reference would error.
bool numa_allocate_cpuset(const NumaNode& n, int num_cpus, int bind, bool required, int excl, int strategy,
                          const std::vector<gs_numa_zone>& split, CpuMask* out);
// takeCPUs (cpu_accumulator.go:83-247) over arrays
bool take_cpus(const TopoClass& t, int max_ref, const CpuMask& available, const uint16_t* ref, const uint8_t* excl,
               int needed, int bind, int excl_policy, int strategy, CpuMask* out);

}  // namespace gs
