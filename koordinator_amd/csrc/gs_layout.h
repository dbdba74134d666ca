// gs_layout.h — HBM layout of the node mirror and the per-pod vectors, shared by host and device code.
//
// Node mirror: structure-of-arrays, one column per field, each column `npad` elements long (npad is
// a multiple of 1024 so every column starts 8 KiB-aligned and every 2-node slice is a 16-B load).
// Every rank holds the FULL mirror (deltas are replicated); a rank's filter+score kernel reads only
// its shard [shard_begin, shard_end).
#pragma once
#include <stdint.h>

namespace gs {

// int64 columns
enum I64Col : int {
  C_FREE_CPU = 0,      // Allocatable - Requested   (Fit filter, fit.go fitsRequest)
  C_FREE_MEM,
  C_FREE_EPH,
  C_FREE_BCPU,         // scalar slots 3..6 (batch-cpu, batch-memory, mid-cpu, mid-memory)
  C_FREE_BMEM,
  C_FREE_MCPU,
  C_FREE_MMEM,
  C_ALLOC_CPU,         // Allocatable                (Fit LeastAllocated capacity)
  C_ALLOC_MEM,
  C_ALLOC_EPH,
  C_ALLOC_BCPU,
  C_ALLOC_BMEM,
  C_ALLOC_MCPU,
  C_ALLOC_MMEM,
  C_NZFREE_CPU,        // Allocatable - NonZeroRequested (Fit LeastAllocated requested side)
  C_NZFREE_MEM,
  C_LA_CAP_CPU,        // EstimateNode (raw-allocatable override)  (LoadAware score capacity)
  C_LA_CAP_MEM,
  C_LA_FREE_CPU,       // EstimateNode - la_used (non-prod scoring: node usage + assigned estimates)
  C_LA_FREE_MEM,
  C_LA_PFREE_CPU,      // EstimateNode - la_used_prod (ScoreAccordingProdUsage for Prod pods)
  C_LA_PFREE_MEM,
  C_UPDATE_TIME,       // NodeMetric Status.UpdateTime (unix ns)
  // NodeNUMAResource (zone z = gs_node_numa.zones[z], sorted by NUMA node id)
  C_ZCAP_CPU0,         // NUMANodeResources[z] cpu (milli) / memory: the zone's allocatable
  C_ZCAP_MEM0 = C_ZCAP_CPU0 + 4,
  C_ZRAW_CPU0 = C_ZCAP_MEM0 + 4,   // NodeAllocation.allocatedResources[z] (raw sums of pod NUMA allocations)
  C_ZRAW_MEM0 = C_ZRAW_CPU0 + 4,
  C_AMP = C_ZRAW_MEM0 + 4,         // options.AmplificationRatios[cpu] (f64 bits)
  C_NAMP,                          // node annotation cpu amplification ratio (f64 bits; -1 unset)
  // device-side cpuset Reserve state (gs_cpuset_dev.h CpuStateDev; read by the commit kernel only)
  // (the 11 columns C_CPU_UN0 .. C_CPU_XC1 are CpuStateDev's first 11 words, in order)
  C_CPU_UN0,                       // 4 packed plane words: CPUs not available (RefCount >= maxRefCount, or reserved)
  C_CPU_XC = C_CPU_UN0 + 4,        // cores holding a PCPULevel-exclusive allocated CPU (ranks 0..63)
  C_CPU_ZAL,                       // allocated CPUs per zone slot (4 x 16 bits)
  C_CPU_RC0,                       // 4 packed plane words: available CPUs at RefCount 1 (maxRefCount 2)
  C_CPU_XC1 = C_CPU_RC0 + 4,       // C_CPU_XC, ranks 64..127
  NUM_I64_COLS
};

// int32 / uint32 columns
enum I32Col : int {
  C_FREE_PODS = 0,     // AllowedPodNumber - len(Pods)
  C_SFLAGS,            // static LoadAware flags (host-derived, time independent)
  C_DFLAGS,            // dynamic flags (node-prep kernel, depend on `now`)
  C_NFLAGS,            // NodeNUMAResource static flags (NF_*), host-derived
  C_NFLAGS2,           // zone allocation entries / keys (NF2_*), changed by device-side Reserve
  C_ALLOC_CPUS,        // |NodeAllocation.allocatedCPUs| (0 when CPUTopology == nil)
  C_TFREE,             // available CPUs of the node: raw | full-core CPUs << 9 | cores with a free CPU << 18
  C_ZFREE0,            // same, restricted to zone z
  C_ZADJ0 = C_ZFREE0 + 4,          // Amplify(c_z*1000) - c_z*1000, c_z = allocated CPUs in zone z (amp > 1)
  C_CPU_META = C_ZADJ0 + 4,        // CpuStateDev.meta (CM_*)
  C_TOPO_DEV,                      // TopoDev index of the node's topology; -1: cpuset Reserve on the host
  NUM_I32_COLS
};

// C_NFLAGS bits
enum : uint32_t {
  NF_HAS_OPTIONS = 1u << 0,   // TopologyOptions exist
  NF_TOPO = 1u << 1,          // CPUTopology != nil
  NF_TOPO_VALID = 1u << 2,    // CPUTopology.IsValid()
  NF_AMP_INVALID = 1u << 3,   // node amplification annotation unparsable
  NF_POLICY_SHIFT = 4,        // 2 bits: gs_numa_topology_policy
  NF_BIND_SHIFT = 6,          // 2 bits: gs_node_cpu_bind_policy
  NF_ZONES_SHIFT = 8,         // 3 bits: number of zones
  NF_ZCPU_SHIFT = 12,         // 4 bits: zone z lists cpu
  NF_ZMEM_SHIFT = 16,         // 4 bits: zone z lists memory
  NF_CPC_SHIFT = 20,          // 8 bits: CPUsPerCore
};
// C_NFLAGS2 bits
enum : uint32_t {
  NF2_ENTRY_SHIFT = 0,        // 4 bits: allocatedResources has an entry for zone z
  NF2_ACPU_SHIFT = 4,         // 4 bits: that entry lists cpu
  NF2_AMEM_SHIFT = 8,         // 4 bits: that entry lists memory
};

// C_SFLAGS bits
enum : uint32_t {
  SF_METRIC = 1u << 0,        // nodeMetricLister.Get found it
  SF_UPDATE_TIME = 1u << 1,   // Status.UpdateTime != nil
  SF_FAIL_NP = 1u << 2,       // filterNodeUsage -> Unschedulable (load_aware.go:173-224)
  SF_FAIL_P = 1u << 3,        // filterProdUsage -> Unschedulable (load_aware.go:226-254)
  SF_PROD_THR = 1u << 4,      // len(filterProfile.ProdUsageThresholds) > 0
  SF_VALID = 1u << 5,         // row populated
  SF_NP_MEM = 1u << 6,        // SF_FAIL_NP names memory (else cpu)
  SF_NP_AGG = 1u << 7,        // SF_FAIL_NP comes from the aggregated-usage profile
  SF_P_MEM = 1u << 8,         // SF_FAIL_P names memory
};
// C_DFLAGS bits
enum : uint32_t {
  DF_LA_FAIL_NP = 1u << 0,    // LoadAware.Filter fails a non-Prod (or DaemonSet-free) pod
  DF_LA_FAIL_P = 1u << 1,     // LoadAware.Filter fails a Prod pod
  DF_LA_ZERO = 1u << 2,       // LoadAware.Score returns 0 (metric missing / expired)
  DF_NP_DETAIL_SHIFT = 3,     // 2 bits: GS_FAIL_LA_MEMORY / GS_FAIL_LA_AGGREGATED >> 10 of the non-Prod verdict
  DF_P_DETAIL_SHIFT = 5,      // 2 bits: the same for the Prod verdict
};

// per-pod vector (PreFilter output), 128 B
struct PodVec {
  int64_t req[7];        // Fit requests per slot (cpu milli, memory, eph, scalar slots)
  int64_t nz[2];         // non-zero requests cpu/memory (Fit LeastAllocated)
  int64_t est[2];        // DefaultEstimator.EstimatePod cpu/memory (LoadAware)
  uint32_t flags;        // PF_*
  uint32_t scalar_mask;  // scalar request keys (slots 3..6)
  uint32_t numa;         // NodeNUMAResource PreFilter state (PN_*)
  int32_t num_cpus;      // preFilterState.numCPUsNeeded
  uint32_t req_keys;     // request keys (slots 0..6)
  uint32_t pad0;
  uint64_t pad[1];
};
enum : uint32_t {
  PF_DAEMONSET = 1u << 0,
  PF_PROD = 1u << 1,          // GetPodPriorityClassWithDefault == Prod
  PF_PROD_SCORE = 1u << 2,    // Prod && ScoreAccordingProdUsage
  PF_ALL_ZERO = 1u << 3,      // cpu == mem == eph == 0 && no scalar keys (Fit filter short cut)
  PF_LA_W_CPU = 1u << 4,      // (unused on device; args carry the weights)
};
// PodVec.numa: preFilterState (nodenumaresource/plugin.go:172-181)
enum : uint32_t {
  PN_SKIP = 1u << 0,          // requests are zero
  PN_BIND = 1u << 1,          // requestCPUBind
  PN_PREFAIL = 1u << 2,       // PreFilter returned ErrInvalidRequestedCPUs
  PN_REQ_SHIFT = 4,           // 3 bits: requiredCPUBindPolicy (gs_cpu_bind_policy)
  PN_PREF_SHIFT = 8,          // 3 bits: preferredCPUBindPolicy
  PN_EXCL_SHIFT = 12,         // 2 bits: preferredCPUExclusivePolicy (with PN_BIND)
};

// kernel-uniform profile constants
struct Profile {
  uint32_t enabled;           // GS_ENABLE_*
  int32_t w_fit, w_la;        // plugin weights
  int32_t la_w[2];            // LoadAware resource weights (0 = absent)
  int32_t la_wsum;            // Σ LoadAware weights (divisor, load_aware.go:385)
  int32_t fit_w[7];           // Fit LeastAllocated weights per slot
  uint32_t fit_scalar_w_mask; // slots 2..6 with non-zero weight
  int32_t w_numa;             // NodeNUMAResource plugin weight
  int32_t numa_w[7];          // NodeNUMAResource ScoringStrategy.Resources weights per slot
  int32_t numa_most;          // ScoringStrategy.Type == MostAllocated
  int32_t numa_hint_most;     // NUMAScoringStrategy.Type == MostAllocated (hint scores)
};

// per (pod, shard) full-row summary for the exact slow path
struct RowStat {
  int32_t max_score;  // -1 if nothing feasible
  int32_t ties;       // nodes at max_score
  int32_t feasible;
  int32_t pad;
};

}  // namespace gs
