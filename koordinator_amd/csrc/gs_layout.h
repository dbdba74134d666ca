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
  NUM_I64_COLS
};

// int32 / uint32 columns
enum I32Col : int {
  C_FREE_PODS = 0,     // AllowedPodNumber - len(Pods)
  C_SFLAGS,            // static LoadAware flags (host-derived, time independent)
  C_DFLAGS,            // dynamic flags (node-prep kernel, depend on `now`)
  NUM_I32_COLS
};

// C_SFLAGS bits
enum : uint32_t {
  SF_METRIC = 1u << 0,        // nodeMetricLister.Get found it
  SF_UPDATE_TIME = 1u << 1,   // Status.UpdateTime != nil
  SF_FAIL_NP = 1u << 2,       // filterNodeUsage -> Unschedulable (load_aware.go:173-224)
  SF_FAIL_P = 1u << 3,        // filterProdUsage -> Unschedulable (load_aware.go:226-254)
  SF_PROD_THR = 1u << 4,      // len(filterProfile.ProdUsageThresholds) > 0
  SF_VALID = 1u << 5,         // row populated
};
// C_DFLAGS bits
enum : uint32_t {
  DF_LA_FAIL_NP = 1u << 0,    // LoadAware.Filter fails a non-Prod (or DaemonSet-free) pod
  DF_LA_FAIL_P = 1u << 1,     // LoadAware.Filter fails a Prod pod
  DF_LA_ZERO = 1u << 2,       // LoadAware.Score returns 0 (metric missing / expired)
};

// per-pod vector (PreFilter output), 128 B
struct PodVec {
  int64_t req[7];        // Fit requests per slot (cpu milli, memory, eph, scalar slots)
  int64_t nz[2];         // non-zero requests cpu/memory (Fit LeastAllocated)
  int64_t est[2];        // DefaultEstimator.EstimatePod cpu/memory (LoadAware)
  uint32_t flags;        // PF_*
  uint32_t scalar_mask;  // scalar request keys (slots 3..6)
  uint64_t pad[3];
};
enum : uint32_t {
  PF_DAEMONSET = 1u << 0,
  PF_PROD = 1u << 1,          // GetPodPriorityClassWithDefault == Prod
  PF_PROD_SCORE = 1u << 2,    // Prod && ScoreAccordingProdUsage
  PF_ALL_ZERO = 1u << 3,      // cpu == mem == eph == 0 && no scalar keys (Fit filter short cut)
  PF_LA_W_CPU = 1u << 4,      // (unused on device; args carry the weights)
};

// kernel-uniform profile constants
struct Profile {
  uint32_t enabled;           // GS_ENABLE_*
  int32_t w_fit, w_la;        // plugin weights
  int32_t la_w[2];            // LoadAware resource weights (0 = absent)
  int32_t la_wsum;            // Σ LoadAware weights (divisor, load_aware.go:385)
  int32_t fit_w[7];           // Fit LeastAllocated weights per slot
  uint32_t fit_scalar_w_mask; // slots 2..6 with non-zero weight
};

// per (pod, shard) full-row summary for the exact slow path
struct RowStat {
  int32_t max_score;  // -1 if nothing feasible
  int32_t ties;       // nodes at max_score
  int32_t feasible;
  int32_t pad;
};

}  // namespace gs
