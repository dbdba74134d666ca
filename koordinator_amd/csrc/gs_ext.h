// gs_ext.h — Reservation + DeviceShare on the device: the HBM image of the nodes' GPU
// devices, the per-pod matched-reservation records the host's BeforePreFilter builds, and the launch interface of
// the kernels of one extension pod (gs_ext.hip):
//   ext_nodes_kernel    every node of the shard: the GPU Fit scalars, DeviceShare Filter + raw Score on the batch-start
//                       score row of the pod (eval pass), the Reservation affinity verdict of unmatched nodes;
//   ext_matched_kernel  the nodes holding reservations the pod matches: the restored NodeInfo re-evaluated (Fit,
//                       LoadAware, NodeNUMAResource), Reservation Filter, NominateReservation and its raw Score;
//   ext select passes   PreScore's preferred node, both DefaultNormalizeScore passes, the weighted totals,
//                       selectHost (max, ties, feasible, the tie-break position) over the whole row: three coalesced
//                       grid passes with global atomics, the last block locating the j*-th tie.
#pragma once
#include <stdint.h>

#include "../../include/gpuscore.h"
#include "gs_kernels.h"

namespace gs {

constexpr int EXT_GPUS = 8;
constexpr int EXT_MAX_RES_PER_NODE = 8;   // matched reservations of one pod on one node (device path)
constexpr int EXT_DEV_STAGE = 1024;       // Device images per staged update (ext_flush_devices)

struct DevGpu {                 // one GPU minor after filterNodeDevice (has_info = 0: not a candidate)
  int64_t total[3];             // gpu-core, gpu-memory-ratio, gpu-memory
  int64_t free[3];              // SubtractWithNonNegativeResult(total, used)
  int32_t minor;
  int16_t has_info;
  int16_t zone;                 // Topology.NodeID as a slot of the node's NUMA zones; GZ_NONE: no topology,
                                // GZ_FOREIGN: a NUMA node that is not one of the node's zones
};
constexpr int16_t GZ_NONE = -1, GZ_FOREIGN = -2;
constexpr int EXT_FIT_NAMES = GS_NUM_GPU_NAMES + GS_MAX_XRES;   // Fit scalars of the extension path: GPU names, then
                                                                  // the registered extended resources
struct DevNode {                // gs_node_devices, as the kernels read it
  int32_t has_device;
  int32_t num_gpus;
  int64_t fit_free[EXT_FIT_NAMES];   // NodeInfo Allocatable - Requested of those names ([upstream] Fit)
  DevGpu g[EXT_GPUS];
};
static_assert(sizeof(DevNode) == 8 + 8 * EXT_FIT_NAMES + EXT_GPUS * 56, "DevNode layout");

struct ExtRes {                 // one matched reservation (ReservationInfo fields the Filter / Score read)
  int64_t alloc[7];             // Allocatable per slot (0 where absent)
  int64_t allocated[7];
  int64_t remained_nn[7];       // SubtractWithNonNegativeResult(Allocatable, Allocated masked to ResourceNames)
  int64_t order;
  uint32_t alloc_mask, allocated_mask, names;
  int32_t policy;
  int32_t skip;                 // allocateOnce with assigned pods (FilterReservation fails)
  int32_t pad;
};
struct ExtRec {                 // a node with matched reservations: the restore deltas against the mirror row
  uint32_t node;
  int32_t nres, first;          // reservations [first, first + nres) of the pod's ExtRes array
  int32_t dpods;                // free_pods delta (reserve pods removed)
  int64_t dfree[7];             // free delta per slot (Requested of the matched view vs the mirror's unmatched view)
  int64_t dnz[2];               // NonZeroRequested delta (free side)
  int64_t pod_requested[7];     // podRequested: Requested after the unmatched trim
  int64_t r_allocated[7];       // Σ matched Allocated
  int64_t order_min;            // findMostPreferredReservationByOrder over the matched (INT64_MAX: none)
  int64_t allocatable[7];       // NodeInfo.Allocatable (fitsNode)
  int64_t restored_pods;        // len(NodeInfo.Pods) after the restore
  int64_t allowed_pods;
};

struct ExtPod {                 // per-pod constants of the three kernels
  int64_t gpu_req[3];           // ConvertDeviceRequest (gpu-core, gpu-memory-ratio, gpu-memory)
  int64_t gpu_name_req[EXT_FIT_NAMES];   // the pod's GPU-name and registered extended-resource requests (Fit scalars)
  int64_t dev_w[3];
  int64_t w_ds, w_rs;
  int64_t pod_req[7];           // PodRequestsAndLimits per slot (Reservation fitsNode / score)
  uint32_t gpu_mask;            // keys of gpu_req (0: no GPU request; DeviceShare skips)
  uint32_t gpu_names;           // keys of gpu_name_req (checked by Fit: the ignored ones left out)
  uint32_t pod_mask;            // keys of pod_req
  int32_t required;             // reservation affinity
  int32_t nrec;
  int32_t ds_on, rs_on;
  int32_t dev_most;
  uint64_t seq;
};

struct ExtOut {
  int32_t node;
  uint32_t feasible;
  int64_t score;
  uint32_t ties;
  int32_t rec;                  // record of the chosen node (-1: none)
  int32_t ds_norm, rs_norm;
  int32_t pref_node;            // PreScore preferred node (-1: none)
  int32_t pad;
  // NodeNUMAResource Reserve of the chosen node (ext_reserve_numa_kernel): the allocation by the Filter-time hint
  uint32_t nflags;              // NumaOut.flags (GS_PLACED_NUMA, affinity bits), PL_RESERVE_FAILED
  uint32_t zkeys;
  int64_t zcpu[4], zmem[4];
  uint32_t aff;                 // 0x10 | zone-slot mask, 0: none (DeviceShare Reserve allocates within it)
  uint32_t err;                 // from ext_numa_kernel: 1 a GPU on a NUMA node outside the zones, 2 a merge past its
                                // permutation bound (the host fails loudly)
};

// (also resets the select accumulators in `scratch`, launch_ext_select's scratch of n1 - n0 nodes)
hipError_t launch_ext_nodes(const DevNode* dev, const int16_t* S, uint32_t n0, uint32_t n1, const ExtPod* pod,
                            int32_t* tot, int16_t* ds, int16_t* rs, int32_t* scratch, hipStream_t st);
hipError_t launch_ext_matched(const MirrorView& m, const PodVec* pods, const Profile& pf, int prod_cols,
                              const DevNode* dev, const ExtPod* pod, const ExtRec* recs, const ExtRes* res, int nrec, int32_t* tot,
                              int16_t* ds, int16_t* rs, int32_t* nominated, uint8_t* aff, uint32_t n0, int32_t* scratch,
                              uint32_t len, hipStream_t st);
// GPU pods on the NUMA-topology-policy nodes (idx, absolute node indices): Filter + Score again with DeviceShare as the
// topology manager's second hint provider, the affinity (aff, the eval pass layout) and DeviceShare Filter / raw Score
// within it; overwrites tot / ds of those nodes (after launch_ext_nodes, before launch_ext_matched, which has the last
// word on the matched nodes; its error word lives in the select scratch, whose accumulators launch_ext_nodes resets).
hipError_t launch_ext_numa(const MirrorView& m, const PodVec* pods, const Profile& pf, int prod_cols, const DevNode* dev,
                           const ExtPod* pod, const uint32_t* idx, uint32_t nidx, uint32_t n0, int32_t* tot, int16_t* ds,
                           uint8_t* aff, int32_t* scratch, uint32_t len, hipStream_t st);
// The pod's end: with numa, the NodeNUMAResource Reserve of the selected node along its Filter-time affinity (aff) ->
// ExtOut.nflags / zkeys / zcpu / zmem / aff; then ExtOut and the nrec nominations written to host_out / host_nom
// (pinned host memory the host reads after the stream synchronizes: no copy).
hipError_t launch_ext_finish(const MirrorView& m, const PodVec* pods, const Profile& pf, int prod_cols,
                             const uint8_t* aff, uint32_t n0, int numa, const ExtOut* out, const int32_t* nom, int nrec,
                             ExtOut* host_out, int32_t* host_nom, hipStream_t st);
size_t ext_select_scratch_words(uint32_t len);   // int32 words of launch_ext_select's scratch
// dev[idx[j]] = img[j], j < n (staged Device image updates)
hipError_t launch_scatter_devnodes(DevNode* dev, const uint32_t* idx, const DevNode* img, uint32_t n, hipStream_t st);
hipError_t launch_ext_select(const int32_t* tot, const int16_t* ds, const int16_t* rs, const ExtRec* recs, uint32_t n0,
                             uint32_t n1, const ExtPod* pod, uint64_t seed, int32_t* scratch, ExtOut* out,
                             hipStream_t st);

}  // namespace gs
