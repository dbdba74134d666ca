"""ctypes mirror of include/gpuscore.h (the drop-in C-ABI of libgpuscore).

Struct layouts here must match the header byte for byte; tests/test_abi.py checks the sizes
against the compiled library (gs_abi_sizes) and that every declared symbol is exported.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

GS_ABI_VERSION = 6
GS_NUM_RES = 8
GS_RES_CPU, GS_RES_MEMORY, GS_RES_EPHEMERAL = 0, 1, 2
GS_RES_BATCH_CPU, GS_RES_BATCH_MEMORY, GS_RES_MID_CPU, GS_RES_MID_MEMORY = 3, 4, 5, 6
GS_SCALAR_RES_MASK = 0x78

GS_PRIO_NONE, GS_PRIO_PROD, GS_PRIO_MID, GS_PRIO_BATCH, GS_PRIO_FREE = 0, 1, 2, 3, 4
GS_AGG_NONE, GS_AGG_AVG, GS_AGG_P50, GS_AGG_P90, GS_AGG_P95, GS_AGG_P99 = -1, 0, 1, 2, 3, 4
GS_NUM_AGG_TYPES = 5
GS_MAX_AGG_USAGES = 4
GS_USAGE_CPU, GS_USAGE_MEMORY, GS_USAGE_OTHER = 0x1, 0x2, 0x80
GS_POD_DAEMONSET, GS_POD_TERMINATED = 0x1, 0x2
GS_NODE_CUSTOM_THRESHOLDS, GS_NODE_CUSTOM_AGGREGATED = 0x1, 0x2

GS_PLUGIN_FIT, GS_PLUGIN_LOADAWARE, GS_PLUGIN_NUMA, GS_NUM_PLUGINS = 0, 1, 2, 3
GS_ENABLE_FIT_FILTER, GS_ENABLE_FIT_SCORE = 0x1, 0x2
GS_ENABLE_LA_FILTER, GS_ENABLE_LA_SCORE = 0x4, 0x8
GS_ENABLE_NUMA_FILTER, GS_ENABLE_NUMA_SCORE = 0x10, 0x20
GS_ENABLE_LA_FIT = 0xF
GS_ENABLE_ALL = 0x3F

# NodeNUMAResource vocabulary
GS_MAX_NUMA, GS_MAX_CPUS, GS_CPU_WORDS = 4, 256, 4
GS_QOS_NONE, GS_QOS_LSE, GS_QOS_LSR, GS_QOS_LS, GS_QOS_BE, GS_QOS_SYSTEM = 0, 1, 2, 3, 4, 5
CPU_BIND = {"": 0, "Default": 1, "FullPCPUs": 2, "SpreadByPCPUs": 3, "ConstrainedBurst": 4}
CPU_EXCLUSIVE = {"": 0, "None": 0, "PCPULevel": 1, "NUMANodeLevel": 2}
NODE_CPU_BIND = {"": 0, "None": 0, "FullPCPUsOnly": 1, "SpreadByPCPUs": 2}
NUMA_POLICY = {"": 0, "BestEffort": 1, "Restricted": 2, "SingleNUMANode": 3}
GS_NUMA_POLICY_NONE, GS_NUMA_POLICY_BEST_EFFORT, GS_NUMA_POLICY_RESTRICTED, GS_NUMA_POLICY_SINGLE_NUMA_NODE = 0, 1, 2, 3
NUMA_ALLOC = {"": 0, "MostAllocated": 1, "LeastAllocated": 2, "DistributeEvenly": 3}
GS_SCORING_LEAST_ALLOCATED, GS_SCORING_MOST_ALLOCATED = 0, 1
GS_FAIL_NUMA_SHIFT, GS_FAIL_NUMA_MASK = 6, 0x3C0
GS_FAIL_LA_MEMORY, GS_FAIL_LA_AGGREGATED = 0x400, 0x800
# gs_numa_reason (the NodeNUMAResource reason in bits GS_FAIL_NUMA_MASK)
(GS_NUMA_OK, GS_NUMA_INVALID_REQUESTED_CPUS, GS_NUMA_INVALID_AMP_RATIO, GS_NUMA_AVAILABLE_CPUS_ERROR,
 GS_NUMA_INSUFFICIENT_AMP_CPU, GS_NUMA_INVALID_TOPOLOGY, GS_NUMA_BIND_POLICY_CONFLICT, GS_NUMA_SMT_ALIGNMENT,
 GS_NUMA_ALLOCATE_FAILED, GS_NUMA_MISSING_NUMA_RESOURCES, GS_NUMA_AFFINITY_ERROR, GS_NUMA_ADMIT_ALLOCATE_FAILED) = range(12)


def reason_string(code: int, scalar_mask: int = 0) -> tuple[int, str]:
    """(framework.Code, message) of the reference's Filter status for a gs_evaluate failure code (gs_reason_string)."""
    buf = C.create_string_buffer(512)
    st = load().gs_reason_string(int(code), int(scalar_mask), None, buf, len(buf))
    return st, buf.value.decode()
NUMA_REASONS = ["OK", "InvalidRequestedCPUs", "InvalidAmplificationRatio", "AvailableCPUsError",
                "InsufficientAmplifiedCPU", "InvalidCPUTopology", "CPUBindPolicyConflict", "SMTAlignment",
                "AllocateFailed", "MissingNUMAResources", "NUMATopologyAffinity", "AdmitAllocateFailed"]
GS_PLACED_NUMA, GS_PLACED_CPUSET, GS_PLACED_AFFINITY_SHIFT = 0x2, 0x4, 8

GS_FAIL_FIT_PODS, GS_FAIL_FIT_CPU, GS_FAIL_FIT_MEMORY = 0x01, 0x02, 0x04
GS_FAIL_FIT_EPHEMERAL, GS_FAIL_FIT_SCALAR, GS_FAIL_LOADAWARE = 0x08, 0x10, 0x20
GS_PLACED_SLOWPATH = 0x1

GS_OK, GS_EINVAL, GS_EDEVICE, GS_ENOMEM, GS_EUNSUPPORTED, GS_ECOMM, GS_ESTATE = 0, -1, -2, -3, -4, -5, -6

i64, u64, i32, u32 = C.c_int64, C.c_uint64, C.c_int32, C.c_uint32


class GsPod(C.Structure):
    _fields_ = [
        ("uid", u64), ("name_key", u64),
        ("requests", i64 * GS_NUM_RES), ("limits", i64 * GS_NUM_RES),
        ("nonzero_requests", i64 * 2),
        ("request_mask", u32), ("priority_class", i32), ("flags", u32),
        ("qos_class", i32), ("required_cpu_bind_policy", i32), ("preferred_cpu_bind_policy", i32),
        ("preferred_cpu_exclusive_policy", i32), ("pad0", i32),
    ]


class GsNode(C.Structure):
    _fields_ = [
        ("allocatable", i64 * GS_NUM_RES), ("requested", i64 * GS_NUM_RES),
        ("nonzero_requested", i64 * 2),
        ("allowed_pod_number", i64), ("pod_count", i64),
        ("raw_allocatable", i64 * 2),
        ("raw_allocatable_mask", u32), ("custom_flags", u32),
        ("custom_usage_thresholds", i64 * 2), ("custom_prod_usage_thresholds", i64 * 2),
        ("custom_agg_usage_thresholds", i64 * 2),
        ("custom_usage_mask", u32), ("custom_prod_usage_mask", u32), ("custom_agg_usage_mask", u32),
        ("custom_agg_type", i32), ("custom_agg_duration_ns", i64),
    ]


class GsCpuTopology(C.Structure):
    _fields_ = [("num_cpus", i32), ("pad0", i32), ("core_id", i32 * GS_MAX_CPUS),
                ("socket_id", C.c_uint8 * GS_MAX_CPUS), ("node_id", C.c_uint8 * GS_MAX_CPUS)]


class GsNumaZone(C.Structure):
    _fields_ = [("node_id", i32), ("mask", u32), ("cpu_milli", i64), ("memory", i64)]


class GsNodeNuma(C.Structure):
    _fields_ = [
        ("has_options", i32), ("topology", i32), ("max_ref_count", i32), ("node_cpu_bind_policy", i32),
        ("numa_topology_policy", i32), ("numa_allocate_strategy", i32),
        ("cpu_amplification_ratio", C.c_double), ("node_cpu_amplification_ratio", C.c_double),
        ("node_amplification_invalid", i32), ("num_zones", i32), ("zones", GsNumaZone * GS_MAX_NUMA),
        ("reserved_cpus", u64 * GS_CPU_WORDS),
    ]


class GsPodAllocation(C.Structure):
    _fields_ = [("uid", u64), ("cpuset", u64 * GS_CPU_WORDS), ("cpu_exclusive_policy", i32), ("num_numa", i32),
                ("numa", GsNumaZone * GS_MAX_NUMA)]


class GsNumaArgs(C.Structure):
    _fields_ = [("default_cpu_bind_policy", i32), ("scoring_type", i32), ("numa_scoring_type", i32), ("pad0", i32),
                ("resource_weights", i64 * GS_NUM_RES)]


class GsUsage(C.Structure):
    _fields_ = [("cpu_milli", i64), ("memory", i64), ("mask", u32), ("pad0", u32)]


class GsAggUsage(C.Structure):
    _fields_ = [("duration_ns", i64), ("type_mask", u32), ("pad0", u32), ("usage", GsUsage * GS_NUM_AGG_TYPES)]


class GsNodeMetric(C.Structure):
    _fields_ = [
        ("exists", i32), ("has_update_time", i32), ("update_time_ns", i64),
        ("has_report_interval", i32), ("has_node_metric", i32), ("report_interval_s", i64),
        ("node_usage", GsUsage), ("n_aggregated", i32), ("pad0", u32),
        ("aggregated", GsAggUsage * GS_MAX_AGG_USAGES),
    ]


class GsPodMetric(C.Structure):
    _fields_ = [("name_key", u64), ("in_lister", i32), ("priority_class", i32), ("usage", GsUsage)]


class GsLoadAwareArgs(C.Structure):
    _fields_ = [
        ("filter_expired_node_metrics", i32), ("has_node_metric_expiration", i32),
        ("node_metric_expiration_seconds", i64),
        ("resource_weights", i64 * 2), ("usage_thresholds", i64 * 2),
        ("prod_usage_thresholds", i64 * 2), ("estimated_scaling_factors", i64 * 2),
        ("resource_weights_mask", u32), ("usage_thresholds_mask", u32),
        ("prod_usage_thresholds_mask", u32), ("estimated_scaling_factors_mask", u32),
        ("score_according_prod_usage", i32), ("has_aggregated", i32),
        ("agg_usage_thresholds", i64 * 2), ("agg_usage_thresholds_mask", u32),
        ("agg_usage_type", i32), ("agg_usage_duration_ns", i64),
        ("agg_score_type", i32), ("pad0", i32), ("agg_score_duration_ns", i64),
    ]


class GsFitArgs(C.Structure):
    _fields_ = [("resource_weights", i64 * GS_NUM_RES)]


class GsConfig(C.Structure):
    _fields_ = [
        ("abi_version", u32), ("device", i32), ("num_nodes", u32), ("enabled", u32),
        ("plugin_weights", i64 * GS_NUM_PLUGINS),
        ("loadaware", GsLoadAwareArgs), ("fit", GsFitArgs), ("numa", GsNumaArgs),
        ("seed", u64), ("batch_size", u32), ("cand_cap", u32),
        ("sample_nodes", i32), ("percentage_of_nodes_to_score", i32),
    ]


class GsPlacement(C.Structure):
    _fields_ = [("node", i32), ("feasible", u32), ("score", i64), ("ties", u32), ("flags", u32)]


class GsStats(C.Structure):
    _fields_ = [
        ("batches", u64), ("pods", u64), ("cuts", u64), ("slowpath_pods", u64),
        ("eval_launches", u64), ("eval_pairs", u64),
        ("eval_ms", C.c_double), ("cand_ms", C.c_double), ("commit_ms", C.c_double), ("exchange_ms", C.c_double),
        ("node_row_bytes", u64), ("shard_begin", u32), ("shard_end", u32),
        ("next_start_node_index", u32), ("pad0", u32), ("delta_rows", u64), ("delta_bytes", u64),
    ]


class GsKv(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p)]


GS_QUOTA_DIMS = 8
GS_QUOTA_RUNTIME, GS_QUOTA_CHECK_PARENT, GS_QUOTA_NON_PREEMPTIBLE = 1, 2, 4
GS_QUOTA_ADMIT, GS_QUOTA_INSUFFICIENT, GS_QUOTA_INSUFFICIENT_NON_PREEMPTIBLE = 0, 1, 2


class GsQuotaGroup(C.Structure):
    _fields_ = [("parent", i32), ("allow_lent", u32), ("max_mask", u32), ("min_mask", u32),
                ("max", i64 * GS_QUOTA_DIMS), ("min", i64 * GS_QUOTA_DIMS), ("guaranteed", i64 * GS_QUOTA_DIMS),
                ("shared_weight", i64 * GS_QUOTA_DIMS), ("request", i64 * GS_QUOTA_DIMS),
                ("used", i64 * GS_QUOTA_DIMS), ("non_preemptible_used", i64 * GS_QUOTA_DIMS)]


class GsQuotaStatus(C.Structure):
    _fields_ = [("code", i32), ("group", i32), ("exceed_mask", u32), ("depth", u32),
                ("used", i64 * GS_QUOTA_DIMS)]


# ---- Reservation + DeviceShare ----
GS_NUM_GPU_RES = 3
GS_GPU_CORE, GS_GPU_MEMORY_RATIO, GS_GPU_MEMORY = 0, 1, 2
GS_NUM_GPU_NAMES = 5
GPU_NAMES = {"nvidia.com/gpu": 0, "koordinator.sh/gpu": 1, "koordinator.sh/gpu-core": 2,
             "koordinator.sh/gpu-memory": 3, "koordinator.sh/gpu-memory-ratio": 4}
GS_MAX_GPUS = 8
GS_MAX_XRES = 8   # registered extended resources (any vendor name outside the fixed slots / GPU names)
RSV_POLICY = {"": 0, "Default": 0, "Aligned": 1, "Restricted": 2}
GS_EXT_DEVICESHARE, GS_EXT_RESERVATION = 0x1, 0x2
GS_POD_EVENT_ADD, GS_POD_EVENT_UPDATE, GS_POD_EVENT_DELETE = 0, 1, 2
GS_EXT_FAIL_DEVICE, GS_EXT_FAIL_RESERVATION, GS_EXT_FAIL_POD = 0x1000, 0x2000, 0x4000


class GsGpuDevice(C.Structure):
    _fields_ = [("minor", i32), ("has_info", i32), ("numa_node", i32), ("pad", i32), ("total", i64 * GS_NUM_GPU_RES),
                ("used", i64 * GS_NUM_GPU_RES)]


class GsNodeDevices(C.Structure):
    _fields_ = [("has_device", i32), ("num_gpus", i32), ("gpus", GsGpuDevice * GS_MAX_GPUS),
                ("allocatable", i64 * GS_NUM_GPU_NAMES), ("requested", i64 * GS_NUM_GPU_NAMES),
                ("xres_allocatable", i64 * GS_MAX_XRES), ("xres_requested", i64 * GS_MAX_XRES)]


class GsReservation(C.Structure):
    _fields_ = [("uid", u64), ("owner_key", u64), ("node", u32), ("allocate_policy", i32), ("order", i64),
                ("available", i32), ("unschedulable", i32), ("allocate_once", i32), ("assigned_pods", i32),
                ("allocatable", i64 * GS_NUM_RES), ("allocated", i64 * GS_NUM_RES), ("allocatable_mask", u32),
                ("allocated_mask", u32), ("resource_names_mask", u32), ("pad0", u32)]


class GsPodExt(C.Structure):
    _fields_ = [("reservation_owner", u64), ("reservation_required", i32), ("gpu_request_mask", u32),
                ("gpu_requests", i64 * GS_NUM_GPU_NAMES), ("xres_request_mask", u32), ("pad0", u32),
                ("xres_requests", i64 * GS_MAX_XRES)]


class GsExtArgs(C.Structure):
    _fields_ = [("enabled", u32), ("device_scoring_type", i32), ("device_weights", i64 * GS_NUM_GPU_RES),
                ("weight_deviceshare", i64), ("weight_reservation", i64), ("fit_ignored_gpu_names", u32),
                ("fit_ignored_xres", u32)]


class GsExtPlacement(C.Structure):
    _fields_ = [("reservation_uid", u64), ("gpu_minor_mask", u32), ("gpu_count", i32),
                ("gpu_per_instance", i64 * GS_NUM_GPU_RES), ("deviceshare_score", i32), ("reservation_score", i32),
                ("fail_code", u32), ("pad0", u32)]


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)

# numpy dtypes with the exact C layout (for bulk construction of node/pod arrays)
class GsMergeCase(C.Structure):
    _fields_ = [("lc", u32), ("totc", u32), ("lm", u32), ("totm", u32), ("nz", i32), ("policy", i32),
                ("nil_hints", i32), ("has_cpu", i32), ("has_mem", i32), ("tot_c_any", i32), ("tot_m_any", i32),
                ("score", i32 * 15), ("gpu_hints", u32), ("pad", i32)]


class GsMergeResult(C.Structure):
    _fields_ = [("admit", i32), ("aff_has", i32), ("aff", u32), ("pad", i32)]


class GsGangArgs(C.Structure):
    _fields_ = [("default_timeout_ns", i64), ("skip_check_schedule_cycle", i32), ("pad", i32)]


class GsGangSpec(C.Structure):
    _fields_ = [("gang_id", u64), ("min_member", i32), ("total_children", i32), ("mode", i32), ("match_policy", i32),
                ("wait_time_ns", i64), ("create_time_ns", i64), ("group_n", u32), ("pad", u32), ("group", u64 * 8)]


class GsGangInfo(C.Structure):
    _fields_ = [(n, i32) for n in ("has_init", "min_member", "total_children", "mode", "match_policy", "schedule_cycle",
                                   "schedule_cycle_valid", "once_resource_satisfied", "children", "waiting", "bound",
                                   "pad")] + [("wait_time_ns", i64)]


MERGE_CASE_DTYPE = np.dtype(GsMergeCase)
MERGE_RESULT_DTYPE = np.dtype(GsMergeResult)
POD_DTYPE = np.dtype(GsPod)
NODE_DTYPE = np.dtype(GsNode)
METRIC_DTYPE = np.dtype(GsNodeMetric)
POD_METRIC_DTYPE = np.dtype(GsPodMetric)
PLACEMENT_DTYPE = np.dtype(GsPlacement)
TOPOLOGY_DTYPE = np.dtype(GsCpuTopology)
NODE_NUMA_DTYPE = np.dtype(GsNodeNuma)
POD_ALLOCATION_DTYPE = np.dtype(GsPodAllocation)
NODE_DEVICES_DTYPE = np.dtype(GsNodeDevices)
RESERVATION_DTYPE = np.dtype(GsReservation)
POD_EXT_DTYPE = np.dtype(GsPodExt)
EXT_PLACEMENT_DTYPE = np.dtype(GsExtPlacement)

STRUCT_SIZES = {
    "gs_pod": C.sizeof(GsPod), "gs_node": C.sizeof(GsNode), "gs_node_metric": C.sizeof(GsNodeMetric),
    "gs_pod_metric": C.sizeof(GsPodMetric), "gs_config": C.sizeof(GsConfig),
    "gs_placement": C.sizeof(GsPlacement), "gs_stats": C.sizeof(GsStats),
    "gs_loadaware_args": C.sizeof(GsLoadAwareArgs), "gs_cpu_topology": C.sizeof(GsCpuTopology),
    "gs_node_numa": C.sizeof(GsNodeNuma), "gs_pod_allocation": C.sizeof(GsPodAllocation),
    "gs_numa_args": C.sizeof(GsNumaArgs), "gs_quota_group": C.sizeof(GsQuotaGroup),
    "gs_quota_status": C.sizeof(GsQuotaStatus), "gs_node_devices": C.sizeof(GsNodeDevices),
    "gs_reservation": C.sizeof(GsReservation), "gs_pod_ext": C.sizeof(GsPodExt), "gs_ext_args": C.sizeof(GsExtArgs),
    "gs_ext_placement": C.sizeof(GsExtPlacement),
}

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libgpuscore.so")

# every symbol include/gpuscore.h declares: name -> (restype, argtypes)
P = C.c_void_p
SIGNATURES = {
    "gs_loadaware_args_default": (None, [C.POINTER(GsLoadAwareArgs)]),
    "gs_fit_args_default": (None, [C.POINTER(GsFitArgs)]),
    "gs_loadaware_args_validate": (C.c_int, [C.POINTER(GsLoadAwareArgs), C.c_char_p, C.c_size_t]),
    "gs_create": (C.c_int, [C.POINTER(GsConfig), C.POINTER(P)]),
    "gs_destroy": (C.c_int, [P]),
    "gs_last_error": (C.c_char_p, [P]),
    "gs_version": (C.c_char_p, []),
    "gs_set_now": (C.c_int, [P, i64]),
    "gs_nodes_upsert": (C.c_int, [P, P, P, u32]),
    "gs_node_metrics_upsert": (C.c_int, [P, P, P, u32, P, P]),
    "gs_pods_assign": (C.c_int, [P, P, P, P, u32]),
    "gs_pods_unassign": (C.c_int, [P, P, P, u32]),
    "gs_pods_forget": (C.c_int, [P, P, P, u32]),
    "gs_evaluate": (C.c_int, [P, P, u32, P, P, P]),
    "gs_schedule": (C.c_int, [P, P, u32, P, P]),
    "gs_schedule_submit": (C.c_int, [P, P, u32, P, P, C.POINTER(u64)]),
    "gs_schedule_wait": (C.c_int, [P, u64]),
    "gs_comm_unique_id": (C.c_int, [P]),
    "gs_comm_init_rccl": (C.c_int, [P, P, C.c_int, C.c_int]),
    "gs_comm_init_callback": (C.c_int, [P, C.c_int, C.c_int, ALLGATHER_FN, P]),
    "gs_local_group_create": (C.c_int, [C.c_int, C.POINTER(P)]),
    "gs_local_group_destroy": (C.c_int, [P]),
    "gs_comm_init_local": (C.c_int, [P, P, C.c_int]),
    "gs_get_stats": (C.c_int, [P, C.POINTER(GsStats)]),
    "gs_reset_stats": (C.c_int, [P]),
    "gs_synchronize": (C.c_int, [P]),
    "gs_debug_mirror_check": (C.c_int, [P]),
    "gs_debug_verify_cpuset": (C.c_int, [P, C.c_int]),
    "gs_debug_pair_probe": (C.c_int, [P, P, C.c_uint32, P, P, C.c_uint32, C.c_int, P, P]),
    "gs_debug_numa_merge": (C.c_int, [P, P, u32, P]),
    "gs_gang_args_default": (None, [C.POINTER(GsGangArgs)]),
    "gs_gang_mgr_create": (C.c_int, [C.POINTER(GsGangArgs), C.POINTER(P)]),
    "gs_gang_mgr_destroy": (C.c_int, [P]),
    "gs_gang_mgr_clone": (C.c_int, [P, C.POINTER(P)]),
    "gs_gang_mgr_assign": (C.c_int, [P, P]),
    "gs_gang_podgroup_upsert": (C.c_int, [P, C.POINTER(GsGangSpec)]),
    "gs_gang_podgroup_delete": (C.c_int, [P, u64]),
    "gs_gang_pod_add": (C.c_int, [P, u64, u64, C.c_int, C.POINTER(GsGangSpec)]),
    "gs_gang_pod_delete": (C.c_int, [P, u64, u64]),
    "gs_gang_prefilter": (C.c_int, [P, u64, u64, C.c_int]),
    "gs_gang_permit": (C.c_int, [P, u64, u64, i64, C.POINTER(i64), P, u32, C.POINTER(u32)]),
    "gs_gang_post_bind": (C.c_int, [P, u64, u64]),
    "gs_gang_post_filter": (C.c_int, [P, u64, u64, P, u32, C.POINTER(u32)]),
    "gs_gang_unreserve": (C.c_int, [P, u64, u64, P, u32, C.POINTER(u32)]),
    "gs_gang_expire": (C.c_int, [P, i64, P, u32, C.POINTER(u32)]),
    "gs_gang_get": (C.c_int, [P, u64, C.POINTER(GsGangInfo)]),
    "gs_gang_child_cycle": (C.c_int, [P, u64, u64]),
    "gs_gang_waiting_pods": (C.c_int, [P, P, u32, C.POINTER(u32)]),
    "gs_gang_debug_set": (C.c_int, [P, u64, u64, C.c_int, C.c_int]),
    "gs_gang_pass_create": (C.c_int, [P, u32, P, P, P, i64, P, P, P, P, C.POINTER(P)]),
    "gs_gang_pass_destroy": (C.c_int, [P]),
    "gs_gang_walk": (C.c_int, [P, u32, u32, P, C.POINTER(u32), C.POINTER(u32)]),
    "gs_gang_replay": (C.c_int, [P, u32, u32, P, u32, P, C.POINTER(u32), C.POINTER(u32), C.POINTER(i32)]),
    "gs_gang_pass_after_single": (C.c_int, [P, u32, i32]),
    "gs_gang_pass_forgets": (C.c_int, [P, P, u32, C.POINTER(u32)]),
    "gs_gang_pass_carried": (C.c_int, [P, P, P, u32, C.POINTER(u32)]),
    "gs_reason_string": (C.c_int, [C.c_uint32, C.c_uint32, P, C.c_char_p, C.c_size_t]),
    "gs_reset": (C.c_int, [P]),
    "gs_abi_sizes": (None, [C.POINTER(u64), u32]),
    "gs_topology_register": (C.c_int, [P, C.POINTER(GsCpuTopology), C.POINTER(i32)]),
    "gs_nodes_numa_upsert": (C.c_int, [P, P, P, u32]),
    "gs_numa_allocations_update": (C.c_int, [P, P, P, u32]),
    "gs_numa_allocations_release": (C.c_int, [P, P, P, u32]),
    "gs_numa_allocation_get": (C.c_int, [P, u32, u64, C.POINTER(GsPodAllocation)]),
    "gs_numa_args_default": (None, [C.POINTER(GsNumaArgs)]),
    "gs_num_feasible_nodes_to_find": (u32, [u32, i32]),
    "gs_decode_quantity": (C.c_int, [C.c_char_p, C.POINTER(i64), C.POINTER(i64)]),
    "gs_decode_cpuset": (C.c_int, [C.c_char_p, C.POINTER(u64)]),
    "gs_decode_node_annotations": (C.c_int, [C.POINTER(GsKv), u32, C.POINTER(GsNode), C.POINTER(GsNodeNuma)]),
    "gs_node_reservation_trim": (C.c_int, [C.POINTER(GsKv), u32, C.POINTER(GsNode)]),
    "gs_node_reserved_cpus": (C.c_int, [C.POINTER(GsKv), u32, C.POINTER(u64), C.POINTER(C.c_int32)]),
    "gs_decode_nrt_reserved_cpus": (C.c_int, [C.POINTER(GsKv), u32, C.POINTER(u64)]),
    "gs_decode_node_labels": (C.c_int, [C.POINTER(GsKv), u32, C.c_char_p, C.c_char_p, C.POINTER(GsNodeNuma)]),
    "gs_decode_resource_spec": (C.c_int, [C.c_char_p, C.POINTER(GsPod)]),
    "gs_decode_cpu_topology": (C.c_int, [C.c_char_p, C.POINTER(GsCpuTopology)]),
    "gs_quota_redistribute": (C.c_int, [P, P, P, P, P, u32, i64, P]),
    "gs_quota_refresh_runtime": (C.c_int, [P, u32, P, P, P, P]),
    "gs_quota_prefilter": (C.c_int, [P, u32, P, P, i32, P, u32, u32, C.POINTER(GsQuotaStatus)]),
    "gs_quota_reserve": (C.c_int, [P, u32, i32, P, u32, i32]),
    "gs_quota_admit_batch": (C.c_int, [P, u32, P, P, P, P, P, P, u32, P, C.POINTER(u32)]),
    "gs_quota_settle_batch": (C.c_int, [P, u32, P, P, P, P, P, P, u32, P, P]),
    "gs_pods_on_event": (C.c_int, [P, C.c_int, P, P, u32]),
    "gs_assign_cache_get": (C.c_int, [P, u32, P, P, u32]),
    "gs_ext_args_default": (None, [C.POINTER(GsExtArgs)]),
    "gs_ext_configure": (C.c_int, [P, C.POINTER(GsExtArgs)]),
    "gs_node_devices_upsert": (C.c_int, [P, P, P, u32]),
    "gs_node_devices_get": (C.c_int, [P, u32, C.POINTER(GsNodeDevices)]),
    "gs_reservations_upsert": (C.c_int, [P, P, u32]),
    "gs_reservations_remove": (C.c_int, [P, P, u32]),
    "gs_reservation_get": (C.c_int, [P, u64, C.POINTER(GsReservation)]),
    "gs_schedule_ext": (C.c_int, [P, P, P, u32, P, P, P]),
}


def header_symbols(header_path: str | None = None) -> list[str]:
    """Function names declared in include/gpuscore.h (parsed, not hard-coded)."""
    import re
    if header_path is None:
        header_path = os.path.join(os.path.dirname(PKG_DIR), "include", "gpuscore.h")
    text = open(header_path).read()
    return sorted(set(re.findall(r"^\s*(?:[A-Za-z_][\w\s\*]*?)\b(gs_\w+)\s*\(", text, re.M)))


_LOADED: dict = {}


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load libgpuscore and declare signatures (once per path). Raises if the HIP extension is missing."""
    lib = _LOADED.get(path)
    if lib is not None:
        return lib
    if not os.path.exists(path):
        raise RuntimeError(f"libgpuscore not built: {path} missing (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LOADED[path] = lib
    return lib


def ptr(a) -> int | None:
    """Address of a numpy array's data (None for None)."""
    if a is None:
        return None
    return a.ctypes.data
