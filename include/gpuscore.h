/*
 * gpuscore.h — C-ABI of libgpuscore, the MI355X-native batched Filter/Score engine
 * for koord-scheduler's LoadAwareScheduling / NodeResourcesFit (LeastAllocated) hot path.
 *
 * This header is the drop-in boundary. A cgo package (pkg/scheduler/gpuscore, see
 * INTEGRATION.md) binds exactly these entry points; a ctypes mirror lives in
 * koordinator_amd/abi.py. Only fixed-width POD structs and plain pointers cross the
 * boundary: the caller owns every host buffer, the library owns every device buffer,
 * and no pointer is retained across calls.
 *
 * Each entry point names the reference interface it replaces (paths relative to
 * hormes/koordinator; "[upstream]" = k8s.io/kubernetes@v1.24.15, pinned at go.mod:57,276).
 *
 * Quantity convention (reference: pkg/scheduler/plugins/loadaware/helper.go:146-151
 * getResourceValue): GS_RES_CPU is carried in milli-CPU (Quantity.MilliValue()), every
 * other resource slot in units (Quantity.Value()). Inputs must be integral in that unit.
 *
 * Return convention: 0 = OK, <0 = error (GS_E*); gs_last_error(ctx) has the message.
 */
#ifndef GPUSCORE_H
#define GPUSCORE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 6u

/* ---- resource slots (corev1.ResourceName restricted to the hot-path set) ---- */
enum gs_resource {
  GS_RES_CPU = 0,          /* "cpu"                          (milli) */
  GS_RES_MEMORY = 1,       /* "memory"                       (bytes) */
  GS_RES_EPHEMERAL = 2,    /* "ephemeral-storage"            (bytes) */
  GS_RES_BATCH_CPU = 3,    /* "kubernetes.io/batch-cpu"      (units, apis/extension/resource.go:26) */
  GS_RES_BATCH_MEMORY = 4, /* "kubernetes.io/batch-memory" */
  GS_RES_MID_CPU = 5,      /* "kubernetes.io/mid-cpu" */
  GS_RES_MID_MEMORY = 6,   /* "kubernetes.io/mid-memory" */
  GS_RES_RESERVED = 7,
  GS_NUM_RES = 8
};
/* Scalar (extended) resources in the sense of [upstream] schedutil.IsScalarResourceName. */
#define GS_SCALAR_RES_MASK 0x78u

/* extension.PriorityClass after GetPodPriorityClassWithDefault (apis/extension/priority_utils.go:26-33) */
enum gs_priority_class {
  GS_PRIO_NONE = 0, GS_PRIO_PROD = 1, GS_PRIO_MID = 2, GS_PRIO_BATCH = 3, GS_PRIO_FREE = 4
};

/* extension.AggregationType (apis/extension/... AggregationType: avg,p50,p90,p95,p99) */
enum gs_aggregation_type {
  GS_AGG_NONE = -1, GS_AGG_AVG = 0, GS_AGG_P50 = 1, GS_AGG_P90 = 2, GS_AGG_P95 = 3, GS_AGG_P99 = 4,
  GS_NUM_AGG_TYPES = 5
};
#define GS_MAX_AGG_USAGES 4

/* gs_usage.mask bits: which keys the ResourceList holds */
#define GS_USAGE_CPU 0x1u
#define GS_USAGE_MEMORY 0x2u
#define GS_USAGE_OTHER 0x80u /* some key outside {cpu,memory}: only len(ResourceList) > 0 observes it */

/* ---- NodeNUMAResource vocabulary (apis/extension/numa_aware.go, pkg/scheduler/apis/config/types.go:103-150) ---- */
#define GS_MAX_NUMA 4            /* NUMA nodes (NodeResourceTopology zones) per node on the device path */
#define GS_MAX_CPUS 256          /* logical CPUs per node: CPUDetails ids 0..255 */
#define GS_CPU_WORDS 4           /* uint64 words of a cpuset.CPUSet over GS_MAX_CPUS */

enum gs_qos_class { GS_QOS_NONE = 0, GS_QOS_LSE = 1, GS_QOS_LSR = 2, GS_QOS_LS = 3, GS_QOS_BE = 4, GS_QOS_SYSTEM = 5 };
enum gs_cpu_bind_policy {          /* schedulingconfig.CPUBindPolicy; UNSET = "" */
  GS_CPU_BIND_UNSET = 0, GS_CPU_BIND_DEFAULT = 1, GS_CPU_BIND_FULL_PCPUS = 2, GS_CPU_BIND_SPREAD_BY_PCPUS = 3,
  GS_CPU_BIND_CONSTRAINED_BURST = 4
};
enum gs_cpu_exclusive_policy {     /* schedulingconfig.CPUExclusivePolicy; NONE = "" or "None" */
  GS_CPU_EXCLUSIVE_NONE = 0, GS_CPU_EXCLUSIVE_PCPU_LEVEL = 1, GS_CPU_EXCLUSIVE_NUMA_NODE_LEVEL = 2
};
enum gs_node_cpu_bind_policy {     /* extension.NodeCPUBindPolicy after GetNodeCPUBindPolicy (numa_aware.go:314-325) */
  GS_NODE_CPU_BIND_NONE = 0, GS_NODE_CPU_BIND_FULL_PCPUS_ONLY = 1, GS_NODE_CPU_BIND_SPREAD_BY_PCPUS = 2
};
enum gs_numa_topology_policy {     /* extension.NUMATopologyPolicy; NONE = "" */
  GS_NUMA_POLICY_NONE = 0, GS_NUMA_POLICY_BEST_EFFORT = 1, GS_NUMA_POLICY_RESTRICTED = 2,
  GS_NUMA_POLICY_SINGLE_NUMA_NODE = 3
};
enum gs_numa_allocate_strategy {   /* extension.NUMAAllocateStrategy; UNSET = no node label (args default) */
  GS_NUMA_ALLOC_UNSET = 0, GS_NUMA_ALLOC_MOST_ALLOCATED = 1, GS_NUMA_ALLOC_LEAST_ALLOCATED = 2,
  GS_NUMA_ALLOC_DISTRIBUTE_EVENLY = 3
};
enum gs_scoring_type { GS_SCORING_LEAST_ALLOCATED = 0, GS_SCORING_MOST_ALLOCATED = 1 };

/* ---- pod (decoded by the caller from corev1.Pod) ---- */
#define GS_POD_DAEMONSET 0x1u  /* loadaware/helper.go:189-196 isDaemonSetPod */
#define GS_POD_TERMINATED 0x2u /* pkg/util IsPodTerminated: podAssignCache.assign skips it */

typedef struct gs_pod {
  uint64_t uid;                    /* types.UID (hashed): podAssignCache key */
  uint64_t name_key;               /* hash of "namespace/name": PodMetricInfo match key (helper.go:142-144) */
  int64_t requests[GS_NUM_RES];    /* [upstream] resourceapi.PodRequestsAndLimits requests (== Fit computePodResourceRequest) */
  int64_t limits[GS_NUM_RES];      /* same, limits */
  int64_t nonzero_requests[2];     /* [upstream] Σ_containers schedutil.GetNonzeroRequests (max init, +overhead): cpu milli, memory */
  uint32_t request_mask;           /* bit r: requests holds key r (Fit: len(podRequest.ScalarResources) > 0) */
  int32_t priority_class;          /* gs_priority_class */
  uint32_t flags;                  /* GS_POD_* */
  int32_t qos_class;               /* gs_qos_class: extension.GetPodQoSClassRaw (label koordinator.sh/qosClass) */
  /* annotation scheduling.koordinator.sh/resource-spec (apis/extension/numa_aware.go:190-245), decoded */
  int32_t required_cpu_bind_policy;       /* gs_cpu_bind_policy: ResourceSpec.RequiredCPUBindPolicy */
  int32_t preferred_cpu_bind_policy;      /* ResourceSpec.PreferredCPUBindPolicy */
  int32_t preferred_cpu_exclusive_policy; /* gs_cpu_exclusive_policy: ResourceSpec.PreferredCPUExclusivePolicy */
  int32_t pad0;
} gs_pod;

/* ---- node snapshot row (NodeInfo + node object annotations, decoded by the caller) ---- */
#define GS_NODE_CUSTOM_THRESHOLDS 0x1u  /* annotation scheduling.koordinator.sh/usage-thresholds present and parsed */
#define GS_NODE_CUSTOM_AGGREGATED 0x2u  /* ... and its aggregatedUsage is non-nil */

typedef struct gs_node {
  int64_t allocatable[GS_NUM_RES];   /* NodeInfo.Allocatable (node.Status.Allocatable after transformers) */
  int64_t requested[GS_NUM_RES];     /* NodeInfo.Requested */
  int64_t nonzero_requested[2];      /* NodeInfo.NonZeroRequested cpu milli, memory */
  int64_t allowed_pod_number;        /* NodeInfo.Allocatable.AllowedPodNumber */
  int64_t pod_count;                 /* len(NodeInfo.Pods) */
  int64_t raw_allocatable[2];        /* annotation node.koordinator.sh/raw-allocatable: cpu milli, memory */
  uint32_t raw_allocatable_mask;     /* GS_USAGE_* keys present in raw-allocatable (0: absent or unparsable) */
  uint32_t custom_flags;             /* GS_NODE_CUSTOM_* (apis/extension/load_aware.go:51-62) */
  int64_t custom_usage_thresholds[2];      /* CustomUsageThresholds.UsageThresholds cpu, memory */
  int64_t custom_prod_usage_thresholds[2]; /* .ProdUsageThresholds */
  int64_t custom_agg_usage_thresholds[2];  /* .AggregatedUsage.UsageThresholds */
  uint32_t custom_usage_mask;        /* GS_USAGE_* keys present in each map */
  uint32_t custom_prod_usage_mask;
  uint32_t custom_agg_usage_mask;
  int32_t custom_agg_type;           /* .AggregatedUsage.UsageAggregationType (GS_AGG_NONE = "") */
  int64_t custom_agg_duration_ns;    /* .AggregatedUsage.UsageAggregatedDuration (0 = nil/0) */
} gs_node;

/* ---- NodeNUMAResource topology (TopologyOptions, nodenumaresource/topology_options.go:40-50), decoded ---- */
/* CPUTopology (cpu_topology.go:25-31) as reported in the NRT annotation: one entry per logical CPU. Many nodes
 * share one hardware shape, so topologies are registered once (gs_topology_register) and referenced by id. */
typedef struct gs_cpu_topology {
  int32_t num_cpus;                  /* CPUDetails holds cpu ids 0..num_cpus-1 (<= GS_MAX_CPUS) */
  int32_t pad0;
  int32_t core_id[GS_MAX_CPUS];      /* CPUInfo.CoreID (socket<<16 | core, CPUTopologyBuilder.AddCPUInfo) */
  uint8_t socket_id[GS_MAX_CPUS];    /* CPUInfo.SocketID */
  uint8_t node_id[GS_MAX_CPUS];      /* CPUInfo.NodeID (NUMA node) */
} gs_cpu_topology;

typedef struct gs_numa_zone {        /* NUMANodeResource (topology_options.go:52-55) */
  int32_t node_id;                   /* NUMA node id (< 64, bitmask.BitMask) */
  uint32_t mask;                     /* GS_USAGE_CPU | GS_USAGE_MEMORY: keys present in Resources */
  int64_t cpu_milli;
  int64_t memory;
} gs_numa_zone;

typedef struct gs_node_numa {
  int32_t has_options;               /* TopologyOptionsManager holds options for the node (an NRT was seen) */
  int32_t topology;                  /* gs_topology_register id; -1 = empty CPUTopology (IsValid() false) */
  int32_t max_ref_count;             /* TopologyOptions.MaxRefCount */
  int32_t node_cpu_bind_policy;      /* gs_node_cpu_bind_policy: GetNodeCPUBindPolicy(labels, options.Policy) */
  int32_t numa_topology_policy;      /* gs_numa_topology_policy: getNUMATopologyPolicy (nodenumaresource/util.go:52-58) */
  int32_t numa_allocate_strategy;    /* gs_numa_allocate_strategy: label node.koordinator.sh/numa-allocate-strategy */
  double cpu_amplification_ratio;    /* options.AmplificationRatios[cpu] after amplifyNUMANodeResources (<= 1: none) */
  double node_cpu_amplification_ratio; /* GetNodeResourceAmplificationRatio(node.Annotations, cpu); -1 = unset */
  int32_t node_amplification_invalid;  /* that annotation fails to parse (filterAmplifiedCPUs error) */
  int32_t num_zones;                 /* len(NUMANodeResources) <= GS_MAX_NUMA */
  gs_numa_zone zones[GS_MAX_NUMA];   /* NUMANodeResources after amplifyNUMANodeResources, sorted by node id */
  uint64_t reserved_cpus[GS_CPU_WORDS]; /* TopologyOptions.ReservedCPUs */
} gs_node_numa;

/* PodAllocation (nodenumaresource/node_allocation.go:40-47): what resourceManager.Update records. */
typedef struct gs_pod_allocation {
  uint64_t uid;
  uint64_t cpuset[GS_CPU_WORDS];     /* CPUSet */
  int32_t cpu_exclusive_policy;      /* gs_cpu_exclusive_policy */
  int32_t num_numa;                  /* len(NUMANodeResources) <= GS_MAX_NUMA */
  gs_numa_zone numa[GS_MAX_NUMA];    /* NUMANodeResources (node id + allocated cpu/memory) */
} gs_pod_allocation;

/* ---- NodeMetric (apis/slo/v1alpha1/nodemetric_types.go:38-137), decoded ---- */
typedef struct gs_usage {
  int64_t cpu_milli;
  int64_t memory;
  uint32_t mask; /* GS_USAGE_* */
  uint32_t pad0;
} gs_usage;

typedef struct gs_agg_usage {
  int64_t duration_ns;                 /* AggregatedUsage.Duration */
  uint32_t type_mask;                  /* bit t: Usage[t] present */
  uint32_t pad0;
  gs_usage usage[GS_NUM_AGG_TYPES];
} gs_agg_usage;

typedef struct gs_node_metric {
  int32_t exists;                      /* nodeMetricLister.Get(node) found it */
  int32_t has_update_time;             /* Status.UpdateTime != nil */
  int64_t update_time_ns;              /* unix ns */
  int32_t has_report_interval;         /* Spec.CollectPolicy.ReportIntervalSeconds != nil */
  int32_t has_node_metric;             /* Status.NodeMetric != nil */
  int64_t report_interval_s;
  gs_usage node_usage;                 /* Status.NodeMetric.NodeUsage */
  int32_t n_aggregated;                /* len(AggregatedNodeUsages) <= GS_MAX_AGG_USAGES */
  uint32_t pad0;
  gs_agg_usage aggregated[GS_MAX_AGG_USAGES];
} gs_node_metric;

/* Status.PodsMetric entry, pre-joined with the pod lister (helper.go:153-170) */
typedef struct gs_pod_metric {
  uint64_t name_key;                   /* namespace/name key, same hash as gs_pod.name_key */
  int32_t in_lister;                   /* podLister.Pods(ns).Get(name) succeeded */
  int32_t priority_class;              /* GetPodPriorityClassWithDefault(listed pod) */
  gs_usage usage;                      /* PodUsage */
} gs_pod_metric;

/* ---- plugin args (pkg/scheduler/apis/config/types.go:30-76; v1beta2 defaults in gs_loadaware_args_default) ---- */
typedef struct gs_loadaware_args {
  int32_t filter_expired_node_metrics;         /* FilterExpiredNodeMetrics (*bool; default true) */
  int32_t has_node_metric_expiration;          /* NodeMetricExpirationSeconds != nil */
  int64_t node_metric_expiration_seconds;      /* default 180 */
  int64_t resource_weights[2];                 /* ResourceWeights cpu, memory */
  int64_t usage_thresholds[2];                 /* UsageThresholds */
  int64_t prod_usage_thresholds[2];            /* ProdUsageThresholds */
  int64_t estimated_scaling_factors[2];        /* EstimatedScalingFactors */
  uint32_t resource_weights_mask;              /* GS_USAGE_* keys present in each map */
  uint32_t usage_thresholds_mask;
  uint32_t prod_usage_thresholds_mask;
  uint32_t estimated_scaling_factors_mask;
  int32_t score_according_prod_usage;          /* ScoreAccordingProdUsage */
  int32_t has_aggregated;                      /* Aggregated != nil */
  int64_t agg_usage_thresholds[2];             /* Aggregated.UsageThresholds */
  uint32_t agg_usage_thresholds_mask;
  int32_t agg_usage_type;                      /* Aggregated.UsageAggregationType (GS_AGG_NONE = "") */
  int64_t agg_usage_duration_ns;               /* Aggregated.UsageAggregatedDuration */
  int32_t agg_score_type;                      /* Aggregated.ScoreAggregationType */
  int32_t pad0;
  int64_t agg_score_duration_ns;               /* Aggregated.ScoreAggregatedDuration */
} gs_loadaware_args;

/* [upstream] NodeResourcesFitArgs.ScoringStrategy (LeastAllocated only on this path) */
typedef struct gs_fit_args {
  int64_t resource_weights[GS_NUM_RES];        /* ScoringStrategy.Resources weights per slot (0 = not listed) */
} gs_fit_args;

/* NodeNUMAResourceArgs (pkg/scheduler/apis/config/types.go:103-114; v1beta2 defaults defaults.go:101-136) */
typedef struct gs_numa_args {
  int32_t default_cpu_bind_policy;             /* DefaultCPUBindPolicy (default FullPCPUs) */
  int32_t scoring_type;                        /* ScoringStrategy.Type (gs_scoring_type) */
  int32_t numa_scoring_type;                   /* NUMAScoringStrategy.Type; its Resources are NOT used (scoring.go:37-52) */
  int32_t pad0;
  int64_t resource_weights[GS_NUM_RES];        /* ScoringStrategy.Resources weights per slot (0 = not listed) */
} gs_numa_args;

/* plugin ids / enabled-plugin bits */
enum gs_plugin { GS_PLUGIN_FIT = 0, GS_PLUGIN_LOADAWARE = 1, GS_PLUGIN_NUMA = 2, GS_NUM_PLUGINS = 3 };
#define GS_ENABLE_FIT_FILTER 0x1u
#define GS_ENABLE_FIT_SCORE 0x2u
#define GS_ENABLE_LA_FILTER 0x4u
#define GS_ENABLE_LA_SCORE 0x8u
#define GS_ENABLE_NUMA_FILTER 0x10u
#define GS_ENABLE_NUMA_SCORE 0x20u

typedef struct gs_config {
  uint32_t abi_version;                /* GS_ABI_VERSION */
  int32_t device;                      /* HIP device ordinal */
  uint32_t num_nodes;                  /* node table size (global, all ranks) */
  uint32_t enabled;                    /* GS_ENABLE_* */
  int64_t plugin_weights[GS_NUM_PLUGINS]; /* profile score weights (framework multiplies, runtime/framework.go) */
  gs_loadaware_args loadaware;
  gs_fit_args fit;
  gs_numa_args numa;
  uint64_t seed;                       /* tie-break stream seed (selectHost) */
  uint32_t batch_size;                 /* pods per device pass (0 = default 128) */
  uint32_t cand_cap;                   /* candidate-list capacity per pod and shard (0 = default 256) */
  /* [upstream] findNodesThatPassFilters node sampling (schedule_one.go numFeasibleNodesToFind,
   * KubeSchedulerConfiguration.PercentageOfNodesToScore). sample_nodes = 0: every node is checked (the parity
   * harness's percentageOfNodesToScore = 100; nextStartNodeIndex never moves). sample_nodes = 1: the scheduler
   * keeps nextStartNodeIndex and checks nodes in rotation order from it until numFeasibleNodesToFind(N) feasible
   * nodes are found (parallelism-1 order; percentage_of_nodes_to_score 0 = the adaptive default
   * 50 - N/125 %, at least 5 % and 100 nodes). Several ranks: with the score-row exchange (every rank resolves the
 * window over the all-gathered rows); GS_EUNSUPPORTED at gs_comm_init_* under GS_XCHG=levels. */
  int32_t sample_nodes;
  int32_t percentage_of_nodes_to_score;
} gs_config;

/* ---- outputs ---- */
/* per (pod,node) filter codes (bits; 0 = feasible) */
#define GS_FAIL_FIT_PODS 0x01u      /* "Too many pods" */
#define GS_FAIL_FIT_CPU 0x02u       /* "Insufficient cpu" */
#define GS_FAIL_FIT_MEMORY 0x04u
#define GS_FAIL_FIT_EPHEMERAL 0x08u
#define GS_FAIL_FIT_SCALAR 0x10u
#define GS_FAIL_LOADAWARE 0x20u     /* "node(s) ... usage exceed threshold" (load_aware.go:45-46) */
/* details of a GS_FAIL_LOADAWARE: the resource the reason names is memory (else cpu), and the aggregated-usage
 * form of the reason (ErrReasonAggregatedUsageExceedThreshold); gs_reason_string renders them */
#define GS_FAIL_LA_MEMORY 0x400u
#define GS_FAIL_LA_AGGREGATED 0x800u
/* NodeNUMAResource: the first failing check of the plugin, as a 4-bit reason at GS_FAIL_NUMA_SHIFT */
#define GS_FAIL_NUMA_SHIFT 6
#define GS_FAIL_NUMA_MASK 0x3C0u
enum gs_numa_reason {
  GS_NUMA_OK = 0,
  GS_NUMA_INVALID_REQUESTED_CPUS = 1,   /* ErrInvalidRequestedCPUs (PreFilter or requestCPUBind, util.go:105-122) */
  GS_NUMA_INVALID_AMP_RATIO = 2,        /* ErrInvalidCPUAmplificationRatio (plugin.go:345-347) */
  GS_NUMA_AVAILABLE_CPUS_ERROR = 3,     /* GetAvailableCPUs error in filterAmplifiedCPUs (plugin.go:357-360) */
  GS_NUMA_INSUFFICIENT_AMP_CPU = 4,     /* ErrInsufficientAmplifiedCPU (plugin.go:368-370) */
  GS_NUMA_INVALID_TOPOLOGY = 5,         /* ErrInvalidCPUTopology (plugin.go:301-303) */
  GS_NUMA_BIND_POLICY_CONFLICT = 6,     /* ErrCPUBindPolicyConflict (plugin.go:311-313) */
  GS_NUMA_SMT_ALIGNMENT = 7,            /* ErrSMTAlignmentError (plugin.go:315-319) */
  GS_NUMA_ALLOCATE_FAILED = 8,          /* resourceManager.Allocate error in Filter (plugin.go:321-330) */
  GS_NUMA_MISSING_NUMA_RESOURCES = 9,   /* "node(s) missing NUMA resources" (topology_hint.go:34-36) */
  GS_NUMA_AFFINITY_ERROR = 10,          /* "node(s) NUMA Topology affinity error" (topologymanager/manager.go:67-69) */
  GS_NUMA_ADMIT_ALLOCATE_FAILED = 11    /* provider Allocate error after admit (topology_hint.go:89-95) */
};

typedef struct gs_placement {
  int32_t node;                        /* selected node index, -1 = unschedulable (no feasible node) */
  uint32_t feasible;                   /* number of feasible nodes */
  int64_t score;                       /* total weighted score of the selected node */
  uint32_t ties;                       /* nodes sharing the max score (selectHost reservoir size) */
  uint32_t flags;                      /* GS_PLACED_* diagnostics */
} gs_placement;
#define GS_PLACED_SLOWPATH 0x1u        /* resolved by the exact full-row path (no valid candidate list) */
#define GS_PLACED_NUMA 0x2u            /* NodeNUMAResource Reserve allocated NUMA resources along an affinity hint */
#define GS_PLACED_CPUSET 0x4u          /* NodeNUMAResource Reserve allocated a cpuset (gs_numa_allocation_get) */
#define GS_PLACED_AFFINITY_SHIFT 8     /* bits 8..11: the affinity hint as a mask over gs_node_numa.zones slots */

/* ---- errors ---- */
#define GS_OK 0
#define GS_EINVAL -1
#define GS_EDEVICE -2
#define GS_ENOMEM -3
#define GS_EUNSUPPORTED -4
#define GS_ECOMM -5
#define GS_ESTATE -6

/* ---------------------------------------------------------------------------------------- */

typedef struct gs_ctx gs_ctx; /* one per scheduler profile and GPU (rank) */

/* Multi-GPU exchange: all-gather of `bytes` from every rank, rank-major into recv (host memory).
 * Used when the caller supplies its own transport (tests); production uses native RCCL. */
typedef int (*gs_allgather_fn)(void* user, const void* send, void* recv, size_t bytes);

typedef struct gs_stats {
  uint64_t batches;          /* device passes (eval + candidate + commit) */
  uint64_t pods;             /* pods placed or found unschedulable by gs_schedule */
  uint64_t cuts;             /* batches cut short because a candidate list was exhausted */
  uint64_t slowpath_pods;    /* pods resolved by the exact full-row path */
  uint64_t eval_launches;    /* launches of the fused filter+score kernel */
  uint64_t eval_pairs;       /* pod x node pairs evaluated by it (this rank's shard) */
  double eval_ms;            /* summed device time of the fused filter+score kernel (HIP events) */
  double cand_ms;            /* summed device time of candidate extraction */
  double commit_ms;          /* summed device time of the sequential commit kernel */
  double exchange_ms;        /* all-gather time (multi-GPU): RCCL from stream events around each collective, the host-callback transport as host wall time */
  uint64_t node_row_bytes;   /* bytes one pod x node evaluation reads from the node mirror */
  uint32_t shard_begin, shard_end; /* this rank's node range */
  uint32_t next_start_node_index;  /* [upstream] Scheduler.nextStartNodeIndex after the last scheduled pod */
  uint32_t pad0;
  uint64_t delta_rows;       /* mirror rows re-derived and copied host -> HBM (incremental snapshot updates) */
  uint64_t delta_bytes;      /* their host -> device bytes (row index + staged row) */
} gs_stats;

/* v1beta2.SetDefaults_LoadAwareSchedulingArgs (pkg/scheduler/apis/config/v1beta2/defaults.go:76-99) */
void gs_loadaware_args_default(gs_loadaware_args* a);
/* [upstream] Scheduler.numFeasibleNodesToFind (schedule_one.go, minFeasibleNodesToFind = 100,
 * minFeasibleNodesPercentageToFind = 5) for N nodes and PercentageOfNodesToScore pct. */
uint32_t gs_num_feasible_nodes_to_find(uint32_t num_all_nodes, int32_t pct);
/* v1beta2 NodeResourcesFitArgs default scoring strategy: LeastAllocated cpu=1, memory=1 */
void gs_fit_args_default(gs_fit_args* a);
/* validation.ValidateLoadAwareSchedulingArgs (pkg/scheduler/apis/config/validation/validation_pluginargs.go:31-84) */
int gs_loadaware_args_validate(const gs_loadaware_args* a, char* msg, size_t msg_len);

/* Plugin construction for one profile: loadaware.New (pkg/scheduler/plugins/loadaware/load_aware.go:76-110)
 * and [upstream] noderesources.NewFit, registered through frameworkext.PluginFactoryProxy
 * (pkg/scheduler/frameworkext/framework_extender_factory.go:209-221). Allocates the HBM mirror. */
int gs_create(const gs_config* cfg, gs_ctx** out);
int gs_destroy(gs_ctx* ctx);
const char* gs_last_error(gs_ctx* ctx);
const char* gs_version(void);

/* Injected clock: replaces time.Now in loadaware/helper.go:36-41 (isNodeMetricExpired) and
 * loadaware/pod_assign_cache.go:30-32,65 (assign timestamps). */
int gs_set_now(gs_ctx* ctx, int64_t now_unix_ns);

/* Node snapshot rows: [upstream] internal/cache Cache.UpdateSnapshot -> NodeInfo (Allocatable, Requested,
 * NonZeroRequested, Pods) plus the node annotations read by EstimateNode
 * (loadaware/estimator/default_estimator.go:110-129) and generateUsageThresholdsFilterProfile (loadaware/helper.go:102-140).
 * Only the given rows are recomputed and copied to HBM. */
int gs_nodes_upsert(gs_ctx* ctx, const uint32_t* idx, const gs_node* nodes, uint32_t n);

/* NodeMetric informer events (lister reads at loadaware/load_aware.go:133,278). pod_metrics holds the
 * PodsMetric of metric i at [pm_offsets[i], pm_offsets[i+1]). */
int gs_node_metrics_upsert(gs_ctx* ctx, const uint32_t* idx, const gs_node_metric* metrics, uint32_t n,
                           const gs_pod_metric* pod_metrics, const uint32_t* pm_offsets);

/* podAssignCache.assign / unAssign (loadaware/pod_assign_cache.go:53-80), i.e. LoadAware Reserve/Unreserve
 * (load_aware.go:260-267) and the pod informer handlers (pod_assign_cache.go:82-117). Does not touch NodeInfo. */
int gs_pods_assign(gs_ctx* ctx, const uint32_t* node_idx, const gs_pod* pods, const int64_t* timestamps_ns,
                   uint32_t n);
int gs_pods_unassign(gs_ctx* ctx, const uint32_t* node_idx, const gs_pod* pods, uint32_t n);
/* The scheduler cache's ForgetPod of assumed pods (gs_schedule placed them) once their Reserve is undone: a rejected
 * Permit or a failed binding cycle ([upstream] schedule_one.go: RunReservePluginsUnreserve + Cache.ForgetPod):
 * NodeInfo.RemovePod, LoadAware Unreserve (podAssignCache.unAssign, load_aware.go:265-267) and NodeNUMAResource
 * Unreserve (resourceManager.Release, nodenumaresource/plugin.go:467-476). node_idx[i]: the node pod i was assumed on. */
int gs_pods_forget(gs_ctx* ctx, const uint32_t* node_idx, const gs_pod* pods, uint32_t n);
/* podAssignCache's pod informer handlers OnAdd / OnUpdate / OnDelete (loadaware/pod_assign_cache.go:82-117):
 * node_idx[i] = pod.Spec.NodeName as a node index (-1: "", a pending pod), the GS_POD_TERMINATED flag =
 * util.IsPodTerminated(pod); assign stamps the injected now (timeNowFn). */
#define GS_POD_EVENT_ADD 0
#define GS_POD_EVENT_UPDATE 1
#define GS_POD_EVENT_DELETE 2
int gs_pods_on_event(gs_ctx* ctx, int event, const int32_t* node_idx, const gs_pod* pods, uint32_t n);
/* podAssignCache.podInfoItems[node] in uid order: up to cap (uid, timestamp) entries; returns the entry count. */
int gs_assign_cache_get(gs_ctx* ctx, uint32_t node, uint64_t* uids, int64_t* timestamps, uint32_t cap);

/* Filter + Score of every pod against every node of the current snapshot, no selection, no state change:
 * [upstream] RunFilterPlugins (Fit.Filter fit.go, LoadAware.Filter load_aware.go:123-171) and
 * RunScorePlugins (Fit.Score least_allocated.go, LoadAware.Score load_aware.go:269-335) with profile weights.
 * scores[p*N+n]  = weighted total, or -1 when the node is infeasible (may be NULL)
 * codes[p*N+n]   = GS_FAIL_* bits of every failing filter (may be NULL)
 * plugin_scores[(p*N+n)*GS_NUM_PLUGINS + k] = unweighted score of plugin k, for every node (may be NULL);
 *   NodeNUMAResource's entry is 0 where its own Filter fails (the reference never scores such a node) */
int gs_evaluate(gs_ctx* ctx, const gs_pod* pods, uint32_t npods, int16_t* scores, uint16_t* codes,
                int16_t* plugin_scores);

/* Sequential scheduling of npods pods, in order: for each pod the [upstream] scheduleOne cycle
 * findNodesThatFitPod (percentageOfNodesToScore = 100) -> prioritizeNodes -> selectHost ->
 * assume (NodeInfo.AddPod) -> Reserve (LoadAware podAssignCache.assign, timestamp = now).
 * seq[i] keys pod i's tie-break stream. Multi-GPU: every rank passes the same pods and gets the same out[]. */
int gs_schedule(gs_ctx* ctx, const gs_pod* pods, uint32_t npods, const uint64_t* seq, gs_placement* out);
/* gs_schedule, asynchronously: the pods join the scheduling stream behind every earlier submission (the queue order
 * across submissions is the order of the calls; results are those of one gs_schedule over their concatenation), and
 * the batch pipeline keeps running across submissions — while one submission's last batch commits, the next one's
 * first batch is evaluated and the host applies the finished batch's placements. pods / seq are copied; out must stay
 * valid until gs_schedule_wait(ticket) returns. Every other call on ctx first waits until all submissions are complete
 * (a scheduler submits the next queue chunk, then waits for the previous one). Node sampling included
 * (nextStartNodeIndex carries across submissions). Several ranks: every
 * rank submits the same runs, at its own pace; the ranks agree at each run boundary whether the pipeline continues
 * into the next run. Returns GS_OK and the submission's ticket, or an error (invalid pod, no mirror yet) with nothing
 * submitted. */
int gs_schedule_submit(gs_ctx* ctx, const gs_pod* pods, uint32_t npods, const uint64_t* seq, gs_placement* out,
                       uint64_t* ticket);
/* Blocks until submission `ticket` is complete: its gs_schedule result. An error fails every later submission
 * (GS_ESTATE), leaving the context as a failed gs_schedule would. */
int gs_schedule_wait(gs_ctx* ctx, uint64_t ticket);

/* ---- NodeNUMAResource state ---- */
/* Register a CPUTopology; returns its id in *id (identical topologies may share one id). */
int gs_topology_register(gs_ctx* ctx, const gs_cpu_topology* topo, int32_t* id);
/* NodeResourceTopology informer (nodenumaresource/topology_eventhandler.go) + node labels/annotations read by the
 * plugin: TopologyOptionsManager.UpdateTopologyOptions (topology_options.go:76-86) for the given nodes. */
int gs_nodes_numa_upsert(gs_ctx* ctx, const uint32_t* idx, const gs_node_numa* numa, uint32_t n);
/* resourceManager.Update / Release (resource_manager.go:362-381): pod allocations restored from pods' resource-status
 * annotations (pod_eventhandler.go) or released on delete. Reserve of gs_schedule records its own. */
int gs_numa_allocations_update(gs_ctx* ctx, const uint32_t* node_idx, const gs_pod_allocation* allocs, uint32_t n);
int gs_numa_allocations_release(gs_ctx* ctx, const uint32_t* node_idx, const uint64_t* uids, uint32_t n);
/* The recorded PodAllocation of a pod on a node (PreBind's resource-status, plugin.go:438-478). 1 = found, 0 = none. */
int gs_numa_allocation_get(gs_ctx* ctx, uint32_t node, uint64_t uid, gs_pod_allocation* out);
/* v1beta2.SetDefaults_NodeNUMAResourceArgs (defaults.go:101-136) */
void gs_numa_args_default(gs_numa_args* a);

/* ---- Reservation + DeviceShare ----
 * The two plugins of the shipped profile that normalize their scores (config/manager/scheduler-config.yaml:80-89:
 * DeviceShare weight 1, Reservation weight 5000). Scope on the device path: GPU devices (the GPU device type of
 * deviceshare/utils.go:47-56; no RDMA / FPGA, no joint allocation, no VF or PCIe hints, no device hint selectors);
 * reservations holding cpu / memory / ephemeral / the scalar slots (no cpuset or device reservations, no host
 * ports, no preemption nomination). A pod uses the extension path when it requests GPUs or matches a reservation
 * (or requires one); it is then scheduled alone, through the normalizing select kernel. Every other pod keeps the
 * batched path: for it both plugins score 0 everywhere (DefaultNormalizeScore keeps an all-zero list) and the
 * reservations it does not match enter its NodeInfo through the unmatched restore, which the mirror rows carry. */
enum gs_gpu_res { GS_GPU_CORE = 0, GS_GPU_MEMORY_RATIO = 1, GS_GPU_MEMORY = 2, GS_NUM_GPU_RES = 3 };
/* pod / node resource names of the GPU device type (apis/extension/device_share.go; deviceshare/utils.go:47-56) */
enum gs_gpu_name {
  GS_GPU_NAME_NVIDIA = 0,        /* "nvidia.com/gpu" */
  GS_GPU_NAME_KOORD_GPU = 1,     /* "koordinator.sh/gpu" */
  GS_GPU_NAME_CORE = 2,          /* "koordinator.sh/gpu-core" */
  GS_GPU_NAME_MEMORY = 3,        /* "koordinator.sh/gpu-memory" (bytes) */
  GS_GPU_NAME_MEMORY_RATIO = 4,  /* "koordinator.sh/gpu-memory-ratio" */
  GS_NUM_GPU_NAMES = 5
};
#define GS_MAX_GPUS 8
/* Extended resources outside the 7 fixed slots and the GPU names ([upstream] v1helper.IsExtendedResourceName, any
 * vendor domain): the caller registers up to GS_MAX_XRES names and passes NodeInfo scalars / pod requests by index. A
 * pod requesting one takes the extension path, where Fit's fitsRequest checks it (IgnoredResources /
 * IgnoredResourceGroups through gs_ext_args.fit_ignored_xres). */
#define GS_MAX_XRES 8

typedef struct gs_gpu_device {     /* one GPU minor of the node's Device object (deviceshare/device_cache.go:38-56) */
  int32_t minor;
  int32_t has_info;                /* a DeviceInfo exists for the minor (filterNodeDevice, device_allocator.go:139-163) */
  int32_t numa_node;               /* DeviceInfo.Topology.NodeID (deviceshare/numa_topology.go:46-96); -1: no topology.
                                      On a node with a NUMA topology policy it must be one of the node's NUMA zones */
  int32_t pad;
  int64_t total[GS_NUM_GPU_RES];   /* deviceTotal[gpu][minor] (all zero: an unhealthy device) */
  int64_t used[GS_NUM_GPU_RES];    /* deviceUsed[gpu][minor] */
} gs_gpu_device;

typedef struct gs_node_devices {
  int32_t has_device;              /* nodeDeviceCache.getNodeDevice(node) != nil (else DeviceShare passes / scores 0) */
  int32_t num_gpus;                /* <= GS_MAX_GPUS, distinct minors */
  gs_gpu_device gpus[GS_MAX_GPUS];
  int64_t allocatable[GS_NUM_GPU_NAMES];  /* NodeInfo.Allocatable.ScalarResources of the GPU names ([upstream] Fit) */
  int64_t requested[GS_NUM_GPU_NAMES];    /* NodeInfo.Requested.ScalarResources of the GPU names */
  /* NodeInfo scalars of the caller's other extended resources (any vendor/name outside the 7 fixed slots and the GPU
   * names; index x = the caller's registered name x, 0 when the node does not report it) */
  int64_t xres_allocatable[GS_MAX_XRES];
  int64_t xres_requested[GS_MAX_XRES];
} gs_node_devices;

enum gs_reservation_policy {       /* schedulingv1alpha1.ReservationAllocatePolicy */
  GS_RSV_POLICY_DEFAULT = 0, GS_RSV_POLICY_ALIGNED = 1, GS_RSV_POLICY_RESTRICTED = 2
};
typedef struct gs_reservation {    /* frameworkext.ReservationInfo (frameworkext/reservation_info.go:80-115) */
  uint64_t uid;
  uint64_t owner_key;              /* ReservationInfo.Match(pod) <=> gs_pod_ext.reservation_owner == owner_key
                                      (the caller evaluates the owner matchers; 0 matches no pod) */
  uint32_t node;                   /* Status.NodeName as a node index */
  int32_t allocate_policy;         /* gs_reservation_policy */
  int64_t order;                   /* label scheduling.koordinator.sh/reservation-order parsed (0: absent or invalid) */
  int32_t available;               /* IsAvailable() && ParseError == nil */
  int32_t unschedulable;           /* IsUnschedulable() */
  int32_t allocate_once;           /* IsAllocateOnce() */
  int32_t assigned_pods;           /* len(AssignedPods) */
  int64_t allocatable[GS_NUM_RES]; /* Allocatable = the reserve pod's requests (ReservationRequests) */
  int64_t allocated[GS_NUM_RES];   /* Allocated */
  uint32_t allocatable_mask;       /* keys of Allocatable */
  uint32_t allocated_mask;         /* keys of Allocated */
  uint32_t resource_names_mask;    /* ResourceNames (restricted options applied) */
  uint32_t pad0;
} gs_reservation;

typedef struct gs_pod_ext {        /* per-pod inputs of the two plugins' PreFilter */
  uint64_t reservation_owner;      /* owner key the pod presents to ReservationInfo.Match (0: none) */
  int32_t reservation_required;    /* reservationutil.GetRequiredReservationAffinity(pod) != nil (hasAffinity) */
  uint32_t gpu_request_mask;       /* bit n: PodRequestsAndLimits holds GPU name n with a non-zero value */
  int64_t gpu_requests[GS_NUM_GPU_NAMES];
  uint32_t xres_request_mask;      /* bit x: the pod requests registered extended resource x (a key of its requests) */
  uint32_t pad0;
  int64_t xres_requests[GS_MAX_XRES];   /* [upstream] Fit fitsRequest checks them like any scalar resource */
} gs_pod_ext;

#define GS_EXT_DEVICESHARE 0x1u    /* DeviceShare Filter + Score + Reserve */
#define GS_EXT_RESERVATION 0x2u    /* Reservation BeforePreFilter restore + Filter + PreScore + Score + Reserve */
typedef struct gs_ext_args {
  uint32_t enabled;                /* GS_EXT_* */
  int32_t device_scoring_type;     /* DeviceShareArgs.ScoringStrategy.Type (gs_scoring_type) */
  int64_t device_weights[GS_NUM_GPU_RES]; /* ScoringStrategy.Resources over gpu-core, gpu-memory-ratio, gpu-memory
                                             (v1beta2 default: gpu-memory-ratio = 1, defaults.go:187-203) */
  int64_t weight_deviceshare;      /* profile score weights */
  int64_t weight_reservation;
  uint32_t fit_ignored_gpu_names;  /* [upstream] NodeResourcesFitArgs.IgnoredResources / IgnoredResourceGroups on the GPU
                                      names (extended resources): bit n = name n is ignored, or its domain (the text
                                      before '/') is an ignored group; Fit then skips its scalar check */
  uint32_t fit_ignored_xres;       /* the same for the registered extended resources (bit x). Their Fit Score weight
                                      is 0 (ScoringStrategy.Resources lists only slot resources): a profile weighing
                                      one is outside this ABI */
} gs_ext_args;

#define GS_EXT_FAIL_DEVICE 0x1000u      /* DeviceShare Filter: "Insufficient gpu devices" and the Prepare errors */
#define GS_EXT_FAIL_RESERVATION 0x2000u /* Reservation Filter (reservation affinity: no satisfying reservation) */
#define GS_EXT_FAIL_POD 0x4000u         /* the pod fails a PreFilter (invalid device request) on every node */

typedef struct gs_ext_placement {
  uint64_t reservation_uid;        /* the nominated reservation the pod was assumed into (0: none) */
  uint32_t gpu_minor_mask;         /* GPU minors the DeviceShare Reserve allocated (bit = minor) */
  int32_t gpu_count;
  int64_t gpu_per_instance[GS_NUM_GPU_RES]; /* the DeviceAllocation.Resources of each minor */
  int32_t deviceshare_score;       /* normalized plugin scores of the selected node (before weighting) */
  int32_t reservation_score;
  uint32_t fail_code;              /* a pod failing PreFilter: GS_EXT_FAIL_POD */
  uint32_t pad0;
} gs_ext_placement;

/* v1beta2.SetDefaults_DeviceShareArgs (defaults.go:187-203) + the shipped profile weights */
void gs_ext_args_default(gs_ext_args* a);
int gs_ext_configure(gs_ctx* ctx, const gs_ext_args* args);
/* Device informer (deviceshare/eventhandler_device.go): the node's GPU Device object + NodeInfo scalars. */
int gs_node_devices_upsert(gs_ctx* ctx, const uint32_t* idx, const gs_node_devices* dev, uint32_t n);
int gs_node_devices_get(gs_ctx* ctx, uint32_t node, gs_node_devices* out);
/* Reservation informer (reservation/eventhandler.go, cache.go): add / update by uid, delete by uid. NodeInfo
 * (gs_nodes_upsert) is the caller's snapshot and already holds the reserve pods. */
int gs_reservations_upsert(gs_ctx* ctx, const gs_reservation* r, uint32_t n);
int gs_reservations_remove(gs_ctx* ctx, const uint64_t* uids, uint32_t n);
int gs_reservation_get(gs_ctx* ctx, uint64_t uid, gs_reservation* out);   /* 1 = found, 0 = none */
/* gs_schedule with the Reservation / DeviceShare plugins: ext[i] (ext may be NULL: no pod uses them) holds pod i's
 * plugin inputs; ext_out[i] (may be NULL) receives the reservation and GPU minors the Reserve assumed. Pods on the
 * extension path need no node sampling, and one rank or several over the score-row exchange (each extension pod then
 * runs whole on every rank; GS_EUNSUPPORTED under GS_XCHG=levels). */
int gs_schedule_ext(gs_ctx* ctx, const gs_pod* pods, const gs_pod_ext* ext, uint32_t npods, const uint64_t* seq,
                    gs_placement* out, gs_ext_placement* ext_out);

/* Multi-GPU: nodes are sharded in contiguous ranges [r*ceil(N/R), (r+1)*ceil(N/R)); every rank keeps the full
 * mirror (replicated deltas) and evaluates only its shard. Per batch the shards' score rows are all-gathered and every
 * rank runs the one-GPU selection and Reserve over all nodes (GS_XCHG=levels at init: the per-shard candidate levels
 * instead, merged on the device). Native RCCL over xGMI: */
int gs_comm_unique_id(uint8_t out[128]);
int gs_comm_init_rccl(gs_ctx* ctx, const uint8_t id[128], int nranks, int rank);
/* Caller-supplied transport (host buffers): */
int gs_comm_init_callback(gs_ctx* ctx, int nranks, int rank, gs_allgather_fn fn, void* user);
/* In-process device transport (the ranks are threads of one process, e.g. several contexts on one GPU in tests): the
 * all-gather is stream-ordered like ncclAllGather — device-to-device copies ordered by events on each rank's stream, no
 * host wait on the GPU (the threads meet twice per exchange on the host to trade buffers and events). One group per
 * set of ranks, created before and destroyed after their contexts. */
typedef struct gs_local_group gs_local_group;
int gs_local_group_create(int nranks, gs_local_group** out);
int gs_local_group_destroy(gs_local_group* g);
int gs_comm_init_local(gs_ctx* ctx, gs_local_group* g, int rank);

/* ---- ingest decoders: the annotation / label text the plugins parse per call in the
 * reference, decoded once on the host into the ABI structs above (pure host functions, no device call) ---- */
typedef struct gs_kv { const char* key; const char* value; } gs_kv;   /* one map[string]string entry */

/* [upstream] k8s.io/apimachinery@v0.24.15 resource.ParseQuantity -> Quantity.Value() and MilliValue() (both
 * round up). GS_EINVAL: malformed; GS_EUNSUPPORTED: outside int64. */
int gs_decode_quantity(const char* s, int64_t* value, int64_t* milli_value);
/* cpuset.Parse (pkg/util/cpuset/cpuset.go:322-366): Linux CPU list -> bit words (CPU ids < GS_MAX_CPUS). */
int gs_decode_cpuset(const char* s, uint64_t out[GS_CPU_WORDS]);
/* Node annotations: node.koordinator.sh/raw-allocatable (GetNodeRawAllocatable,
 * apis/extension/node_resource_amplification.go:113-125, as EstimateNode reads it: a malformed one is ignored,
 * loadaware/estimator/default_estimator.go:110-129), scheduling.koordinator.sh/usage-thresholds
 * (GetCustomUsageThresholds, apis/extension/load_aware.go:51-62; malformed = the args' thresholds,
 * loadaware/helper.go:102-140), node.koordinator.sh/resource-amplification-ratio
 * (GetNodeResourceAmplificationRatio, node_resource_amplification.go:61-73; malformed = the
 * ErrInvalidCPUAmplificationRatio path, nodenumaresource/plugin.go:345-347). Fills the raw_allocatable* and
 * custom_* fields of *node and (numa != NULL) the node amplification fields of *numa. */
int gs_decode_node_annotations(const gs_kv* annotations, uint32_t n, gs_node* node, gs_node_numa* numa);
/* Node reservation, annotation node.koordinator.sh/reservation (NodeReservation, apis/extension/node_reservation.go
 * :37-68): the scheduler's node transformer TransformNodeWithNodeReservation (pkg/util/transformer/node_transformer.go
 * :66-68) = TrimNodeAllocatableByNodeReservation (pkg/util/node.go:121-151) applied in place to node->allocatable and
 * allowed_pod_number (the caller fills them with node.Status.Allocatable first): with applyPolicy "" or "Default" the
 * reserved resources (GetNodeReservationResources, node.go:102-119: cpu = |reservedCPUs| when that is set) are
 * subtracted, floored at 0 (quotav1.SubtractWithNonNegativeResult), batch-cpu / batch-memory kept. Returns 1 when the
 * allocatable changed, 0 when not (absent or undecodable annotation, ReservedCPUsOnly, nothing reserved, an
 * unparsable reservedCPUs: the reference leaves Allocatable as it is), GS_EUNSUPPORTED for a negative quantity. */
int gs_node_reservation_trim(const gs_kv* annotations, uint32_t n, gs_node* node);
/* GetReservedCPUs (node_reservation.go:70-90): the reservation's reservedCPUs as bit words and numReservedCPUs
 * (ceil of a positive reserved cpu quantity, 0 when reservedCPUs is set). 1: reservedCPUs is set but unparsable. */
int gs_node_reserved_cpus(const gs_kv* annotations, uint32_t n, uint64_t cpus[GS_CPU_WORDS], int32_t* num_reserved_cpus);
/* TopologyOptions.ReservedCPUs (nodenumaresource/topology_options.go:90-146) from the NRT annotations: kubelet-managed
 * pods' cpusets (node.koordinator.sh/pod-cpu-allocs) | kubelet reservedCPUs (kubelet.koordinator.sh/cpu-manager-policy)
 * | the node reservation's reservedCPUs | an exclusive system-QoS cpuset (node.koordinator.sh/system-qos-resource); a
 * part that does not decode adds nothing (the reference logs it). -> gs_node_numa.reserved_cpus. */
int gs_decode_nrt_reserved_cpus(const gs_kv* nrt_annotations, uint32_t n, uint64_t out[GS_CPU_WORDS]);
/* Node labels + the NRT's kubelet CPU manager policy JSON and topology-manager policy (either may be NULL):
 * GetNodeCPUBindPolicy (apis/extension/numa_aware.go:301-325), getNUMATopologyPolicy
 * (nodenumaresource/util.go:52-58), GetNUMAAllocateStrategy (util.go:35-41) -> *numa. */
int gs_decode_node_labels(const gs_kv* labels, uint32_t n, const char* kubelet_cpu_manager_policy,
                          const char* kubelet_topology_policy, gs_node_numa* numa);
/* Pod annotation scheduling.koordinator.sh/resource-spec (GetResourceSpec, numa_aware.go:191-202); NULL =
 * absent. Fills the bind / exclusive policy fields of *pod. */
int gs_decode_resource_spec(const char* json, gs_pod* pod);
/* NRT annotation node.koordinator.sh/cpu-topology (GetCPUTopology, numa_aware.go:249-260) -> gs_cpu_topology
 * (CoreID = socket<<16 | core, nodenumaresource/cpu_topology.go:45); NULL = an empty topology. */
int gs_decode_cpu_topology(const char* json, gs_cpu_topology* out);

/* ---- ElasticQuota admission: the per-pod quota gate in front of the node loop. A host
 * function over the quota forest, not a device kernel: it reads O(depth) groups per pod, nothing per node.
 * Quantities per resource dimension d < GS_QUOTA_DIMS in getQuantityValue units
 * (elasticquota/core/runtime_quota_calculator.go:500-505: cpu in milli, everything else Value()); the caller
 * fixes the dimension -> resource-name map. A *_mask bit d says resource d is a key of that ResourceList. ---- */
#define GS_QUOTA_DIMS 8
typedef struct gs_quota_group {
  int32_t parent;            /* index of the parent group; -1 = a child of the root quota (ParentName == root) */
  uint32_t allow_lent;       /* QuotaInfo.AllowLentResource */
  uint32_t max_mask;         /* keys of CalculateInfo.Max */
  uint32_t min_mask;         /* keys of CalculateInfo.Min (= AutoScaleMin: scale-min-quota is not restated) */
  int64_t max[GS_QUOTA_DIMS];
  int64_t min[GS_QUOTA_DIMS];
  int64_t guaranteed[GS_QUOTA_DIMS];     /* CalculateInfo.Guaranteed (0 unless ElasticQuotaGuaranteeUsage) */
  int64_t shared_weight[GS_QUOTA_DIMS];  /* CalculateInfo.SharedWeight (defaults to Max, quota_info.go) */
  int64_t request[GS_QUOTA_DIMS];        /* sum of the requests of the pods charged to this quota itself */
  int64_t used[GS_QUOTA_DIMS];           /* CalculateInfo.Used (this quota and, for a parent, its subtree) */
  int64_t non_preemptible_used[GS_QUOTA_DIMS];
} gs_quota_group;

/* quotaTree.redistribution + iterationForRedistribution (runtime_quota_calculator.go:106-166): one resource
 * dimension of one parent's children. request = the children's limited requests. runtime[i] out. */
int gs_quota_redistribute(const int64_t* request, const int64_t* min, const int64_t* guaranteed,
                          const int64_t* shared_weight, const uint8_t* allow_lent, uint32_t n, int64_t total,
                          int64_t* runtime);
/* GroupQuotaManager.refreshRuntimeNoLock (group_quota_manager.go:264-321) for every group at once, from a settled
 * request tree: Request = ChildRequest (own + the children's limited requests), floored at Min when lending is
 * off (recursiveUpdateGroupTreeWithDeltaRequest, :184-224); limited request = min(Request, Max) on Max's keys
 * (quota_info.go:201-212); each parent's children share the parent's runtime (root: total = cluster total
 * except system/default used) per dimension of the union of all Max keys (updateResourceKeyNoLock, :558-576).
 * runtime and limit_request (either may be NULL) are n x GS_QUOTA_DIMS; runtime_mask (n entries, may be NULL)
 * = the keys of each group's Runtime (that union).
 * GS_EINVAL on a parent index out of range or a cycle. */
int gs_quota_refresh_runtime(const gs_quota_group* groups, uint32_t n, const int64_t total[GS_QUOTA_DIMS],
                             int64_t* runtime, int64_t* limit_request, uint32_t* runtime_mask);

#define GS_QUOTA_RUNTIME 1u          /* ElasticQuotaArgs.EnableRuntimeQuota: the limit is Runtime, else Max */
#define GS_QUOTA_CHECK_PARENT 2u     /* ElasticQuotaArgs.EnableCheckParentQuota */
#define GS_QUOTA_NON_PREEMPTIBLE 4u  /* extension.IsPodNonPreemptible(pod) */
#define GS_QUOTA_ADMIT 0
#define GS_QUOTA_INSUFFICIENT 1                 /* "Insufficient quotas, ..." (Unschedulable) */
#define GS_QUOTA_INSUFFICIENT_NON_PREEMPTIBLE 2 /* "Insufficient non-preemptible quotas, ..." (Unschedulable) */
typedef struct gs_quota_status {
  int32_t code;        /* GS_QUOTA_ADMIT / _INSUFFICIENT / _INSUFFICIENT_NON_PREEMPTIBLE */
  int32_t group;       /* the group whose check failed (a parent when the recursive check failed), else -1 */
  uint32_t exceed_mask;/* exceedDimensions */
  uint32_t depth;      /* parent hops above the pod's quota for a recursive failure (quotaNameTopo length - 1) */
  int64_t used[GS_QUOTA_DIMS];   /* the failing group's used (non-preemptible used for _NON_PREEMPTIBLE) as checked */
} gs_quota_status;
/* Plugin.PreFilter (elasticquota/plugin.go:210-254) + checkQuotaRecursive (plugin_helper.go:281-297) for one
 * pod of quota `quota` (-1: no quota label -> admit). runtime: n x GS_QUOTA_DIMS, group i's keys runtime_mask[i]
 * (from gs_quota_refresh_runtime, or the caller's). pod_request: PodRequestsAndLimits, keys pod_request_mask. */
int gs_quota_prefilter(const gs_quota_group* groups, uint32_t n, const int64_t* runtime, const uint32_t* runtime_mask,
                       int32_t quota, const int64_t pod_request[GS_QUOTA_DIMS], uint32_t pod_request_mask,
                       uint32_t flags, gs_quota_status* out);

/* GroupQuotaManager.ReservePod / UnreservePod (group_quota_manager.go:791-805): request joins (sign = +1) or
 * leaves (-1) used — and, with GS_QUOTA_NON_PREEMPTIBLE in flags, non-preemptible used — of `quota` and every
 * ancestor. */
int gs_quota_reserve(gs_quota_group* groups, uint32_t n, int32_t quota, const int64_t request[GS_QUOTA_DIMS],
                     uint32_t flags, int32_t sign);
/* Quota-gated batch admission: gs_quota_prefilter per pod in order (pod j: quota[j], requests[j*GS_QUOTA_DIMS..],
 * request_mask[j], flags[j]); each admitted pod is reserved speculatively; a rejected pod is final when it is
 * also rejected against the certain used (its chain's used minus this call's speculative Reserves), otherwise the
 * call stops before it (admission is monotone in used, so admitted verdicts stand). Follow each run with
 * gs_quota_settle_batch.
 * status[0..*consumed) = the decided pods' verdicts. */
int gs_quota_admit_batch(gs_quota_group* groups, uint32_t n, const int64_t* runtime, const uint32_t* runtime_mask,
                         const int32_t* quota, const int64_t* requests, const uint32_t* request_mask,
                         const uint32_t* flags, uint32_t count, gs_quota_status* status, uint32_t* consumed);

/* Settles a run of gs_quota_admit_batch after the node loop: withdraws its speculative Reserves and replays it
 * in order with the engine's placements (placed_node[j] >= 0: Reserve), recomputing every status against the
 * used the one-pod-at-a-time order would have seen. GS_ESTATE if a verdict would change (monotonicity bug). */
int gs_quota_settle_batch(gs_quota_group* groups, uint32_t n, const int64_t* runtime, const uint32_t* runtime_mask,
                          const int32_t* quota, const int64_t* requests, const uint32_t* request_mask,
                          const uint32_t* flags, uint32_t count, const int32_t* placed_node, gs_quota_status* status);

/* Recovery after a failed call (any return < 0 from gs_schedule / gs_evaluate / an upsert): the host state is the
 * truth — placements of the failed gs_schedule call past the last completed batch were not assumed (gs_stats.pods
 * counts the pods that were) — and the HBM mirror may hold a partial batch. gs_reset drains the device queues and
 * rebuilds every mirror row from the host state (the reference's informer snapshot). GS_EDEVICE: the device is
 * unusable; destroy the context and create a new one. */
int gs_reset(gs_ctx* ctx);

int gs_get_stats(gs_ctx* ctx, gs_stats* out);
int gs_reset_stats(gs_ctx* ctx);
/* Blocks until all device work of ctx has completed. */
int gs_synchronize(gs_ctx* ctx);

/* Diagnostics: re-derives every node row on the host and compares it with the HBM mirror; returns the
 * number of mismatching rows (0 = the device-side Assume/Reserve replay matches the host mirror). */
int gs_debug_mirror_check(gs_ctx* ctx);
/* Diagnostics: on != 0 makes gs_schedule re-run the host takeCPUs (cpu_accumulator.go:87-232) for every cpuset
 * the commit kernel selected and fail with GS_ESTATE on any difference. */
int gs_debug_verify_cpuset(gs_ctx* ctx, int on);
/* The reference's Filter status for a GS_FAIL_* code of gs_evaluate (codes[]): the first failing plugin in the
 * profile's Filter order (NodeResourcesFit, LoadAwareScheduling, NodeNUMAResource), its message as
 * framework.Status.Message() prints it (the Fit reasons joined by ", ", [upstream] fit.go; load_aware.go:45-46 with
 * the resource; nodenumaresource/plugin.go:48-55, topology_hint.go:36, topologymanager/manager.go:70,
 * resource_manager.go:292 for the reasons the device reports) written to buf (NUL-terminated, truncated to len).
 * scalar_names: the names of resource slots 3..6 for "Insufficient <name>" (NULL: the kubernetes.io/batch-cpu,
 * batch-memory, mid-cpu, mid-memory defaults). Returns the framework.Code: 0 Success (code 0), 1 Unschedulable,
 * 2 UnschedulableAndUnresolvable; GS_EINVAL for a malformed code.
 * Scalar resources: the code does not say which requested scalar was short, so every slot of scalar_mask is
 * named (pass the pod's gs_pod.scalar_mask; 0 names none). GS_NUMA_ADMIT_ALLOCATE_FAILED renders the allocator's
 * cpuset-count error; when the reference's Allocate fails earlier, on the hint's NUMA amounts, it prints
 * "Insufficient NUMA <resource>" instead (the device code does not carry which; parity unpinned). */
int gs_reason_string(uint32_t code, uint32_t scalar_mask, const char* const* scalar_names, char* buf, size_t len);

/* Diagnostics: s_memtime cycles of the commit kernel's per-pair evaluation on mirror rows. Probe i evaluates
 * node nodes[i]: mode 0 with pod pod_of[i] on a whole wave (the selector's re-score), mode 2 likewise with the
 * lane-parallel evaluation, mode 1 with pods 0..npods-1 (npods <= 64) one per lane over the row's hint table (the
 * re-scoring waves). scores: n (modes 0, 2) or n*64 (mode 1) total scores (-1 infeasible); cycles: 2n, the
 * warm-instruction-cache evaluation of probe i at [i], the cold first one at [n + i]; mode 2 also leaves the
 * s_memtime stamps of its 8 phases at [2n + 8i ..] (cycles: 10n entries). */
int gs_debug_pair_probe(gs_ctx* ctx, const gs_pod* pods, uint32_t npods, const uint32_t* nodes, const int32_t* pod_of,
                        uint32_t n, int mode, int32_t* scores, uint64_t* cycles);
/* Diagnostics: the device's topology-manager Merge + admit (frameworkext/topologymanager/policy.go:68-186 and
 * policy_{best_effort,restricted,single_numa_node}.go, as every NUMA-policy pair evaluation runs it) on given hint
 * lists, one gs_merge_case each. The lists are those NodeNUMAResource's hint provider produces
 * (resource_manager.go:418-532 generateHints), in filterProvidersHints' resource order cpu, memory: positions of the
 * IterateBitMasks order over nz NUMA nodes (bit i = the i-th mask), lc / lm = the masks listed as hints, totc / totm =
 * the masks whose total covers the request (a hint is Preferred iff its size is the smallest of tot*), tot_*_any =
 * totc / totm non-empty; a resource the pod does not request (has_* = 0) or nil_hints (no provider output) adds no
 * list, an empty lc / lm with tot_*_any adds the reference's {nil, false} marker. score[i]: the hint score of
 * position i (numaScorer). out: admit, whether an affinity is set, and its mask. */
typedef struct gs_merge_case {
  uint32_t lc, totc, lm, totm;
  int32_t nz, policy;
  int32_t nil_hints, has_cpu, has_mem, tot_c_any, tot_m_any;
  int32_t score[15];
  /* A second provider (DeviceShare, deviceshare/topology_hint.go:33-214), merged after these lists: bits 0-14 its hint
   * positions, bits 16-18 the preferred size, bits 20-21 the number of identical lists (one per resource name; 0 = no
   * second provider: the two-list merge every pair evaluation runs); no position with lists = each list empty. */
  uint32_t gpu_hints;
  int32_t pad;
} gs_merge_case;
typedef struct gs_merge_result {
  int32_t admit, aff_has;
  uint32_t aff;
  int32_t pad;
} gs_merge_result;
int gs_debug_numa_merge(gs_ctx* ctx, const gs_merge_case* cases, uint32_t n, gs_merge_result* out);
/* ---- Coscheduling: the PodGroupManager of pkg/scheduler/plugins/coscheduling/core/core.go over its
 * gang cache (gang.go, gang_cache.go) as host state. A per-pod gate in front of gs_schedule (PreFilter) and the Permit /
 * PostFilter / Unreserve / PostBind decisions on assumed pods; a rejected pod's Reserve is undone by gs_pods_forget.
 * Gangs are keyed by the caller's 64-bit key of GetId(namespace, name), pods by UID (koordinator_amd/gang.py). */
#define GS_GANG_STRICT 0
#define GS_GANG_NONSTRICT 1
#define GS_GANG_ONCE_SATISFIED 0        /* extension.GangMatchPolicyOnceSatisfied (the default) */
#define GS_GANG_ONLY_WAITING 1
#define GS_GANG_WAITING_AND_RUNNING 2
#define GS_GANG_GROUP_MAX 8
typedef struct gs_gang_args {           /* CoschedulingArgs */
  int64_t default_timeout_ns;           /* DefaultTimeout (600 s) */
  int32_t skip_check_schedule_cycle;    /* SkipCheckScheduleCycle */
  int32_t pad;
} gs_gang_args;
typedef struct gs_gang_spec {           /* a PodGroup, or a pod's gang annotations, decoded (gang.go:112-232) */
  uint64_t gang_id;
  int32_t min_member;                   /* Spec.MinMember / the min-available annotation (< 0: illegal: no init) */
  int32_t total_children;               /* the total-number annotation (-1: absent or not an integer) */
  int32_t mode;                         /* GS_GANG_STRICT / _NONSTRICT (-1: absent or illegal: Strict) */
  int32_t match_policy;                 /* GS_GANG_* policy (-1: absent or illegal: once-satisfied) */
  int64_t wait_time_ns;                 /* ScheduleTimeoutSeconds / the wait-time annotation (-1: absent or illegal) */
  int64_t create_time_ns;
  uint32_t group_n, pad;                /* the gang-groups annotation (0: the gang alone) */
  uint64_t group[GS_GANG_GROUP_MAX];
} gs_gang_spec;
typedef struct gs_gang_info {
  int32_t has_init, min_member, total_children, mode, match_policy, schedule_cycle, schedule_cycle_valid,
      once_resource_satisfied, children, waiting, bound, pad;
  int64_t wait_time_ns;
} gs_gang_info;
#define GS_GANG_PREFILTER_OK 0
#define GS_GANG_PREFILTER_NOT_FOUND 1           /* "can't find gang" */
#define GS_GANG_PREFILTER_NOT_INIT 2            /* "gang has not init" */
#define GS_GANG_PREFILTER_NOT_ENOUGH_CHILDREN 3 /* "gang child pod not collect enough" */
#define GS_GANG_PREFILTER_CYCLE_INVALID 4       /* "gang scheduleCycle not valid" */
#define GS_GANG_PREFILTER_CYCLE_TOO_LARGE 5     /* "pod's schedule cycle too large" */
#define GS_GANG_PERMIT_SUCCESS 0
#define GS_GANG_PERMIT_WAIT 1
#define GS_GANG_PERMIT_NOT_FOUND 2
typedef struct gs_gang_mgr gs_gang_mgr;
void gs_gang_args_default(gs_gang_args* a);
int gs_gang_mgr_create(const gs_gang_args* args, gs_gang_mgr** out);
int gs_gang_mgr_destroy(gs_gang_mgr* m);
int gs_gang_mgr_clone(const gs_gang_mgr* m, gs_gang_mgr** out);      /* a copy of the whole state (speculation) */
int gs_gang_mgr_assign(gs_gang_mgr* dst, const gs_gang_mgr* src);    /* dst := src */
int gs_gang_podgroup_upsert(gs_gang_mgr* m, const gs_gang_spec* s);  /* onPodGroupAdd / Update: tryInitByPodGroup */
int gs_gang_podgroup_delete(gs_gang_mgr* m, uint64_t gang_id);
/* onPodAdd / onPodUpdate of a gang pod (gang_cache.go:85-120); annot: the pod's gang annotations when it has no PodGroup
 * label (NULL otherwise); assigned: Spec.NodeName is set. */
int gs_gang_pod_add(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, int assigned, const gs_gang_spec* annot);
int gs_gang_pod_delete(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid);
/* PreFilter (core.go:221-272); gang_id 0: not a gang pod. Returns a GS_GANG_PREFILTER_* code (not OK:
 * UnschedulableAndUnresolvable, then PostFilter). nominated: Status.NominatedNodeName is set. */
int gs_gang_prefilter(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, int nominated);
/* Permit (core.go:312-339, coscheduling.go:190-210) of an assumed pod: GS_GANG_PERMIT_SUCCESS with allowed[] = the gang
 * group's waiting pods that go on to bind, _WAIT (deadline now_ns + *wait_ns), or _NOT_FOUND. */
int gs_gang_permit(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, int64_t now_ns, int64_t* wait_ns, uint64_t* allowed,
                   uint32_t cap, uint32_t* n_allowed);
int gs_gang_post_bind(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid);   /* PostBind (core.go:397-447) */
/* PostFilter (core.go:277-307) of a gang pod that found no node: rejected[] = waiting pods to Unreserve. */
int gs_gang_post_filter(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, uint64_t* rejected, uint32_t cap,
                        uint32_t* n_rejected);
/* Unreserve (core.go:344-361) of a rejected / failed assumed gang pod: rejected[] = further waiting pods to Unreserve. */
int gs_gang_unreserve(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, uint64_t* rejected, uint32_t cap,
                      uint32_t* n_rejected);
/* The framework's Permit timeout at now_ns: rejected[] = waiting pods past their deadline (Unreserve follows). */
int gs_gang_expire(gs_gang_mgr* m, int64_t now_ns, uint64_t* rejected, uint32_t cap, uint32_t* n_rejected);
int gs_gang_get(const gs_gang_mgr* m, uint64_t gang_id, gs_gang_info* out);   /* 1: found, 0: no such gang */
int gs_gang_child_cycle(const gs_gang_mgr* m, uint64_t gang_id, uint64_t uid); /* ChildrenScheduleRoundMap (-1: none) */
int gs_gang_waiting_pods(const gs_gang_mgr* m, uint64_t* uids, uint32_t cap, uint32_t* n);
/* Test hook (the reference's tests set gang fields directly): what 0 ScheduleCycleValid, 1 the pod's schedule cycle,
 * 2 OnceResourceSatisfied, 3 GangMatchPolicy (3: a value outside the three), 4 SkipCheckScheduleCycle. */
int gs_gang_debug_set(gs_gang_mgr* m, uint64_t gang_id, uint64_t uid, int what, int value);

/* Coscheduling around the batched node loop, natively (the per-pod gate loop of koordinator_amd/gang.py
 * schedule_with_gangs): the reference runs PreFilter -> node loop -> Reserve -> Permit (PostFilter after a failure,
 * the Unreserve chain of rejected waiting pods) one pod at a time; a pass runs the gang side of that order over a
 * queue of n pods between the caller's engine calls.
 *  - gs_gang_walk: from pod i, the speculative walk (snapshot of the gang state taken first): every pod whose PreFilter
 *    passes is assumed to find a node and joins the run (run[], *run_n); the walk stops after run_cap pods, after a
 *    PreFilter failure whose PostFilter rejects waiting pods, or after a Permit "Gang not found"; *j = the pod after it.
 *  - the caller schedules the run's pods in one engine call (gs_schedule) -> got_node[run_n];
 *  - gs_gang_replay: restores the snapshot and replays [i, j) pod by pod with the true nodes (PreFilter, PostFilter,
 *    Reserve -> Permit, PostBind of the pods Permit allows, Unreserve chains), checking the walk: it stops at the first
 *    pod whose real PreFilter verdict differs from the walk's or whose transitions forget an assumed pod. *r_stop: the
 *    run positions kept (the caller withdraws the run's later placements with gs_pods_forget), *j_next: the next pod;
 *    *single >= 0: that pod passes PreFilter where the walk assumed not — the caller schedules it alone and reports its
 *    node with gs_gang_pass_after_single.
 * Per-pod results go to the pass's arrays (PreFilter code, Permit status or -1, GS_GANG_ST_*, node); the pods the
 * Unreserve chains reject are listed for ForgetPod (gs_gang_pass_forgets: uids in rejection order, this queue's pods
 * and pods waiting from earlier passes), and state changes of pods waiting from earlier passes are listed too
 * (gs_gang_pass_carried). Restatement: oracle/coscheduling.py schedule_sequential. */
enum { GS_GANG_ST_UNSCHEDULABLE = 0, GS_GANG_ST_WAITING = 1, GS_GANG_ST_BOUND = 2, GS_GANG_ST_REJECTED = 3 };
typedef struct gs_gang_pass gs_gang_pass;
int gs_gang_pass_create(gs_gang_mgr* m, uint32_t n, const uint64_t* gang_ids, const uint64_t* uids,
                        const uint8_t* nominated, int64_t now_ns, int8_t* prefilter, int8_t* permit, int8_t* state,
                        int32_t* node, gs_gang_pass** out);
int gs_gang_pass_destroy(gs_gang_pass* p);
int gs_gang_walk(gs_gang_pass* p, uint32_t i, uint32_t run_cap, uint32_t* run, uint32_t* run_n, uint32_t* j);
int gs_gang_replay(gs_gang_pass* p, uint32_t i, uint32_t j, const uint32_t* run, uint32_t run_n,
                   const int32_t* got_node, uint32_t* r_stop, uint32_t* j_next, int32_t* single);
int gs_gang_pass_after_single(gs_gang_pass* p, uint32_t k, int32_t node);
/* the rejected pods to forget since the last call (uids; cleared by the call), and the new states of pods waiting
 * from earlier passes (uid, GS_GANG_ST_*; cumulative over the pass) */
int gs_gang_pass_forgets(gs_gang_pass* p, uint64_t* uids, uint32_t cap, uint32_t* n);
int gs_gang_pass_carried(gs_gang_pass* p, uint64_t* uids, int8_t* states, uint32_t cap, uint32_t* n);

/* sizeof() of the ABI structs as compiled into the library, in this order: gs_pod, gs_node,
 * gs_node_metric, gs_pod_metric, gs_config, gs_placement, gs_stats, gs_loadaware_args, gs_cpu_topology,
 * gs_node_numa, gs_pod_allocation, gs_numa_args, gs_quota_group, gs_quota_status. */
void gs_abi_sizes(uint64_t* out, uint32_t n);

#ifdef __cplusplus
}
#endif

#endif /* GPUSCORE_H */
