"""Plugin args and profile construction (host side).

Mirrors pkg/scheduler/apis/config/types.go:30-76 (LoadAwareSchedulingArgs) with the v1beta2 defaulting
of pkg/scheduler/apis/config/v1beta2/defaults.go:76-99 applied after the user's fields, exactly as
the scheduler's config decoding does (v1beta2 object -> SetDefaults -> Convert to internal config).
"""
from __future__ import annotations

from . import abi
from .objects import AGG_TYPES

DEFAULT_EXPIRATION_S = 180                       # defaults.go:33
DEFAULT_WEIGHTS = {"cpu": 1, "memory": 1}        # defaults.go:35-38
DEFAULT_THRESHOLDS = {"cpu": 65, "memory": 95}   # defaults.go:40-43
DEFAULT_SCALING = {"cpu": 85, "memory": 70}      # defaults.go:45-48


def _put(arr, mask_name, args, d: dict | None):
    vals, mask = [0, 0], 0
    for k, v in (d or {}).items():
        if k == "cpu":
            vals[0], mask = int(v), mask | abi.GS_USAGE_CPU
        elif k == "memory":
            vals[1], mask = int(v), mask | abi.GS_USAGE_MEMORY
        else:
            raise ValueError(f"LoadAware resource {k!r} is outside the supported set {{cpu, memory}}")
    getattr(args, arr)[0], getattr(args, arr)[1] = vals
    setattr(args, mask_name, mask)


def loadaware_args(filterExpiredNodeMetrics=None, nodeMetricExpirationSeconds=None, resourceWeights=None,
                   usageThresholds=None, prodUsageThresholds=None, scoreAccordingProdUsage=None,
                   estimatedScalingFactors=None, aggregated=None) -> abi.GsLoadAwareArgs:
    """v1beta2.LoadAwareSchedulingArgs fields (None = unset) -> defaulted internal args."""
    a = abi.GsLoadAwareArgs()
    a.filter_expired_node_metrics = 1 if filterExpiredNodeMetrics is None else int(bool(filterExpiredNodeMetrics))
    a.has_node_metric_expiration = 1
    a.node_metric_expiration_seconds = DEFAULT_EXPIRATION_S if nodeMetricExpirationSeconds is None \
        else int(nodeMetricExpirationSeconds)
    _put("resource_weights", "resource_weights_mask", a, resourceWeights or DEFAULT_WEIGHTS)
    _put("usage_thresholds", "usage_thresholds_mask", a, usageThresholds or DEFAULT_THRESHOLDS)
    _put("prod_usage_thresholds", "prod_usage_thresholds_mask", a, prodUsageThresholds)
    sf = dict(DEFAULT_SCALING) if estimatedScalingFactors is None else {**DEFAULT_SCALING, **estimatedScalingFactors}
    _put("estimated_scaling_factors", "estimated_scaling_factors_mask", a, sf)
    a.score_according_prod_usage = int(bool(scoreAccordingProdUsage))
    a.agg_usage_type = abi.GS_AGG_NONE
    a.agg_score_type = abi.GS_AGG_NONE
    if aggregated is not None:
        a.has_aggregated = 1
        _put("agg_usage_thresholds", "agg_usage_thresholds_mask", a, aggregated.get("usageThresholds"))
        a.agg_usage_type = AGG_TYPES[aggregated.get("usageAggregationType", "")]
        a.agg_usage_duration_ns = int(aggregated.get("usageAggregatedDurationSeconds", 0) * 10**9)
        a.agg_score_type = AGG_TYPES[aggregated.get("scoreAggregationType", "")]
        a.agg_score_duration_ns = int(aggregated.get("scoreAggregatedDurationSeconds", 0) * 10**9)
    return a


def fit_args(resources: dict | None = None) -> abi.GsFitArgs:
    """NodeResourcesFitArgs.ScoringStrategy (LeastAllocated) resources -> per-slot weights."""
    from .objects import RESOURCE_SLOTS
    f = abi.GsFitArgs()
    for k, w in (resources or {"cpu": 1, "memory": 1}).items():
        f.resource_weights[RESOURCE_SLOTS[k]] = int(w)
    return f


def numa_args(defaultCPUBindPolicy: str | None = None, scoringStrategy: dict | None = None,
              numaScoringStrategy: dict | None = None) -> abi.GsNumaArgs:
    """v1beta2.NodeNUMAResourceArgs (None = unset) -> defaulted internal args (defaults.go:101-136).
    scoringStrategy = {"type": "LeastAllocated"|"MostAllocated", "resources": {"cpu": 1, "memory": 1}}."""
    from .objects import RESOURCE_SLOTS
    a = abi.GsNumaArgs()
    a.default_cpu_bind_policy = abi.CPU_BIND["FullPCPUs" if defaultCPUBindPolicy is None else defaultCPUBindPolicy]
    ss = scoringStrategy or {"type": "LeastAllocated", "resources": {"cpu": 1, "memory": 1}}
    a.scoring_type = abi.GS_SCORING_MOST_ALLOCATED if ss.get("type") == "MostAllocated" else abi.GS_SCORING_LEAST_ALLOCATED
    for k, w in ss.get("resources", {}).items():
        a.resource_weights[RESOURCE_SLOTS[k]] = int(w)
    ns = numaScoringStrategy or {"type": "LeastAllocated"}
    a.numa_scoring_type = abi.GS_SCORING_MOST_ALLOCATED if ns.get("type") == "MostAllocated" \
        else abi.GS_SCORING_LEAST_ALLOCATED
    return a


def make_config(num_nodes: int, la: abi.GsLoadAwareArgs | None = None, fit: abi.GsFitArgs | None = None,
                enabled: int = abi.GS_ENABLE_LA_FIT, weights=(1, 1, 1), seed: int = 0x6B6F6F7264, device: int = 0,
                batch_size: int = 0, cand_cap: int = 0, numa: abi.GsNumaArgs | None = None,
                percentage_of_nodes_to_score: int | None = None) -> abi.GsConfig:
    """One scheduler profile: NodeResourcesFit + LoadAwareScheduling (+ NodeNUMAResource) with score weights."""
    cfg = abi.GsConfig()
    cfg.abi_version = abi.GS_ABI_VERSION
    cfg.device = device
    cfg.num_nodes = num_nodes
    cfg.enabled = enabled
    cfg.plugin_weights[abi.GS_PLUGIN_FIT] = weights[0]
    cfg.plugin_weights[abi.GS_PLUGIN_LOADAWARE] = weights[1]
    cfg.plugin_weights[abi.GS_PLUGIN_NUMA] = weights[2] if len(weights) > 2 else 1
    cfg.loadaware = la if la is not None else loadaware_args()
    cfg.fit = fit if fit is not None else fit_args()
    cfg.numa = numa if numa is not None else numa_args()
    cfg.seed = seed
    cfg.batch_size = batch_size
    cfg.cand_cap = cand_cap
    # None: every node is checked (percentageOfNodesToScore = 100, the parity harness); else the reference's
    # node sampling with this percentage (0 = adaptive)
    cfg.sample_nodes = 0 if percentage_of_nodes_to_score is None else 1
    cfg.percentage_of_nodes_to_score = percentage_of_nodes_to_score or 0
    return cfg
