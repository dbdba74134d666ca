"""C-ABI boundary checks that need no GPU: exports, struct layout, args defaulting/validation,
and that the product path refuses to run (loudly) without a device."""
import ctypes as C
import os

import numpy as np
import pytest

from koordinator_amd import abi, build, config, objects

torch_cuda = None
try:
    import torch
    torch_cuda = torch.cuda.is_available()
except Exception:
    torch_cuda = False


@pytest.fixture(scope="module")
def lib():
    build.build()
    return abi.load()


def test_exports_every_header_symbol(lib):
    syms = abi.header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/gpuscore.h but not exported"
    assert set(syms) == set(abi.SIGNATURES), "abi.SIGNATURES out of sync with the header"


def test_struct_sizes_match_library(lib):
    names = ["gs_pod", "gs_node", "gs_node_metric", "gs_pod_metric", "gs_config", "gs_placement", "gs_stats",
             "gs_loadaware_args", "gs_cpu_topology", "gs_node_numa", "gs_pod_allocation", "gs_numa_args",
             "gs_quota_group", "gs_quota_status", "gs_node_devices", "gs_reservation", "gs_pod_ext", "gs_ext_args",
             "gs_ext_placement"]
    arr = (C.c_uint64 * len(names))()
    lib.gs_abi_sizes(arr, len(names))
    for name, size in zip(names, arr):
        assert abi.STRUCT_SIZES[name] == size, name


def test_loadaware_defaults_match_v1beta2(lib):
    a = abi.GsLoadAwareArgs()
    lib.gs_loadaware_args_default(C.byref(a))
    b = config.loadaware_args()
    assert bytes(a) == bytes(b)
    assert a.node_metric_expiration_seconds == 180 and a.filter_expired_node_metrics == 1
    assert list(a.usage_thresholds) == [65, 95] and list(a.estimated_scaling_factors) == [85, 70]


@pytest.mark.parametrize("kw,msg", [
    ({"nodeMetricExpirationSeconds": -1}, b"nodeMetricExpiredSeconds should be a positive value"),
    ({"resourceWeights": {"cpu": 0}}, b"resource Weight should be a positive value"),
    ({"resourceWeights": {"cpu": 101}}, b"resource Weight should be less than 100"),
    ({"usageThresholds": {"cpu": 101}}, b"resource Threshold should be less than 100"),
    ({"estimatedScalingFactors": {"cpu": 0}}, b"estimated resource Threshold should be a positive value"),
])
def test_loadaware_validation(lib, kw, msg):
    a = config.loadaware_args(**kw)
    buf = C.create_string_buffer(256)
    assert lib.gs_loadaware_args_validate(C.byref(a), buf, 256) == abi.GS_EINVAL
    assert buf.value == msg


def test_validation_accepts_defaults(lib):
    a = config.loadaware_args()
    assert lib.gs_loadaware_args_validate(C.byref(a), None, 0) == 0


def test_unsupported_resource_rejected():
    with pytest.raises(ValueError):
        config.loadaware_args(resourceWeights={"nvidia.com/gpu": 1})


@pytest.mark.skipif(bool(torch_cuda), reason="GPU present: the no-GPU failure path is not reachable")
def test_no_gpu_fails_loudly():
    from koordinator_amd import engine
    cfg = config.make_config(16)
    with pytest.raises(engine.GpuScoreError):
        engine.Engine(cfg)


def test_local_group_host_side(lib):
    """The device transport's group is host-only state: it is created and destroyed without a GPU, and refuses a bad
    rank count; binding a context to it needs one (GPU tests: test_gpu_parity.py)."""
    import ctypes as C
    from koordinator_amd.engine import LocalGroup
    g = LocalGroup(4)
    assert g._h
    del g
    h = C.c_void_p()
    assert lib.gs_local_group_create(0, C.byref(h)) != 0
    assert lib.gs_local_group_create(abi.MAX_RANKS + 1 if hasattr(abi, "MAX_RANKS") else 9, C.byref(h)) != 0
    assert lib.gs_comm_init_local(None, None, 0) != 0


def test_pod_decoding_quantities():
    p = objects.make_pod({"containers": [{"requests": {"cpu": "1500m", "memory": "1Gi"},
                                          "limits": {"cpu": "2", "memory": "1Gi"}}]})
    assert list(p["requests"][:2]) == [1500, 1 << 30]
    assert list(p["limits"][:2]) == [2000, 1 << 30]
    assert list(p["nonzero_requests"]) == [1500, 1 << 30]
    assert p["priority_class"] == abi.GS_PRIO_PROD     # Burstable -> LS -> Prod
    be = objects.make_pod({"containers": [{}]})
    assert be["priority_class"] == abi.GS_PRIO_BATCH   # BestEffort -> BE -> Batch
    assert list(be["nonzero_requests"]) == [100, 200 << 20]


def test_reason_strings():
    """gs_reason_string renders the reference's Filter statuses: NodeNUMAResource's Err* constants
    (nodenumaresource/plugin.go:48-55) and the reasons of util.go:117, topology_hint.go:36, manager.go:70,
    resource_manager.go:292, with their framework codes; upstream Fit reasons joined like Status.Message()."""
    S = abi.GS_FAIL_NUMA_SHIFT
    want = {
        abi.GS_NUMA_INVALID_REQUESTED_CPUS: (2, "the requested CPUs must be integer"),
        abi.GS_NUMA_INVALID_AMP_RATIO: (2, "node(s) invalid CPU amplification ratio"),
        abi.GS_NUMA_AVAILABLE_CPUS_ERROR: (2, "node(s) invalid CPU Topology"),
        abi.GS_NUMA_INSUFFICIENT_AMP_CPU: (1, "Insufficient amplified cpu"),
        abi.GS_NUMA_INVALID_TOPOLOGY: (2, "node(s) invalid CPU Topology"),
        abi.GS_NUMA_BIND_POLICY_CONFLICT: (2, "node(s) cpu bind policy conflicts with pod's required cpu bind policy"),
        abi.GS_NUMA_SMT_ALIGNMENT: (2, "node(s) requested cpus not multiple cpus per core"),
        abi.GS_NUMA_ALLOCATE_FAILED: (1, "not enough cpus available to satisfy request"),
        abi.GS_NUMA_MISSING_NUMA_RESOURCES: (2, "node(s) missing NUMA resources"),
        abi.GS_NUMA_AFFINITY_ERROR: (1, "node(s) NUMA Topology affinity error"),
    }
    for r, w in want.items():
        assert abi.reason_string(r << S) == w, r
    assert abi.reason_string(0) == (0, "")
    assert abi.reason_string(abi.GS_FAIL_FIT_CPU | abi.GS_FAIL_FIT_MEMORY | abi.GS_FAIL_LOADAWARE) == \
        (1, "Insufficient cpu, Insufficient memory")           # the first failing plugin only
    assert abi.reason_string(abi.GS_FAIL_FIT_PODS) == (1, "Too many pods")
    assert abi.reason_string(abi.GS_FAIL_FIT_SCALAR, 1 << 3) == (1, "Insufficient kubernetes.io/batch-cpu")
    assert abi.reason_string(abi.GS_FAIL_LOADAWARE | abi.GS_FAIL_LA_MEMORY) == (1, "node(s) memory usage exceed threshold")
    assert abi.reason_string(abi.GS_FAIL_LOADAWARE | abi.GS_FAIL_LA_AGGREGATED) == \
        (1, "node(s) cpu aggregated usage exceed threshold")
    assert abi.reason_string(1 << 15)[0] < 0 and abi.reason_string(abi.GS_FAIL_LA_MEMORY)[0] < 0
