"""Node reservation: the node transformer's allocatable trim, GetReservedCPUs and the NRT's
TopologyOptions.ReservedCPUs, through the C-ABI decoders (pure host functions: CPU tests). The vectors are the
reference's own test tables, transcribed as data:
  pkg/util/node_test.go:231-311                      TestTrimNodeAllocatableByNodeReservation
  pkg/util/transformer/node_transformer_test.go:89-258 TestNodeReservationTransformer (3 fake nodes per case)
  apis/extension/node_reservation_test.go:37-146     TestGetReservedCPUs
  pkg/scheduler/plugins/nodenumaresource/topology_options_test.go:50-139 (the ReservedCPUs union)
The reservation annotation is what json.Marshal(NodeReservation) writes (Quantity as a string, omitempty fields).
NodeResourcesFit's extended resources outside the 7 gs_node slots (nvidia.com/gpu in the first vector) live in the
DeviceShare mirror: not checked here."""
import json

import pytest

from koordinator_amd import abi, ingest

GI = 1 << 30
ANN = "node.koordinator.sh/reservation"


def _node(cpu_milli, mem, pods=0, eph=0, batch_cpu=0, batch_mem=0):
    n = abi.GsNode()
    n.allocatable[abi.GS_RES_CPU] = cpu_milli
    n.allocatable[abi.GS_RES_MEMORY] = mem
    n.allocatable[abi.GS_RES_EPHEMERAL] = eph
    n.allocatable[abi.GS_RES_BATCH_CPU] = batch_cpu
    n.allocatable[abi.GS_RES_BATCH_MEMORY] = batch_mem
    n.allowed_pod_number = pods
    return n


def _alloc(n):
    return [n.allocatable[i] for i in range(7)] + [n.allowed_pod_number]


def _rsv(resources=None, reserved_cpus="", policy=""):
    d = {}
    if resources:
        d["resources"] = resources
    if reserved_cpus:
        d["reservedCPUs"] = reserved_cpus
    if policy:
        d["applyPolicy"] = policy
    return json.dumps(d)


# node_test.go:231-293: 96 cores, 512Gi, batch-cpu 16, batch-memory 32Gi
TRIM = [
    ("trim cpu and memory but skip other resources", {"cpu": "16", "memory": "12Gi"}, "Default",
     (80_000, 500 * GI, 16, 32 * GI), True),
    ("skip trim", {"cpu": "16", "memory": "12Gi"}, "ReservedCPUsOnly", (96_000, 512 * GI, 16, 32 * GI), False),
]


@pytest.mark.parametrize("name,res,policy,want,trimmed", TRIM, ids=[t[0] for t in TRIM])
def test_trim_node_allocatable_by_node_reservation(name, res, policy, want, trimmed):
    n = _node(96_000, 512 * GI, batch_cpu=16, batch_mem=32 * GI)
    got = ingest.node_reservation_trim({ANN: _rsv(res, policy=policy)}, n)
    assert got == trimmed
    a = _alloc(n)
    assert (a[abi.GS_RES_CPU], a[abi.GS_RES_MEMORY], a[abi.GS_RES_BATCH_CPU], a[abi.GS_RES_BATCH_MEMORY]) == want


# node_transformer_test.go:33-87: allocatable cpu 10, memory 10Gi, pods 200, batch-cpu 1, ephemeral 10Gi, batch-mem 1Gi;
# expected = allocatable - GetNodeReservationFromAnnotation(...) for cpu / memory / ephemeral / pods / other scalars,
# batch-cpu and batch-memory unchanged, nothing trimmed for applyPolicy ReservedCPUsOnly
TRANSFORM = [
    ("reserve nothing", None, "", "", (0, 0)),
    ("reserve cpu by quantity", {"cpu": "1"}, "", "", (1000, 0)),
    ("reserve cpu by quantity with default policy", {"cpu": "1"}, "", "Default", (1000, 0)),
    ("reserve specific cores", None, "0-1", "", (2000, 0)),
    ("reserve specific cores with policy", None, "0-1", "Default", (2000, 0)),
    ("reserve specific cores and quantity", {"cpu": "1"}, "0-1", "", (2000, 0)),
    ("reserve memory by quantity", {"memory": "2Gi"}, "", "", (0, 2 * GI)),
    ("reserve memory and cpu by quantity", {"memory": "2Gi", "cpu": "1"}, "", "", (1000, 2 * GI)),
    ("reserve memory by quantity and reserve some specific cores", {"memory": "1Gi"}, "2", "", (1000, 1 * GI)),
    ("reserve batch memory by quantity", {"kubernetes.io/batch-memory": "1Gi"}, "", "", (0, 0)),
    ("reserve batch cpu by quantity", {"kubernetes.io/batch-cpu": "1"}, "", "", (0, 0)),
    ("only reserve cpus and do not trim allocatable", None, "0-3", "ReservedCPUsOnly", (0, 0)),
]


@pytest.mark.parametrize("name,res,cpus,policy,cut", TRANSFORM, ids=[t[0] for t in TRANSFORM])
@pytest.mark.parametrize("fake", ["with-reservation", "without-annotations", "without-node-reservation"])
def test_node_reservation_transformer(name, res, cpus, policy, cut, fake):
    base = (10_000, 10 * GI, 200, 10 * GI, 1, 1 * GI)
    n = _node(*base)
    ann = {"with-reservation": {ANN: _rsv(res, cpus, policy)}, "without-annotations": {},
           "without-node-reservation": {"k": "v"}}[fake]
    ingest.node_reservation_trim(ann, n)
    dcpu, dmem = cut if fake == "with-reservation" else (0, 0)
    a = _alloc(n)
    assert a[abi.GS_RES_CPU] == base[0] - dcpu
    assert a[abi.GS_RES_MEMORY] == base[1] - dmem
    assert a[abi.GS_RES_EPHEMERAL] == base[3]
    assert a[7] == base[2]
    assert a[abi.GS_RES_BATCH_CPU] == base[4] and a[abi.GS_RES_BATCH_MEMORY] == base[5]


def test_trim_floors_at_zero_and_pods():
    n = _node(2_000, 1 * GI, pods=10)
    assert ingest.node_reservation_trim({ANN: _rsv({"cpu": "4", "memory": "2Gi", "pods": "3"})}, n)
    assert _alloc(n)[abi.GS_RES_CPU] == 0 and _alloc(n)[abi.GS_RES_MEMORY] == 0 and n.allowed_pod_number == 7


def test_trim_malformed_annotation_is_ignored():
    for bad in ["{", "[]", json.dumps({"resources": {"cpu": "x"}}), json.dumps({"reservedCPUs": "0-a"}),
                json.dumps({"applyPolicy": 3})]:
        n = _node(8_000, 8 * GI)
        assert not ingest.node_reservation_trim({ANN: bad}, n), bad
        assert _alloc(n)[:2] == [8_000, 8 * GI]


def test_trim_negative_quantity_refused():
    with pytest.raises(ingest.DecodeError):
        ingest.node_reservation_trim({ANN: _rsv({"cpu": "-2"})}, _node(8_000, 8 * GI))


# node_reservation_test.go:37-146 GetReservedCPUs -> (reservedCPUs, numReservedCPUs); "-1" is returned as a string by
# the reference and fails cpuset.Parse where it is used (topology_options.go:110): no CPUs
RESERVED = [
    ("node.annotation is nil", None, [], 0, True),
    ("without cpu reserved", _rsv(), [], 0, True),
    ("reserve cpu only by quantity", _rsv({"cpu": "10"}), [], 10, True),
    ("reserve cpu only by quantity but value not integer", _rsv({"cpu": "2.5"}), [], 3, True),
    ("reserve cpu only by quantity but value is negative", _rsv({"cpu": "-2"}), [], 0, True),
    ("reserve cpu only by specific cpus", _rsv(reserved_cpus="0-1"), [0, 1], 0, True),
    ("reserve cpu only by specific cpus but core id is unavailable", _rsv(reserved_cpus="-1"), [], 0, False),
    ("reserve cpu by specific cpus and quantity", _rsv({"cpu": "10"}, "0-1"), [0, 1], 0, True),
]


@pytest.mark.parametrize("name,ann,cpus,num,parsed", RESERVED, ids=[t[0] for t in RESERVED])
def test_get_reserved_cpus(name, ann, cpus, num, parsed):
    got = ingest.node_reserved_cpus({} if ann is None else {ANN: ann})
    assert got == (cpus, num, parsed)


def test_topology_options_reserved_cpus_union():
    """topology_options_test.go:50-139: kubelet reservedCPUs 0-1, a kubelet-managed pod's 0-3, system QoS 4-5
    (exclusive by default), node reservation 6-7 -> 0-7; without the pod allocs -> 0-1,4-7."""
    ann = {
        "kubelet.koordinator.sh/cpu-manager-policy": json.dumps(
            {"policy": "static", "options": {"static": "true"}, "reservedCPUs": "0-1"}),
        "node.koordinator.sh/pod-cpu-allocs": json.dumps(
            [{"namespace": "default", "name": "pod-1", "uid": "4b6b1c38-5a25-4d5e-9f3d-2d8f0d7b6c11", "cpuset": "0-3",
              "managedByKubelet": True}]),
        "node.koordinator.sh/system-qos-resource": json.dumps({"cpuset": "4-5"}),
        ANN: _rsv(reserved_cpus="6-7"),
    }
    assert ingest.nrt_reserved_cpus(ann) == list(range(8))
    del ann["node.koordinator.sh/pod-cpu-allocs"]
    assert ingest.nrt_reserved_cpus(ann) == [0, 1, 4, 5, 6, 7]
    # a non-exclusive system-QoS cpuset and a pod not managed by kubelet add nothing
    ann["node.koordinator.sh/system-qos-resource"] = json.dumps({"cpuset": "4-5", "cpusetExclusive": False})
    ann["node.koordinator.sh/pod-cpu-allocs"] = json.dumps([{"uid": "u", "cpuset": "8-9"}])
    assert ingest.nrt_reserved_cpus(ann) == [0, 1, 6, 7]
