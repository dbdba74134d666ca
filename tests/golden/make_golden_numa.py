"""Transcribes the reference's own NodeNUMAResource test vectors into tests/golden/numa_takecpus.json.

Data only (inputs and expected outputs typed in from the Go tests); no reference code is copied or run.
Source: pkg/scheduler/plugins/nodenumaresource/cpu_accumulator_test.go
  TestTakeFullPCPUs                          :59-173   (FullPCPUs, NUMAMostAllocated)
  TestTakeFullPCPUsWithNUMALeastAllocated    :175-289  (FullPCPUs, NUMALeastAllocated)
  TestCPUSpreadByPCPUs                       :291-299  (freeCPUs + spreadCPUs order)
  TestTakeSpreadByPCPUs                      :301-361  (SpreadByPCPUs, NUMAMostAllocated)
  TestTakeSpreadByPCPUsWithNUMALeastAllocated:373-433
  TestTakeCPUsWithExclusivePolicy            :435-558
  TestTakeCPUsWithMaxRefCount                :560-599  (sequence, maxRefCount 2)
  TestTakeCPUsSortByRefCount                 :601-648  (sequence, maxRefCount 2)
  TestTakePreferredCPUs                      :724-744  (first call only: plain takeCPUs)

Topologies are buildCPUTopologyForTest(sockets, nodesPerSocket, coresPerNode, cpusPerCore) (:30-57).
Run: python tests/golden/make_golden_numa.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def parse(s):
    """cpuset.MustParse / NewCPUSet -> sorted list"""
    if isinstance(s, list):
        return sorted(s)
    out = []
    for part in s.split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return sorted(out)


def case(src, name, topo, need, want, allocated=(), bind="FullPCPUs", excl="None", strategy="MostAllocated",
         max_ref=1, alloc_excl=None, error=False):
    return {"src": src, "name": name, "topology": list(topo), "max_ref": max_ref, "allocated": parse(list(allocated)
            if not isinstance(allocated, str) else allocated), "alloc_excl": alloc_excl or "None", "needed": need,
            "bind": bind, "excl": excl, "strategy": strategy, "want": parse(want), "want_error": error}


T = "cpu_accumulator_test.go"
cases = []
# TestTakeFullPCPUs (Most) / ...WithNUMALeastAllocated
full_most = [
    ("allocate on non-NUMA node", (1, 1, 4, 2), [], 2, [0, 1]),
    ("with allocated cpus", (1, 1, 4, 2), [0, 1], 2, [2, 3]),
    ("allocate whole socket", (2, 1, 4, 2), [], 8, "0-7"),
    ("allocate across socket", (2, 1, 4, 2), [], 12, "0-11"),
    ("allocate whole socket with partially-allocated socket", (2, 1, 4, 2), [0, 1], 8, "8-15"),
    ("allocate in the smallest idle socket", (2, 2, 4, 2), "0-5,16-23", 6, "24-29"),
    ("allocate the most of CPUs on the same socket", (2, 2, 4, 2), "0-5,16-23", 12, "6-15,24-25"),
    ("allocate from first socket", (2, 2, 4, 2), "0-3,8-11", 4, "4-7"),
    ("allocate with less spread cpus", (2, 2, 2, 2), [0, 2, 4, 8, 12], 4, [10, 11, 14, 15]),
    ("allocate with the most spread cpus", (2, 2, 2, 2), [0, 2, 4, 8, 10, 12], 6, [5, 6, 7, 13, 14, 15]),
    ("allocate with the most spread cpus on the smallest idle cpus socket", (2, 2, 2, 2), [0, 2, 4, 8, 9, 10, 12], 6,
     [6, 7, 11, 13, 14, 15]),
]
for n, topo, al, need, want in full_most:
    cases.append(case(f"{T}:59-173 TestTakeFullPCPUs", n, topo, need, want, al))
full_least = [
    ("allocate on non-NUMA node", (1, 1, 4, 2), [], 2, [0, 1]),
    ("with allocated cpus", (1, 1, 4, 2), [0, 1], 2, [2, 3]),
    ("allocate whole socket", (2, 1, 4, 2), [], 8, "0-7"),
    ("allocate across socket", (2, 1, 4, 2), [], 12, "0-11"),
    ("allocate whole socket with partially-allocated socket", (2, 1, 4, 2), [0, 1], 8, "8-15"),
    ("allocate in the most idle socket", (2, 2, 4, 2), "0-5,16-23", 6, "8-13"),
    ("allocate the most of CPUs on the same socket", (2, 2, 4, 2), "0-5,16-23", 12, "6-15,24-25"),
    ("allocate from second socket", (2, 2, 4, 2), "0-3,8-11", 4, "16-19"),
    ("allocate with less spread cpus", (2, 2, 2, 2), [0, 2, 4, 8, 12], 4, [10, 11, 14, 15]),
    ("allocate with the less spread cpus 2", (2, 2, 2, 2), [0, 2, 4, 8, 10, 12], 6, [6, 7, 14, 15, 1, 3]),
    ("allocate with the most spread cpus on the most idle cpus socket 3", (2, 2, 4, 2), [0, 2, 4, 8, 9, 10, 12], 6,
     [16, 17, 18, 19, 20, 21]),
]
for n, topo, al, need, want in full_least:
    cases.append(case(f"{T}:175-289 TestTakeFullPCPUsWithNUMALeastAllocated", n, topo, need, want, al,
                      strategy="LeastAllocated"))
spread_most = [
    ("allocate on non-NUMA node", (1, 1, 4, 2), [], 4, [0, 2, 4, 6]),
    ("allocate satisfied the partially-allocated socket", (2, 1, 4, 2), [0, 2], 4, [1, 3, 4, 6]),
    ("allocate cpus on full-free socket", (2, 1, 4, 2), [0, 1, 2, 3], 4, [8, 10, 12, 14]),
    ("allocate most of CPUs in the same socket and overlapped-cores", (2, 1, 4, 2), [0, 2], 6, "1,3-7"),
]
for n, topo, al, need, want in spread_most:
    cases.append(case(f"{T}:301-361 TestTakeSpreadByPCPUs", n, topo, need, want, al, bind="SpreadByPCPUs"))
spread_least = [
    ("allocate on non-NUMA node", (1, 1, 4, 2), [], 4, [0, 2, 4, 6]),
    ("allocate satisfied the partially-allocated socket", (2, 1, 4, 2), [0, 2], 4, [8, 10, 12, 14]),
    ("allocate cpus on full-free socket", (2, 1, 4, 2), [0, 1, 2, 3], 4, [8, 10, 12, 14]),
    ("allocate most of CPUs in the same socket and overlapped-cores", (2, 1, 4, 2), [0, 2], 6,
     [8, 10, 12, 14, 9, 11]),
]
for n, topo, al, need, want in spread_least:
    cases.append(case(f"{T}:373-433 TestTakeSpreadByPCPUsWithNUMALeastAllocated", n, topo, need, want, al,
                      bind="SpreadByPCPUs", strategy="LeastAllocated"))
# TestTakeCPUsWithExclusivePolicy: allocated CPUs carry allocatedExclusivePolicy (default PCPULevel);
# exclusivePolicy defaults to PCPULevel, bindPolicy to SpreadByPCPUs
excl_cases = [
    ("allocate cpus on full-free socket with PCPULevel", (2, 1, 4, 2), [0, 2], None, None, None, 4, [8, 10, 12, 14]),
    ("allocate overlapped cpus with PCPULevel", (2, 1, 4, 2), [], None, None, None, 10, [0, 1, 2, 3, 4, 6, 8, 10, 12, 14]),
    ("allocate cpus on large-size partially-allocated socket with PCPULevel", (2, 1, 8, 2), [0, 2], None, None, None, 4,
     [4, 6, 8, 10]),
    ("allocate cpus with none exclusive policy", (2, 1, 8, 2), [0, 2], None, "None", None, 4, [1, 3, 4, 6]),
    ("allocate cpus on full-free socket with NUMANodeLevel", (2, 1, 4, 2), [0, 2], "NUMANodeLevel", "NUMANodeLevel",
     None, 4, [8, 10, 12, 14]),
    ("allocate cpus on partially-allocated socket without NUMANodeLevel", (2, 1, 4, 2), [0, 2], "NUMANodeLevel", "None",
     None, 4, [1, 3, 4, 6]),
    ("allocate cpus on full-free socket with NUMANodeLevel with PCPUs", (2, 1, 4, 2), [0, 2], "NUMANodeLevel",
     "NUMANodeLevel", "FullPCPUs", 4, [8, 9, 10, 11]),
    ("allocate cpus on partially-allocated socket without NUMANodeLevel with PCPUs", (2, 1, 4, 2), [0, 2],
     "NUMANodeLevel", "None", "FullPCPUs", 4, [4, 5, 6, 7]),
]
for n, topo, al, aexcl, excl, bind, need, want in excl_cases:
    # an unset exclusivePolicy ("") is defaulted to PCPULevel; CPUExclusivePolicyNone is the string "None"
    e = "PCPULevel" if excl is None else excl
    cases.append(case(f"{T}:435-558 TestTakeCPUsWithExclusivePolicy", n, topo, need, want, al,
                      bind=bind or "SpreadByPCPUs", excl=e, alloc_excl=aexcl or "PCPULevel"))
cases.append(case(f"{T}:724-744 TestTakePreferredCPUs", "takeCPUs spread 2", (2, 1, 16, 2), 2, [0, 2],
                  bind="SpreadByPCPUs"))

# sequences (maxRefCount 2): each step takes CPUs then addCPUs(..., PCPULevel)
sequences = [
    {"src": f"{T}:560-599 TestTakeCPUsWithMaxRefCount", "topology": [1, 1, 4, 2], "max_ref": 2,
     "steps": [{"needed": 4, "bind": "FullPCPUs", "want": parse("0-3")},
               {"needed": 5, "bind": "FullPCPUs", "want": parse("0,4-7")},
               {"needed": 4, "bind": "FullPCPUs", "want": parse("2-5")}]},
    {"src": f"{T}:601-648 TestTakeCPUsSortByRefCount", "topology": [1, 1, 16, 2], "max_ref": 2,
     "steps": [{"needed": 16, "bind": "SpreadByPCPUs", "want": parse("0,2,4,6,8,10,12,14,16,18,20,22,24,26,28,30")},
               {"needed": 16, "bind": "FullPCPUs", "want": parse("0-15")},
               {"needed": 16, "bind": "SpreadByPCPUs", "want": parse("1,3,5,7,9,11,13,15,17,19,21,23,25,27,29,31")},
               {"needed": 16, "bind": "FullPCPUs", "want": parse("16-31")}],
     "final_available": []},
]

out = {"takecpus": cases, "sequences": sequences,
       "spread_order": {"src": f"{T}:291-299 TestCPUSpreadByPCPUs", "topology": [2, 2, 4, 2], "needed": 8,
                        "want": [0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20, 22, 24, 26, 28, 30,
                                 1, 3, 5, 7, 9, 11, 13, 15, 17, 19, 21, 23, 25, 27, 29, 31]}}
with open(os.path.join(HERE, "numa_takecpus.json"), "w") as f:
    json.dump(out, f, indent=1)
print(f"wrote {len(cases)} takeCPUs cases, {len(sequences)} sequences")

# ---- plugin-level vectors: scoring_test.go --------------------------------------------------------
S = "scoring_test.go"
GI = 1 << 30


def numa_node(cpu, mem_gi, policy, count):
    """TestNUMANodeScore node: Capacity(cpu, memory) + numa-topology-policy label; options per scoring_test.go:255-272"""
    cpu_milli, mem = cpu * 1000, mem_gi * GI
    cores = cpu_milli // 1000 // 2 // count
    return {"cpu_milli": cpu_milli, "memory": mem, "numa_policy": policy, "topology": [count, 1, cores, 2],
            "zones": [[i, cpu_milli // count, mem // count] for i in range(count)]}


def existing(node, uid, cpu, mem_gi, cpuset_pod):
    """resourceManager.Update of an existing pod (scoring_test.go:274-293): cpuset 0..cpu-1 when LSR+Prod,
    NUMANodeResources [{Node 0, container requests}]"""
    return {"node": node, "uid": uid, "cpus": list(range(cpu)) if cpuset_pod else [],
            "numa": [[0, cpu * 1000, mem_gi * GI]]}


most = {"scoring": "MostAllocated", "weights": {"cpu": 1, "memory": 1}}
score_cases = [
    {"src": f"{S}:47-330 TestNUMANodeScore", "name": "single numa nodes score", "args": most,
     "nodes": [numa_node(104, 256, "SingleNUMANode", 2), numa_node(64, 128, "SingleNUMANode", 1)],
     "allocations": [], "pod": {"cpu": 21000, "memory": 40 * GI}, "filter": True, "want": [35, 31]},
    {"src": f"{S}:47-330 TestNUMANodeScore", "name": "restricted numa nodes score", "args": most,
     "nodes": [numa_node(104, 256, "Restricted", 2), numa_node(64, 128, "Restricted", 1)],
     "allocations": [], "pod": {"cpu": 50000, "memory": 40 * GI}, "filter": True, "want": [63, 54]},
    {"src": f"{S}:47-330 TestNUMANodeScore", "name": "single numa nodes score with same capacity but different requested",
     "args": most, "nodes": [numa_node(104, 256, "SingleNUMANode", 2)] * 3,
     "allocations": [existing(0, 0, 4, 8, False), existing(1, 0, 8, 32, False), existing(2, 0, 32, 40, False)],
     "pod": {"cpu": 4000, "memory": 40 * GI}, "filter": True, "want": [19, 19, 19]},
    {"src": f"{S}:47-330 TestNUMANodeScore",
     "name": "single numa nodes score with same capacity but different requested and LSR", "args": most,
     "nodes": [numa_node(104, 256, "SingleNUMANode", 2)] * 3,
     "allocations": [existing(0, 0, 4, 8, False), existing(0, 123, 4, 8, True),
                     existing(1, 0, 8, 32, False), existing(1, 123, 8, 32, True),
                     existing(2, 0, 16, 40, False), existing(2, 123, 16, 40, True)],
     "pod": {"cpu": 4000, "memory": 40 * GI, "qos": "LSR", "prod": True}, "filter": True, "want": [23, 27, 34]},
]


def plain_node(topo, labels=None):
    """TestPlugin_Score node (scoring_test.go:478-496): allocatable cpu = |CPUs|, memory 512Gi; options hold only
    the CPUTopology (MaxRefCount defaulted to 1 by UpdateTopologyOptions)"""
    s, n, c, p = topo
    d = {"cpu_milli": s * n * c * p * 1000, "memory": 512 * GI, "numa_policy": "", "topology": list(topo),
         "zones": []}
    d.update(labels or {})
    return d


cpu_most = {"scoring": "MostAllocated", "weights": {"cpu": 1}}
plugin_score = [
    ("score with full empty node FullPCPUs", (2, 1, 4, 2), "FullPCPUs", 4, {}, 25),
    ("score with satisfied node FullPCPUs", (2, 1, 4, 2), "FullPCPUs", 8, {}, 50),
    ("score with full empty node SpreadByPCPUs", (2, 1, 4, 2), "SpreadByPCPUs", 4, {}, 25),
    ("score with exceed socket FullPCPUs", (2, 1, 4, 2), "FullPCPUs", 16, {}, 100),
    ("score with satisfied socket FullPCPUs", (2, 2, 4, 2), "FullPCPUs", 16, {}, 50),
    ("score with full empty socket SpreadByPCPUs", (2, 1, 4, 2), "SpreadByPCPUs", 4, {}, 25),
    ("score with Node NUMA Allocate Strategy", (2, 1, 4, 2), "SpreadByPCPUs", 2,
     {"numa_allocate_strategy": "LeastAllocated"}, 12),
    ("score with Node CPU Bind Policy", (2, 1, 4, 2), "SpreadByPCPUs", 8, {"node_cpu_bind": "FullPCPUsOnly"}, 50),
]
for name, topo, pref, n, labels, want in plugin_score:
    # the Go test injects preFilterState{requestCPUBind, preferredCPUBindPolicy, numCPUsNeeded, requests{cpu}};
    # an LSR Prod pod with that preferred policy and cpu request makes PreFilter produce the same state
    score_cases.append({"src": f"{S}:332-554 TestPlugin_Score", "name": name, "args": cpu_most,
                        "nodes": [plain_node(topo, labels)], "allocations": [],
                        "pod": {"cpu": n * 1000, "qos": "LSR", "prod": True, "preferred": pref},
                        "filter": False, "want": [want]})

with open(os.path.join(HERE, "numa_score.json"), "w") as f:
    json.dump({"cases": score_cases}, f, indent=1)
print(f"wrote {len(score_cases)} NodeNUMAResource score cases")

# ---- plugin-level Filter / affinity / Reserve vectors: plugin_test.go -----------------------------------------
P = "plugin_test.go"


def filter_node(labels=None):
    """TestPlugin_Filter node (plugin_test.go:827-876): allocatable cpu 96, memory 512Gi; options = CPUTopology
    (2,1,4,2) + one NUMANodeResource per NUMA node {cpu: CPUsPerNode, memory: 32Gi}"""
    d = {"cpu_milli": 96000, "memory": 512 * GI, "numa_policy": "", "topology": [2, 1, 4, 2],
         "zones": [[0, 8000, 32 * GI], [1, 8000, 32 * GI]]}
    d.update(labels or {})
    return d


# (name, lines, node labels, pod, want reason); the Go test writes preFilterState directly: requestCPUBind
# true <=> an LSR Prod pod with the listed policies, false <=> an LS pod with the same cpu request
LSR = {"qos": "LSR", "prod": True}
filter_cases = [
    ("failed to verify Node FullPCPUsOnly with SMTAlignmentError", "592-605", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 5000, **LSR, "preferred": "FullPCPUs"}, "SMT_ALIGNMENT"),
    ("LS Pod failed to verify Node FullPCPUsOnly with SMTAlignmentError", "606-621", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 5000}, "SMT_ALIGNMENT"),
    ("LS Pod failed to verify Node FullPCPUsOnly with non-integer request", "622-637", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 5200}, "INVALID_REQUESTED_CPUS"),
    ("verify Node FullPCPUsOnly", "638-651", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 4000, **LSR, "preferred": "FullPCPUs"}, None),
    ("failed to verify required FullPCPUs SMTAlignmentError", "652-662", {},
     {"cpu": 5000, **LSR, "required": "FullPCPUs"}, "SMT_ALIGNMENT"),
    ("verify required FullPCPUs", "663-673", {}, {"cpu": 4000, **LSR, "required": "FullPCPUs"}, None),
    ("verify FullPCPUsOnly with preferred SpreadByPCPUs", "674-687", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 4000, **LSR, "preferred": "SpreadByPCPUs"}, None),
    ("failed to verify FullPCPUsOnly with required SpreadByPCPUs", "688-701", {"node_cpu_bind": "SpreadByPCPUs"},
     {"cpu": 4000, **LSR, "required": "FullPCPUs"}, "BIND_POLICY_CONFLICT"),
    ("verify FullPCPUsOnly with required FullPCPUs", "702-715", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 4000, **LSR, "required": "FullPCPUs"}, None),
    # the kubelet static policy with full-pcpus-only decodes to the node CPU bind policy FullPCPUsOnly
    ("verify Kubelet FullPCPUsOnly with SMTAlignmentError", "716-732", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 5000, **LSR, "preferred": "FullPCPUs"}, "SMT_ALIGNMENT"),
    ("verify Kubelet FullPCPUsOnly with required SpreadByPCPUs", "733-749", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 4000, **LSR, "required": "SpreadByPCPUs"}, "BIND_POLICY_CONFLICT"),
    ("verify Kubelet FullPCPUsOnly with required FullPCPUs", "750-766", {"node_cpu_bind": "FullPCPUsOnly"},
     {"cpu": 4000, **LSR, "required": "FullPCPUs"}, None),
    ("verify required FullPCPUs with none NUMA topology policy", "767-777", {},
     {"cpu": 4000, **LSR, "required": "FullPCPUs", "preferred": "FullPCPUs"}, None),
    ("verify FullPCPUs with NUMA Topology Policy", "778-791", {"numa_policy": "SingleNUMANode"},
     {"cpu": 4000, **LSR, "required": "FullPCPUs", "preferred": "FullPCPUs"}, None),
    ("verify FullPCPUs with NUMA Topology Policy and amplification ratio", "792-808",
     {"numa_policy": "SingleNUMANode", "node_cpu_ratio": 1.5},
     {"cpu": 4000, **LSR, "required": "FullPCPUs", "preferred": "FullPCPUs"}, None),
    ("verify FullPCPUs with None NUMA Topology Policy and amplification ratio", "809-825", {"node_cpu_ratio": 1.5},
     {"cpu": 4000, **LSR, "required": "FullPCPUs", "preferred": "FullPCPUs"}, None),
]
default_args = {"scoring": "LeastAllocated", "weights": {"cpu": 1, "memory": 1}}
plugin_cases = []
for name, lines, labels, pod, want in filter_cases:
    plugin_cases.append({"kind": "filter", "src": f"{P}:{lines} TestPlugin_Filter", "name": name, "args": default_args,
                         "nodes": [filter_node(labels)], "allocations": [], "pod": pod, "filter": True,
                         "want_reason": want})


def amp_node(ratio, nrt, requested_cpu):
    """TestFilterWithAmplifiedCPUs node (plugin_test.go:969-996): makeNode(cpu = NumCPUs of (2,1,8,2) = 32,
    memory 40Gi, ratio) amplifies allocatable cpu; with NRT the options hold the CPUTopology and per NUMA node
    {cpu: Amplify(CPUsPerNode, ratio), memory 20Gi}; without NRT there are no topology options"""
    amp = lambda x: x if ratio <= 1 else int(-(-x * ratio // 1))   # noqa: E731  (ceil; integral here)
    d = {"cpu_milli": amp(32000), "memory": 40 * GI, "numa_policy": "", "node_cpu_ratio": ratio,
         "requested_cpu": requested_cpu}
    if nrt:
        d.update({"topology": [2, 1, 8, 2], "zones": [[0, amp(16) * 1000, 20 * GI], [1, amp(16) * 1000, 20 * GI]]})
    else:
        d.update({"topology": None, "zones": [], "has_options": False})
    return d


# (name, lines, pod cpu (None: no requests), pod is cpuset, existing cpu, existing is cpuset, nrt, ratio, want)
amp_cases = [
    ("no resources requested always fits", "911-917", None, False, 4, False, False, 2.0, None),
    ("no filtering without node cpu amplification", "918-924", 32, False, 32, False, False, 1.0, None),
    ("cpu fits on no NRT node", "925-931", 32, False, 32, False, False, 2.0, None),
    ("insufficient cpu", "932-939", 32, False, 64, False, False, 2.0, "INSUFFICIENT_AMP_CPU"),
    ("insufficient cpu with cpuset pod on node", "940-948", 32, False, 32, True, True, 2.0, "INSUFFICIENT_AMP_CPU"),
    ("insufficient cpu when scheduling cpuset pod", "949-957", 32, True, 32, False, True, 2.0, "INSUFFICIENT_AMP_CPU"),
    ("insufficient cpu when scheduling cpuset pod with cpuset pod on node", "958-966", 32, True, 32, True, True, 2.0,
     "INSUFFICIENT_AMP_CPU"),
]
for name, lines, pcpu, pcs, ecpu, ecs, nrt, ratio, want in amp_cases:
    # makePod / makePodOnNode (plugin_test.go:122-139): Prod priority; cpuset pods carry the LSR label and, once on
    # the node, a resource-status cpuset 0..n-1 that the pod event handler records (only with a valid topology)
    pod = {"prod": True}
    if pcpu is not None:
        pod["cpu"] = pcpu * 1000
    if pcs:
        pod["qos"] = "LSR"
    allocs = [{"node": 0, "uid": 0x1E, "cpus": list(range(ecpu)), "numa": []}] if (ecs and nrt) else []
    plugin_cases.append({"kind": "filter", "src": f"{P}:{lines} TestFilterWithAmplifiedCPUs", "name": name,
                         "args": default_args, "nodes": [amp_node(ratio, nrt, ecpu * 1000)], "allocations": allocs,
                         "pod": pod, "filter": True, "want_reason": want})


def affinity_node(policy, count):
    n = numa_node(104, 256, policy, count)   # TestFilterWithNUMANodeScoring (plugin_test.go:1819-1840)
    return n


least = {"type": "LeastAllocated", "resources": {"cpu": 1, "memory": 1}}
mostS = {"type": "MostAllocated", "resources": {"cpu": 1, "memory": 1}}
affinity_cases = [
    ("single numa nodes and select most allocated", "1685-1706", "SingleNUMANode", 2, {0: (4, 8), 1: (40, 8)}, mostS, [1]),
    ("single numa nodes and select least allocated", "1707-1728", "SingleNUMANode", 2, {0: (4, 8), 1: (40, 8)}, least, [0]),
    ("single numa nodes and only one node can be used", "1729-1750", "SingleNUMANode", 2, {0: (4, 8), 1: (52, 8)}, least,
     [0]),
    ("restricted numa nodes and select most allocated and preferred", "1751-1778", "Restricted", 4,
     {0: (24, 8), 1: (23, 8), 2: (4, 8), 3: (8, 8)}, mostS, [3]),
    ("restricted numa nodes and select least allocated and preferred", "1779-1806", "Restricted", 4,
     {0: (24, 8), 1: (23, 8), 2: (4, 8), 3: (8, 8)}, least, [2]),
]
for name, lines, policy, count, existing_pods, nss, want in affinity_cases:
    allocs = [{"node": 0, "uid": 0x100 + z, "cpus": [], "numa": [[z, c * 1000, m * GI]]}
              for z, (c, m) in existing_pods.items()]
    plugin_cases.append({"kind": "affinity", "src": f"{P}:{lines} TestFilterWithNUMANodeScoring", "name": name,
                         "args": {**default_args, "numa_scoring": nss}, "nodes": [affinity_node(policy, count)],
                         "allocations": allocs, "pod": {"cpu": 4000, "memory": 40 * GI}, "filter": True,
                         "want_affinity": want})


def reserve_node(topo, labels=None):
    """TestPlugin_Reserve node (plugin_test.go:1152-1191): allocatable cpu 96, memory 512Gi; options hold only the
    CPUTopology (no NUMANodeResources); allocated CPUs added with CPUExclusivePolicyNone"""
    d = {"cpu_milli": 96000, "memory": 512 * GI, "numa_policy": "", "topology": list(topo), "zones": []}
    d.update(labels or {})
    return d


FULL = {"cpu": 4000, **LSR, "preferred": "FullPCPUs"}
reserve_cases = [
    ("succeed with valid cpu topology", "1048-1059", reserve_node((2, 1, 4, 2)), [], FULL, [0, 1, 2, 3]),
    ("allocated by node cpu bind policy", "1060-1076", reserve_node((2, 1, 4, 2), {"node_cpu_bind": "SpreadByPCPUs"}),
     [], {"cpu": 4000}, [0, 2, 4, 6]),
    ("BE Pod reserves with node cpu bind policy", "1077-1093",
     reserve_node((2, 1, 4, 2), {"node_cpu_bind": "SpreadByPCPUs"}), [], {"batch_cpu": 4000}, []),
    ("succeed with valid cpu topology and node numa least allocate strategy", "1104-1119",
     reserve_node((2, 1, 8, 2), {"numa_allocate_strategy": "LeastAllocated"}), [0, 1, 2, 3], FULL, [16, 17, 18, 19]),
    ("succeed with valid cpu topology and node numa most allocate strategy", "1120-1135",
     reserve_node((2, 1, 8, 2), {"numa_allocate_strategy": "MostAllocated"}), [0, 1, 2, 3], FULL, [4, 5, 6, 7]),
]
for name, lines, node, allocated, pod, want in reserve_cases:
    allocs = [{"node": 0, "uid": 0x77, "cpus": allocated, "numa": []}] if allocated else []
    plugin_cases.append({"kind": "reserve", "src": f"{P}:{lines} TestPlugin_Reserve", "name": name,
                         "args": default_args, "nodes": [node], "allocations": allocs, "pod": pod, "filter": True,
                         "want_cpuset": want})

# ---- resourceManager.Allocate: resource_manager_test.go TestResourceManagerAllocate ----------------------------
R = "resource_manager_test.go"


def rm_node(policy, ratio=-1.0):
    """TestResourceManagerAllocate node (resource_manager_test.go:536-580): allocatable cpu 104 / memory 256Gi,
    CPUTopology (2,1,26,2), NUMANodeResources {cpu 52, memory 128Gi} per NUMA node, the resource manager's default
    NUMA allocate strategy LeastAllocated (written as the node label here), optional amplification ratio. The Go
    test hands Allocate its hint directly; here the node's topology policy makes the topology manager produce it
    (the case's want_affinity asserts it did): SingleNUMANode for the single-node hints, BestEffort for {0,1}."""
    d = {"cpu_milli": 104000, "memory": 256 * GI, "numa_policy": policy, "topology": [2, 1, 26, 2],
         "zones": [[0, 52000, 128 * GI], [1, 52000, 128 * GI]], "numa_allocate_strategy": "LeastAllocated"}
    if ratio > 0:
        d["node_cpu_ratio"] = ratio
    return d


def rm_cpus(text):
    """cpuset.MustParse of the test; CPU 104 lies outside the 104-CPU topology (ids 0..103) and is inert in the
    reference (available = all CPUs minus allocated), so it is dropped"""
    return [c for c in parse(text) if c < 104]


def rm_alloc(cpus, zone_cpu):
    return [{"node": 0, "uid": 0x123456, "cpus": rm_cpus(cpus) if cpus else [],
             "numa": [[z, c * 1000, None] for z, c in enumerate(zone_cpu)]}]


REQ_FULL = {"qos": "LSR", "prod": True, "required": "FullPCPUs", "preferred": "FullPCPUs"}
REQ_SPREAD = {"qos": "LSR", "prod": True, "required": "SpreadByPCPUs", "preferred": "SpreadByPCPUs"}
# (name, lines, node, allocated, pod, want cpuset (None: Allocate fails), want NUMA cpu per zone, want hint)
rm_cases = [
    # the test's pod also requests 10Gi gpu-memory, a resource no NUMA node holds (not in the intersection): it only
    # checks that such a resource is left out; the engine's pods carry no gpu-memory, so it is omitted
    ("allocate with non-existing resources in NUMA", "45-72", rm_node("SingleNUMANode"), [], {"cpu": 4000},
     [], {0: 4000}, [0]),
    ("allocate with insufficient resources", "73-91", rm_node("SingleNUMANode"), [], {"cpu": 54000}, None, None, None),
    ("allocate with required CPUBindPolicyFullPCPUs", "92-122", rm_node("SingleNUMANode"), [],
     {"cpu": 4000, **REQ_FULL}, parse("0-3"), {0: 4000}, [0]),
    ("allocate with required CPUBindPolicyFullPCPUs and allocated", "123-173", rm_node("SingleNUMANode"),
     rm_alloc("4-104", [48, 52]), {"cpu": 4000, **REQ_FULL}, parse("0-3"), {0: 4000}, [0]),
    ("failed to allocate with required CPUBindPolicyFullPCPUs and allocated", "174-214", rm_node("SingleNUMANode"),
     rm_alloc("1,3,5,7-104", [48, 52]), {"cpu": 4000, **REQ_FULL}, None, None, None),
    ("allocate with required CPUBindPolicySpreadByPCPUs", "215-245", rm_node("SingleNUMANode"), [],
     {"cpu": 4000, **REQ_SPREAD}, parse("0,2,4,6"), {0: 4000}, [0]),
    ("allocate with required CPUBindPolicySpreadByPCPUs and allocated", "246-296", rm_node("SingleNUMANode"),
     rm_alloc("1,3,5,7-104", [48, 52]), {"cpu": 4000, **REQ_SPREAD}, parse("0,2,4,6"), {0: 4000}, [0]),
    ("failed to allocate with required CPUBindPolicySpreadByPCPUs and allocated", "297-337",
     rm_node("SingleNUMANode"), rm_alloc("4-104", [48, 52]), {"cpu": 4000, **REQ_SPREAD}, None, None, None),
    # requests = the amplified 6 CPUs, originalRequests = 4: the engine takes the pod's 4 and the node's ratio
    ("allocate with required CPUBindPolicySpreadByPCPUs and amplified requests", "338-374",
     rm_node("SingleNUMANode", 1.5), [], {"cpu": 4000, **REQ_SPREAD}, parse("0,2,4,6"), {0: 4000}, [0]),
    ("allocate with required CPUBindPolicySpreadByPCPUs and allocated and amplified requests", "375-431",
     rm_node("SingleNUMANode", 1.5), rm_alloc("1,3,5,7-104", [48, 52]), {"cpu": 4000, **REQ_SPREAD},
     parse("0,2,4,6"), {0: 4000}, [0]),
    ("failed to allocate with CPU Share and allocated and amplified ratios", "432-477",
     rm_node("SingleNUMANode", 1.5), rm_alloc("0-49,52-101", [50, 50]), {"cpu": 4000}, None, None, None),
    ("allocate by numa hint on mixed cpuset/share node", "478-534", rm_node("BestEffort"),
     rm_alloc("0-43,53-96", [48, 48]), {"cpu": 8000, **REQ_FULL}, parse("44-47,98-101"), {0: 4000, 1: 4000}, [0, 1]),
]
for name, lines, node, allocs, pod, want_cpus, want_numa, want_aff in rm_cases:
    plugin_cases.append({"kind": "allocate", "src": f"{R}:{lines} TestResourceManagerAllocate", "name": name,
                         "args": default_args, "nodes": [node], "allocations": allocs, "pod": pod, "filter": True,
                         "want_placed": want_cpus is not None, "want_cpuset": want_cpus or [],
                         "want_numa_cpu": {str(k): v for k, v in (want_numa or {}).items()},
                         "want_affinity": want_aff})

# ---- resourceManager.GetTopologyHints: resource_manager_test.go TestResourceManagerGetTopologyHint ----------------
# want: resource -> [(NUMA node ids, preferred), ...] in the returned order; [] is an empty (non-nil) list. The last
# case of the table ("failed to generate hints with insufficient memory and hugepages", :906-968) is not transcribed:
# its memory verdict comes from the 1Gi hugepages sharing memory's hint loop, and the engine models no hugepages.
hint_cases = [
    ("allocate with required CPUBindPolicyFullPCPUs", "601-639", [], REQ_FULL, [([0], True), ([1], True), ([0, 1], False)]),
    ("allocate with required CPUBindPolicyFullPCPUs and allocated", "640-691", rm_alloc("4-104", [48, 52]), REQ_FULL,
     [([0], True), ([0, 1], False)]),
    ("failed to allocate with required CPUBindPolicyFullPCPUs and allocated", "692-728",
     rm_alloc("1,3,5,7-104", [48, 52]), REQ_FULL, []),
    ("allocate with required CPUBindPolicySpreadByPCPUs", "729-767", [], REQ_SPREAD, [([0], True), ([1], True), ([0, 1], False)]),
    ("allocate with required CPUBindPolicySpreadByPCPUs and allocated", "768-819", rm_alloc("1,3,5,7-104", [48, 52]),
     REQ_SPREAD, [([0], True), ([0, 1], False)]),
    ("failed to allocate with required CPUBindPolicySpreadByPCPUs and allocated", "820-856",
     rm_alloc("4-104", [48, 52]), REQ_SPREAD, []),
    ("failed to allocate with CPU Share and allocated and amplified ratios", "857-905",
     rm_alloc("0-49,52-101", [50, 50]), {}, [([0, 1], False)]),
]
for name, lines, allocs, pol, want in hint_cases:
    node = rm_node("SingleNUMANode", 1.5 if "amplified" in name else -1.0)
    plugin_cases.append({"kind": "hints", "src": f"{R}:{lines} TestResourceManagerGetTopologyHint", "name": name,
                         "args": default_args, "nodes": [node], "allocations": allocs, "pod": {"cpu": 4000, **pol},
                         "filter": True, "want_hints": {"cpu": [[ids, pref] for ids, pref in want]}})

with open(os.path.join(HERE, "numa_plugin.json"), "w") as f:
    json.dump({"cases": plugin_cases}, f, indent=1)
print(f"wrote {len(plugin_cases)} NodeNUMAResource plugin cases (Filter, affinity, Reserve)")
