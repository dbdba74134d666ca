"""The oracle's takeCPUs restatement (oracle/numa.cpp) against the reference's own test vectors
(tests/golden/numa_takecpus.json, transcribed from cpu_accumulator_test.go by make_golden_numa.py)."""
import json
import os

import numpy as np
import pytest

from koordinator_amd import abi
from oracle import oracle as orc

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "numa_takecpus.json")))
STRATEGY = {"MostAllocated": 1, "LeastAllocated": 2}


def n_cpus(topo):
    s, n, c, p = topo
    return s * n * c * p


@pytest.mark.parametrize("case", G["takecpus"], ids=lambda c: c["name"].replace(" ", "_"))
def test_take_cpus_golden(case):
    total = n_cpus(case["topology"])
    allocated = set(case["allocated"])
    available = [c for c in range(total) if c not in allocated]
    ref = [0 if c in allocated else -1 for c in range(256)]
    ex = [abi.CPU_EXCLUSIVE[case["alloc_excl"]] if c in allocated else 0 for c in range(256)]
    ok, got = orc.take_cpus_test(case["topology"], case["max_ref"], available, ref, ex, case["needed"],
                                 abi.CPU_BIND[case["bind"]], abi.CPU_EXCLUSIVE[case["excl"]],
                                 STRATEGY[case["strategy"]])
    assert ok != case["want_error"], case["src"]
    assert got == case["want"], f'{case["src"]}: {case["name"]}'


@pytest.mark.parametrize("seq", G["sequences"], ids=lambda s: s["src"].split()[-1])
def test_take_cpus_sequences(seq):
    total = n_cpus(seq["topology"])
    ref = [0] * total        # NodeAllocation refcounts (node_allocation.go addCPUs)
    ex = [0] * total
    for step in seq["steps"]:
        # getAvailableCPUs(topology, maxRefCount=2, {}, {}): allocated = RefCount >= maxRefCount
        available = [c for c in range(total) if ref[c] < seq["max_ref"]]
        aref = [ref[c] if c < total and ref[c] > 0 else -1 for c in range(256)]
        aex = [ex[c] if c < total else 0 for c in range(256)]
        ok, got = orc.take_cpus_test(seq["topology"], seq["max_ref"], available, aref, aex, step["needed"],
                                     abi.CPU_BIND[step["bind"]], 0, 1)
        assert ok and got == step["want"], seq["src"]
        for c in got:
            ref[c] += 1
            ex[c] = abi.CPU_EXCLUSIVE["PCPULevel"]
    if "final_available" in seq:
        assert [c for c in range(total) if ref[c] < seq["max_ref"]] == seq["final_available"]


from tests import numa_util as nu  # noqa: E402

S = nu.load()


@pytest.mark.parametrize("case", S["cases"], ids=lambda c: c["name"].replace(" ", "_"))
def test_numa_score_golden_oracle(case):
    o, pod = nu.build(case, orc.Oracle)
    _, codes, plugin = o.evaluate(np.array([pod], abi.POD_DTYPE))
    assert (codes[0] == 0).all(), f"{case['src']}: filter rejected {codes[0]}"
    assert list(plugin[0, :, abi.GS_PLUGIN_NUMA]) == case["want"], case["src"]
