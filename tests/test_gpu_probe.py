"""The commit kernel's per-pair evaluations (whole-wave, lane-parallel, one-pod-per-lane) on real mirror rows:
identical totals to gs_evaluate (the eval pass's per-pair Filter + Score, itself bit-exact vs the oracle), and their
cycle cost (s_memtime on the box), printed for DESIGN.md §7. Needs an MI355X: -m gpu."""
import numpy as np
import pytest

from koordinator_amd import abi, config, synth

pytestmark = pytest.mark.gpu

VARIANTS = {
    "c3": ({}, {}),
    "dense": ({"numa_policy_pct": 90, "cpuset_pod_pct": 60}, {}),
    "mixed": ({"mixed": True, "numa_policy_pct": 60, "cpuset_pod_pct": 40}, {}),
    "most_allocated": ({"numa_policy_pct": 60, "cpuset_pod_pct": 40},
                       {"numa": config.numa_args(scoringStrategy={"type": "MostAllocated", "resources": {"cpu": 2, "memory": 1}},
                                                 numaScoringStrategy={"type": "MostAllocated"})}),
    "score_only": ({"numa_policy_pct": 60, "cpuset_pod_pct": 40}, {"score_only": True}),
    "spread": ({"numa_policy_pct": 60, "cpuset_pod_pct": 40}, {"numa": config.numa_args(defaultCPUBindPolicy="SpreadByPCPUs")}),
}


@pytest.mark.parametrize("variant", list(VARIANTS))
def test_pair_probe_matches_evaluate(variant):
    from koordinator_amd.engine import Engine
    nkw, ckw = VARIANTS[variant]
    c = synth.make_cluster(1500, 64, 2)
    synth.make_numa(c, **nkw)
    score_only = ckw.pop("score_only", False)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL, **ckw)
    if score_only:
        cfg.enabled = abi.GS_ENABLE_ALL & ~abi.GS_ENABLE_NUMA_FILTER
    e = Engine(cfg)
    synth.load_into(e, c)
    want, _, _ = e.evaluate(c.pods)                      # [pod, node]
    rng = np.random.default_rng(7)
    nodes = rng.integers(0, c.num_nodes, 512).astype(np.uint32)
    pod_of = rng.integers(0, len(c.pods), 512).astype(np.int32)
    policy = np.array([int(r["numa_topology_policy"]) != 0 for r in c.numa["node_numa"][nodes]])
    s0, cy0, k0 = e.pair_probe(c.pods, nodes, pod_of, 0)
    s2, cy2, k2 = e.pair_probe(c.pods, nodes, pod_of, 2)
    ls = e.last_probe_stamps
    st = np.diff(np.maximum.accumulate(np.where(ls > 0, ls, 0), axis=1), axis=1)   # phases skipped by an early return: 0
    ph = " ".join(f"{float(np.median(st[policy, j])):.0f}/{float(np.median(st[~policy, j])):.0f}" for j in range(7))
    print(f"\n[{variant}] pair_score_wave phases (policy/plain): filters, prelude, setup, divisions, fixups, merge, allocate+select: {ph}")
    ref = want[pod_of, nodes].astype(np.int32)
    assert np.array_equal(s0, ref), f"row_score_wave differs at {np.nonzero(s0 != ref)[0][:5]}"
    bad = np.nonzero(s2 != ref)[0]
    assert not len(bad), f"pair_score_wave differs at probes {bad[:5]}: got {s2[bad[:5]]} want {ref[bad[:5]]}"
    s1, cy1, k1 = e.pair_probe(c.pods, nodes[:128], pod_of[:128], 1)
    assert np.array_equal(s1, want[:, nodes[:128]].T.astype(np.int32)), "row_score (per-lane) differs"

    def med(cy, sel):
        return float(np.median(cy[sel])) if sel.any() else 0.0
    print(f"\n[{variant}] cycles per pair (median) policy/plain rows: row_score_wave {med(cy0, policy):.0f}/"
          f"{med(cy0, ~policy):.0f}  pair_score_wave {med(cy2, policy):.0f}/{med(cy2, ~policy):.0f}  "
          f"one pod per lane x64 {med(cy1, policy[:128]):.0f}/{med(cy1, ~policy[:128]):.0f}  | cold: "
          f"{med(k0, policy):.0f}/{med(k0, ~policy):.0f}  {med(k2, policy):.0f}/{med(k2, ~policy):.0f}  "
          f"{med(k1, policy[:128]):.0f}/{med(k1, ~policy[:128]):.0f}")
