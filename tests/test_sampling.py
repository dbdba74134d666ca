"""Node sampling ([upstream] kube-scheduler 1.24 schedule_one.go findNodesThatPassFilters / numFeasibleNodesToFind,
SURVEY §8(f) rank 1): the oracle's rotation-window scheduleOne against an independent restatement built from the
oracle's own per-pair verdicts, plus the numFeasibleNodesToFind table. CPU only.

Parity unpinned: the reference holds no test of numFeasibleNodesToFind or nextStartNodeIndex (upstream code, not
vendored); the order is the parallelism-1 rotation order."""
import numpy as np
import pytest

from koordinator_amd import abi, config, synth
from oracle import oracle as orc

# (N, percentageOfNodesToScore, expected numFeasibleNodesToFind) from the upstream formula:
# N < 100 or pct >= 100 -> N; pct <= 0 -> max(5, 50 - N/125) %; result at least 100 nodes.
TABLE = [
    (50, 0, 50), (99, 0, 99), (100, 0, 100), (1000, 0, 420), (5000, 0, 500), (6000, 0, 300),
    (50_000, 0, 2500), (100_000, 0, 5000), (5000, 10, 500), (5000, 1, 100), (5000, 100, 5000),
    (5000, 150, 5000), (250, 0, 120), (20_000, 0, 1000), (3000, 50, 1500),
]


@pytest.mark.parametrize("n,pct,want", TABLE)
def test_num_feasible_nodes_to_find(n, pct, want):
    assert orc.num_feasible_nodes_to_find(n, pct) == want


@pytest.mark.parametrize("n,pct,want", TABLE)
def test_num_feasible_nodes_to_find_library(n, pct, want):
    """The product library's own implementation (a pure host function: no GPU call)."""
    assert abi.load().gs_num_feasible_nodes_to_find(n, pct) == want


def restated_schedule(c, pods, pct, seq):
    """scheduleOne with node sampling, restated over a non-sampling oracle: the verdicts of pod p on the current
    state (or_evaluate), the rotation window, selectHost's reservoir loop, then a replayed placement."""
    cfg = config.make_config(c.num_nodes)
    ref = orc.Oracle(cfg)
    synth.load_into(ref, c)
    N = c.num_nodes
    K = orc.num_feasible_nodes_to_find(N, pct)
    start = 0
    out = []
    for p in range(len(pods)):
        scores, _, _ = ref.evaluate(pods[p:p + 1])
        s = scores[0].astype(np.int64)
        window, diagnosed = [], 0
        for i in range(N):
            n = (start + i) % N
            if s[n] < 0:
                diagnosed += 1
                continue
            if len(window) >= K:
                break
            window.append(n)
        start = (start + len(window) + diagnosed) % N
        if not window:
            out.append((-1, 0, 0, 0))
            ref.schedule_replay(pods[p:p + 1], np.array([-2], np.int32), seq[p:p + 1])
            continue
        sel, best, cnt = window[0], s[window[0]], 1
        for n in window[1:]:
            if s[n] > best:
                sel, best, cnt = n, s[n], 1
            elif s[n] == best:
                cnt += 1
                if orc.tiebreak_intn(cfg.seed, int(seq[p]), cnt) == 0:
                    sel = n
        out.append((sel, int(best), cnt, len(window)))
        ref.schedule_replay(pods[p:p + 1], np.array([sel], np.int32), seq[p:p + 1])
    return out, start


@pytest.mark.parametrize("nodes,npods,pct", [(600, 120, 0), (1500, 80, 0), (1200, 60, 10)])
def test_oracle_sampling_matches_restatement(nodes, npods, pct):
    c = synth.make_cluster(nodes, npods, 4)
    c.pods["requests"][::3, 0] = 60_000     # 60-core pods: many infeasible nodes
    c.pods["requests"][5::17, 0] = 400_000  # 400 cores: FitError (every node processed, nothing assumed)
    c.pods["request_mask"][:] |= 0x1
    seq = np.arange(len(c.pods), dtype=np.uint64)
    want, start = restated_schedule(c, c.pods, pct, seq)
    cfg = config.make_config(c.num_nodes, percentage_of_nodes_to_score=pct)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    got = o.schedule(c.pods, seq)
    for p, (node, score, ties, feas) in enumerate(want):
        assert (got["node"][p], got["feasible"][p]) == (node, feas), f"pod {p}"
        if node >= 0:
            assert (got["score"][p], got["ties"][p]) == (score, ties), f"pod {p}"
    assert o.next_start_node_index == start
    # the window really rotates and really samples
    assert 0 < (got["feasible"] < nodes).sum() and start != 0
    assert (got["node"] < 0).any()
