"""World-size-2 CPU tests of the multi-rank protocol over torch.distributed gloo on 127.0.0.1.

The device path needs a GPU; what runs here is the host side of it with the oracle standing in for each rank's
device: (1) the node shard ranges [r*ceil(N/R), (r+1)*ceil(N/R)) and the per-shard selection records
(max feasible score, count of max ties, first tie index in rotation order, feasible count) exchanged with an
all-gather and merged in rank order — the merge must give the single-rank answer; (2) the replicated commit:
every rank runs the same quota-gated schedule on the same inputs and must reach identical verdicts and
placements (no second exchange per batch)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def shard_range(n: int, world: int, rank: int) -> tuple[int, int]:
    per = -(-n // world)
    return min(n, rank * per), min(n, (rank + 1) * per)


def _worker(rank, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        from koordinator_amd import synth
        from koordinator_amd.quota import schedule_with_quota
        from oracle import oracle as orc
        from tests import quota_util as qu

        # (1) per-shard selection records, all-gathered and merged in rank (= rotation) order
        c, cfg = qu.setup(1000, 64, 11)
        o = orc.Oracle(cfg)
        synth.load_into(o, c)
        scores, codes, _ = o.evaluate(c.pods)
        lo, hi = shard_range(c.num_nodes, WORLD, rank)
        feas = codes[:, lo:hi] == 0
        s = np.where(feas, scores[:, lo:hi].astype(np.int64), -1)
        mx = s.max(axis=1)
        first = np.where(mx >= 0, s.argmax(axis=1) + lo, -1)
        ties = np.where(mx >= 0, (s == mx[:, None]).sum(axis=1), 0)
        rec = torch.tensor(np.stack([mx, ties, first, feas.sum(axis=1)], axis=1), dtype=torch.int64)
        allrec = [torch.zeros_like(rec) for _ in range(WORLD)]
        dist.all_gather(allrec, rec)
        allrec = [r.numpy() for r in allrec]
        best = np.full(len(c.pods), -1)
        nties = np.zeros(len(c.pods), np.int64)
        firstg = np.full(len(c.pods), -1)
        nfeas = np.zeros(len(c.pods), np.int64)
        for r in allrec:                                 # rank order = global rotation order
            m, t, f, nf = r[:, 0], r[:, 1], r[:, 2], r[:, 3]
            up = m > best
            eq = (m == best) & (m >= 0)
            firstg = np.where(up, f, firstg)
            nties = np.where(up, t, np.where(eq, nties + t, nties))
            best = np.maximum(best, m)
            nfeas += nf
        fs = np.where(codes == 0, scores.astype(np.int64), -1)
        want_best = fs.max(axis=1)
        assert np.array_equal(best, want_best)
        assert np.array_equal(firstg, np.where(want_best >= 0, fs.argmax(axis=1), -1))
        assert np.array_equal(nties, np.where(want_best >= 0, (fs == want_best[:, None]).sum(axis=1), 0))
        assert np.array_equal(nfeas, (codes == 0).sum(axis=1))

        # (2) replicated commit: identical quota-gated schedules on every rank
        c2, cfg2 = qu.setup(600, 160, 2)
        o2 = orc.Oracle(cfg2)
        synth.load_into(o2, c2)
        p = qu.plugin()
        pq = qu.pod_quotas(c2, p)
        got, st = schedule_with_quota(o2, p, c2.pods, pq, np.arange(len(c2.pods), dtype=np.uint64))
        mine = torch.tensor(np.stack([got["node"].astype(np.int64),
                                      np.array([s.code == "Success" for s in st], np.int64)], axis=1))
        both = [torch.zeros_like(mine) for _ in range(WORLD)]
        dist.all_gather(both, mine)
        assert torch.equal(both[0], both[1])
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # surfaced by the parent
        q.put((rank, repr(e)))
        raise


def test_two_rank_gloo_protocol():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = dict(q.get(timeout=5) for _ in range(WORLD))
    assert res == {0: "ok", 1: "ok"}, res
    assert all(p.exitcode == 0 for p in procs)


@pytest.mark.parametrize("n,world", [(50_000, 8), (100_000, 8), (7, 2), (1, 2), (10, 4)])
def test_shard_ranges_cover_in_order(n, world):
    rs = [shard_range(n, world, r) for r in range(world)]
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
