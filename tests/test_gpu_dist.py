"""The sharded path across two PROCESSES (one rank each, both on the box's one GPU): every rank evaluates its node
shard, the per-shard candidate levels are all-gathered by torch.distributed (gloo) through the library's
host-callback transport (gs_comm_init_callback), and each rank runs the replicated commit on the merged levels.
Placements must equal the CPU oracle's single-process sequential loop. (RCCL is the production transport of the
same exchange, used by `bench.py --gpus N`; no RCCL run has executed in this pipeline yet, since the driver has not
had an 8-GPU node.) Needs an MI355X: -m gpu."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _cluster(numa: bool):
    from koordinator_amd import synth
    c = synth.make_cluster(3001, 400, 13)
    if numa:
        synth.make_numa(c)
    return c


def _worker(rank: int, port: int, numa: bool, q, skew: str = ""):
    os.environ["GPU_MAX_HW_QUEUES"] = "2"   # ranks sharing the box's one GPU: no hardware-queue oversubscription (test_gpu_c4)
    try:
        if skew:   # GS_DEBUG_XCHG_SKEW: rank:batch skips one exchange sequence number there
            os.environ["GS_DEBUG_XCHG_SKEW"] = skew
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=2)
        from koordinator_amd import abi, config, synth
        from koordinator_amd.engine import Engine
        c = _cluster(numa)
        cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL if numa else abi.GS_ENABLE_LA_FIT)
        e = Engine(cfg)

        def allgather(data: bytes):
            out = [None, None]
            dist.all_gather_object(out, data)
            return out

        e.comm_init_callback(2, rank, allgather)
        synth.load_into(e, c)
        if skew:
            try:
                e.schedule(c.pods[:250])
                q.put((rank, "no error", -2, 0, 0))
            except Exception as ex:
                q.put((rank, str(ex), -3, 0, 0))
            dist.destroy_process_group()
            return
        got = e.schedule(c.pods[:250])
        got2 = e.schedule(c.pods[250:])   # a second call: the replicated mirrors stayed identical
        st = e.stats()
        q.put((rank, np.concatenate([got, got2]).tobytes(), e.mirror_check(), st["shard_begin"], st["shard_end"]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as ex:  # report instead of hanging the parent
        q.put((rank, repr(ex), -1, 0, 0))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("numa", [False, True], ids=["la-fit", "numa"])
def test_two_processes_sharded_schedule_matches_oracle(numa):
    from koordinator_amd import abi, config, synth
    from oracle import oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, numa, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, data, mirror_bad, s0, s1 = q.get(timeout=240)
        assert mirror_bad >= 0, f"rank {r}: {data}"
        res[r] = (np.frombuffer(data, abi.PLACEMENT_DTYPE), mirror_bad, s0, s1)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = _cluster(numa)
    cfg = config.make_config(c.num_nodes, enabled=abi.GS_ENABLE_ALL if numa else abi.GS_ENABLE_LA_FIT)
    o = orc.Oracle(cfg)
    synth.load_into(o, c)
    want = np.concatenate([o.schedule(c.pods[:250], np.arange(250, dtype=np.uint64)),
                           o.schedule(c.pods[250:], np.arange(150, dtype=np.uint64))])
    for r in range(2):
        got, mirror_bad, _, _ = res[r]
        assert mirror_bad == 0, f"rank {r}: HBM mirror diverged"
        for f in ("node", "score", "ties", "feasible"):
            bad = np.nonzero(got[f] != want[f])[0]
            assert not len(bad), f"rank {r}: {f} differs at pod {bad[:5]}"
    assert res[0][3] == res[1][2], "contiguous shards"


def test_exchange_sequence_divergence_fails_on_every_rank():
    """A rank whose exchange sequence diverges (GS_DEBUG_XCHG_SKEW=1:1: rank 1 skips one sequence number at its
    second batch pass) must make EVERY rank fail with GS_ECOMM at that exchange, naming the batch, instead of leaving
    one rank inside a collective the others never enter (the round-4 four-process hang's failure mode)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, True, q, "1:1")) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r, msg, code, _, _ = q.get(timeout=240)
        res[r] = (msg, code)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        msg, code = res[r]
        assert code == -3, f"rank {r}: schedule did not fail ({msg})"
        assert "exchange sequence diverged" in msg and "batch 1" in msg, f"rank {r}: {msg}"
