#!/bin/bash
# Multi-rank checks on one GPU: the sharded tests (threads, processes, C4 at 100k nodes), then the bench flow at
# 1 rank and at 2 processes over gloo (host-callback transport, both on device 0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_numa.py tests/test_gpu_dist.py \
    tests/test_gpu_c4.py -m gpu -x -v -s --timeout 300 --timeout-method thread -k "rank or process or dist or c4" \
    > gpurun_out/t_mr.log 2>&1
rc=$?; grep -E "C4 |passed|failed|Error" gpurun_out/t_mr.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/b1.json 2> gpurun_out/b1.err
rc=$?; [ $rc -eq 0 ] || { tail gpurun_out/b1.err; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --transport gloo --share-gpu --steps 10 --warmup 2 --no-cpu-baseline \
    ${BENCH_ARGS} > gpurun_out/b2.json 2> gpurun_out/b2.err
rc=$?
python - <<'PY'
import json
for f in ("gpurun_out/b1.json", "gpurun_out/b2.json"):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, d["n_gpus"], round(d["pods_per_s"]), d["breakdown_ms"])
    except Exception as e:
        print(f, "no line:", e)
PY
tail -3 gpurun_out/b2.err
exit $rc
