#!/bin/bash
# Round 6: gs_schedule_submit on several ranks — the device-transport tests, then bench.py as 2 gloo processes on the
# box's one GPU (submission one step ahead, the host callback called from the submit worker thread).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "submit_across or device_transport" -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/r6_submit_tests.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -3 gpurun_out/r6_submit_tests.log; grep -E "^E |FAILED" gpurun_out/r6_submit_tests.log | head -8
[ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 4 --warmup 1 --transport gloo --share-gpu --nodes 20000 \
    --no-cpu-baseline > gpurun_out/r6_submit_gloo.log 2>&1
rc=$?; echo "GLOO rc=$rc"; grep -E '^\{' gpurun_out/r6_submit_gloo.log | tail -1 | cut -c1-400; tail -3 gpurun_out/r6_submit_gloo.log
exit $rc
