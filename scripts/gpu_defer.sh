#!/bin/bash
# Deferred host apply: parity / async / cpuset / NUMA / gang tests, then an A/B against GS_DEFER_APPLY=0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_async.py tests/test_gpu_cpuset.py tests/test_gpu_numa.py tests/test_gpu_gang.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_defer.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -3 gpurun_out/pt_defer.log; [ $rc -eq 0 ] || exit $rc
ENVS="- GS_DEFER_APPLY=0 - GS_DEFER_APPLY=0 - GS_DEFER_APPLY=0" bash scripts/exp_env_ab.sh
