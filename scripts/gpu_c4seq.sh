#!/bin/bash
# The round-4 hang sequence: GPU tests in one pytest process, then the multi-process C4 tests (watchdog on).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_assign_cache.py tests/test_gpu_async.py tests/test_gpu_c4.py \
    tests/test_gpu_dist.py ${EXTRA_TESTS} -m gpu -v -s --timeout 150 --timeout-method thread > gpurun_out/c4seq5.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed|watchdog|PASSED|FAILED" gpurun_out/c4seq5.log | tail -30
exit $rc
