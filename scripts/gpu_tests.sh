#!/bin/bash
# GPU parity tests only (stops at the first failure); log under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${SUITE_TIMEOUT:-500} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20
exit $rc
