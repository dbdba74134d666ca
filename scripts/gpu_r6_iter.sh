#!/bin/bash
# Round-6 iteration: targeted GPU tests (PYTEST_ARGS, default the parity / cpuset / NUMA / bench-size files), then
# an A/B of AB_VARIANTS on the default bench (scripts/exp_ab_multi.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest ${PYTEST_ARGS:-tests/test_gpu_parity.py tests/test_gpu_cpuset.py tests/test_gpu_numa.py} \
    -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_iter_tests.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -3 gpurun_out/r6_iter_tests.log
grep -E "FAILED|Error" gpurun_out/r6_iter_tests.log | head -10
[ $rc -eq 0 ] || exit $rc
if [ -n "$AB_VARIANTS" ]; then bash scripts/exp_ab_multi.sh; fi
