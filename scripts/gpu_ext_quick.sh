#!/bin/bash
# The extension-path GPU tests alone (Reservation + DeviceShare, incl. DeviceShare's NUMA hints).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ext.py tests/test_gpu_c5.py -m gpu -v --timeout 200 \
    --timeout-method thread > gpurun_out/pytest_ext.log 2>&1
rc=$?; echo "PYTEST_EXT rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_ext.log | tail -2
grep -E "FAILED|Error" gpurun_out/pytest_ext.log | head -20
exit $rc
