#!/bin/bash
# The multi-process stall's cause, checked: (1) the 1-GPU bench with polling host waits (default) vs HIP's blocking
# synchronisation; (2) the stall sequence with the merged readback (the bisected trigger) and polling waits; (3) the
# full C4 / dist multi-process tests with both merged copies and polling waits; (4) last, the trigger with blocking
# waits again (expected: the watchdog reports the ranks parked in a HIP wait with nothing pending on the device).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB_ENV="GS_WAIT_BLOCKING=1" bash scripts/gpu_iter5.sh || exit $?
COMBOS="0 1" bash scripts/gpu_c4bisect.sh || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_c4.py tests/test_gpu_dist.py -m gpu -x -v -s --timeout 300 \
    --timeout-method thread > gpurun_out/c4full.log 2>&1
rc=$?; echo "C4 full rc=$rc"; grep -E "^C4|PASSED|FAILED|passed|failed|watchdog" gpurun_out/c4full.log | tail -14
[ $rc -eq 0 ] || exit $rc
GS_WAIT_BLOCKING=1 COMBOS="0 1" bash scripts/gpu_c4bisect.sh
