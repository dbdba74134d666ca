#!/bin/bash
# The round-4 multi-process stall: the same GPU test sequence (one pytest process: assign-cache, async, then the
# 2- and 4-process C4 tests) under each combination of the merged per-batch copies; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=, read -ra combos <<< "${COMBOS:-0 0,1 0,0 1,1 1}"
for combo in "${combos[@]}"; do
  set -- $combo
  log=gpurun_out/c4bisect_up$1_rb$2.log
  GS_MERGE_UP=$1 GS_MERGE_RB=$2 timeout -k 10 300 python -u -m pytest tests/test_assign_cache.py tests/test_gpu_async.py \
      "tests/test_gpu_c4.py::test_c4_sharded_processes_replay_parity[2proc-c2set]" \
      "tests/test_gpu_c4.py::test_c4_sharded_processes_replay_parity[4proc-c2set]" \
      -m gpu -x -v -s --timeout 120 --timeout-method thread > $log 2>&1
  rc=$?
  echo "UP=$1 RB=$2 rc=$rc $(grep -c PASSED $log) passed; $(grep -m1 -o 'schedule wall [0-9.]* s' <(grep 'C4 4 processes' $log))"
  grep "watchdog" $log | head -8
  [ $rc -eq 0 ] || exit $rc
done
