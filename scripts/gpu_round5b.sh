#!/bin/bash
# selector micro-changes: parity subset, bench x2 (+ stamps), then the full multi-process C4 / dist suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PYTEST_ARGS="tests/test_gpu_parity.py tests/test_gpu_numa.py tests/test_gpu_cpuset.py tests/test_gpu_fullsize.py::test_c3_bench_config_50k_nodes_replay_parity" \
  AB_ENV="" bash scripts/gpu_iter5.sh || exit $?
timeout -k 10 900 python -u -m pytest tests/test_assign_cache.py tests/test_gpu_async.py tests/test_gpu_c4.py \
    tests/test_gpu_dist.py -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/c4full.log 2>&1
rc=$?; echo "C4 full rc=$rc"; grep -E "^C4|PASSED|FAILED|passed|failed|watchdog" gpurun_out/c4full.log | tail -24
exit $rc
