#!/bin/bash
# GPU parity tests, then one bench line without the CPU baseline leg.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "PYTEST rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err
rc=$?; echo "BENCH rc=$rc"; cat gpurun_out/bench_quick.json; tail -5 gpurun_out/bench_quick.err
exit $rc
