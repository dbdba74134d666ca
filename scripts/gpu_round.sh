#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace. Stops at the first fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { [ "$1" -eq 0 ]; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
  grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20
  ok $rc || exit $rc
fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "BENCH rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o bench -- \
      python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
  rc=$?; echo "PROF rc=$rc"; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
fi
