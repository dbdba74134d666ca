#!/bin/bash
# Commit-kernel phase stamps (diagnostic build path, GS_COMMIT_STAMPS=1) + GPU parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
GS_COMMIT_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/stamps.json 2> gpurun_out/stamps.err
rc=$?; echo "STAMPS rc=$rc"; cat gpurun_out/stamps.json; tail -3 gpurun_out/stamps.err
exit $rc
