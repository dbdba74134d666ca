#!/bin/bash
# C5 at 100k nodes under a runtime trace (HIP API + kernels + copies), 2 steps: where the host time of the
# one-pod-at-a-time extension path goes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/c5trace
timeout -k 10 400 rocprofv3 --runtime-trace -d "$PWD/gpurun_out/c5trace" -o c5 --output-format csv -- \
    python -u bench.py --profile c5 --nodes 100000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5trace.log 2>&1
rc=$?; echo "TRACE rc=$rc"; tail -2 gpurun_out/c5trace.log; ls gpurun_out/c5trace/*/ 2>/dev/null | head; exit $rc
