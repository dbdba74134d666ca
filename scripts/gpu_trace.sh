#!/bin/bash
# Kernel trace only (rocprofv3 --kernel-trace --stats) of a short default bench run -> gpurun_out/prof.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o bench --output-format csv -- \
    python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?; echo "PROF rc=$rc"; tail -2 gpurun_out/prof.log
exit $rc
