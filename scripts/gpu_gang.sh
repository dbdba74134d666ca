#!/bin/bash
# Coscheduling throughput (scripts/bench_gang.py) and its kernel trace summary.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/bench_gang.py ${GANG_ARGS} > gpurun_out/gang.json 2> gpurun_out/gang.err
rc=$?; echo "GANG rc=$rc"; cat gpurun_out/gang.json; tail -3 gpurun_out/gang.err
[ $rc -eq 0 ] || exit $rc
if [ -n "$GANG_PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/gangprof -o gang -- python -u scripts/bench_gang.py ${GANG_ARGS} \
      > gpurun_out/gangprof.log 2>&1
  rc=$?; echo "PROF rc=$rc"; find gpurun_out/gangprof -name "*kernel_stats.csv" | head -2
  f=$(find gpurun_out/gangprof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f"
fi
