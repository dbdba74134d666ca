#!/bin/bash
# Sharded-flow rehearsal over the device transport: 1, 2 and 4 ranks as threads on the box's GPU (scripts/bench_local_ranks.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in ${RANKS:-1 2 4}; do
  timeout -k 10 300 python -u scripts/bench_local_ranks.py --ranks $n ${LR_ARGS} > gpurun_out/lr_$n.json 2> gpurun_out/lr_$n.err
  rc=$?; echo "RANKS $n rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/lr_$n.err; exit $rc; }
  cat gpurun_out/lr_$n.json
done
