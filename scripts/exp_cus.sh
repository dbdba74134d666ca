#!/bin/bash
# Commit-chain CU partition sweep (GS_COMMIT_CUS), default bench, 2 rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 1 2; do
  for n in ${CUS_LIST:-0 32 48 64}; do
    GS_COMMIT_CUS=$n timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/cus.json 2> gpurun_out/cus.err
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/cus.err; exit $rc; }
    python -c "
import json; d=json.loads(open('gpurun_out/cus.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']
print('CUS=$n', round(d['pods_per_s']), 'pods/s', round(d['ms_per_step'],3), 'ms/step commit', round(b['commit']/b['batches'],3), 'eval', round(b['eval']/b['batches'],3), 'cand', round(b['cand']/b['batches'],3))"
  done
done
