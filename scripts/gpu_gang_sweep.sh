#!/bin/bash
# run_cap sweep of the Coscheduling bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rc_ in ${CAPS:-4096 1024 512 256}; do
  timeout -k 10 200 python -u scripts/bench_gang.py --run-cap $rc_ > gpurun_out/gang_$rc_.json 2> gpurun_out/gang_$rc_.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 gpurun_out/gang_$rc_.err; exit $rc; }
  python -c "
import json; d=json.loads(open('gpurun_out/gang_$rc_.json').read())
print('cap $rc_', round(d['pods_per_s']), 'calls', d['engine_calls'], 'engine_s', round(d['engine_s'],3), 'forgets', d['forget_calls'], 'forget_s', round(d['forget_s'],3), 'run mean', round(d['run_pods_mean']), 'total', round(d['total_s'],3))"
done
