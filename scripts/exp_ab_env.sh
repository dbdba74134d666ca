#!/bin/bash
# A/B of an environment switch on the default bench: BENCH lines with $AB_ENV unset / set (3 alternations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 1 2 3; do
  for v in "" "$AB_ENV"; do
    env $v timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/ab.err; exit $rc; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
b=d['breakdown_ms']
print('${v:-default}', round(d['pods_per_s']), 'pods/s', round(d['ms_per_step'],3), 'ms/step', 'commit/batch', round(b['commit']/b['batches'],3), 'eval/batch', round(b['eval']/b['batches'],3), 'cand/batch', round(b['cand']/b['batches'],3))"
  done
done
