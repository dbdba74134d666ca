#!/bin/bash
# A/B of bench arguments: BENCH lines with $AB_A / $AB_B extra arguments, alternated $AB_N times (default 3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in $(seq 1 ${AB_N:-3}); do
  for v in "$AB_A" "$AB_B"; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $v > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/ab.err; exit $rc; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print('[${v:-default}]', round(d['pods_per_s']), 'pods/s', round(d['ms_per_step'],3), 'ms/step', d['breakdown_ms']['commit'])"
  done
done
