#!/bin/bash
# A/B/C of environment settings on the default bench: one BENCH line per variant per alternation.
# AB_VARIANTS: variants separated by '|', each a space-separated list of VAR=value ('-' = defaults); AB_REPS alternations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra VARS <<< "${AB_VARIANTS:--}"
for k in $(seq 1 ${AB_REPS:-2}); do
  for v in "${VARS[@]}"; do
    [ "$v" = "-" ] && v=""
    env $v timeout -k 10 300 python -u bench.py --steps ${AB_STEPS:-20} --warmup 3 --no-cpu-baseline --no-extras ${BENCH_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/ab.err; exit $rc; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
b=d['breakdown_ms']
print('${v:-default}', round(d['pods_per_s']), 'pods/s', round(d['ms_per_step'],3), 'ms/step', 'commit/batch', round(b['commit']/b['batches'],4), 'eval/batch', round(b['eval']/b['batches'],3), 'cand/batch', round(b['cand']/b['batches'],3), 'cuts', b.get('cuts'))" | tee -a gpurun_out/ab_multi.log
  done
done
