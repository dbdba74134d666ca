#!/bin/bash
# The split selector (GS_SPEC_SPLIT=1): parity tests under it (PYTEST_ARGS), an A/B against the default bench
# (2 alternations), then the commit-kernel stamps of the split variant. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$PYTEST_ARGS" ]; then
  GS_SPEC_SPLIT=${SPLIT_VAL:-1} timeout -k 10 500 python -u -m pytest $PYTEST_ARGS -m gpu -x -v -s --timeout 150 --timeout-method thread \
      > gpurun_out/pytest_split.log 2>&1
  rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_split.log | tail -2
  grep -E "FAILED|Error|assert" gpurun_out/pytest_split.log | head -10
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$NO_STAMPS" ]; then
  GS_SPEC_SPLIT=${SPLIT_VAL:-1} GS_COMMIT_STAMPS=1 timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} \
      > gpurun_out/stamps_split.json 2> gpurun_out/stamps_split.err
  rc=$?; echo "STAMPS rc=$rc"; grep -A20 "gpuscore spec" gpurun_out/stamps_split.err
  [ $rc -eq 0 ] || { tail -5 gpurun_out/stamps_split.err; exit $rc; }
fi
[ -n "$NO_AB" ] && exit 0
for k in 1 2; do
  for v in "" GS_SPEC_SPLIT=${SPLIT_VAL:-1}; do
    env $v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/ab.err; exit $rc; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
b=d['breakdown_ms']
print('${v:-default}', round(d['pods_per_s']), 'pods/s', round(d['ms_per_step'],3), 'ms/step', 'commit/batch', round(b['commit']/b['batches'],3), 'cand/batch', round(b['cand']/b['batches'],3), 'cuts', b.get('cuts'), 'slow', b.get('slowpath_pods'))"
  done
done
