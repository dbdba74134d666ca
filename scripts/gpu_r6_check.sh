#!/bin/bash
# Round 6 iteration: parity + full-size golden tests, commit stamps, then CHECK_BENCH default bench runs (no extras).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py ${CHECK_TESTS:-} -m gpu -x -q \
    --timeout 250 --timeout-method thread > gpurun_out/r6_check_tests.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -2 gpurun_out/r6_check_tests.log; grep -E "^E |FAILED" gpurun_out/r6_check_tests.log | head -8
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_stamps_only.sh 2>&1 | grep -E "fix_levels|^[0-9]" || exit 1
for i in $(seq 1 ${CHECK_BENCH:-2}); do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/r6_check_bench_$i.json 2> gpurun_out/r6_check_bench_$i.err || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/r6_check_bench_$i.json').read().strip().splitlines()[-1])
b=d['breakdown_ms']; print('bench', round(d['pods_per_s']), 'frac', round(d['roofline']['frac'],4), 'commit/batch', round(b['commit']/b['batches'],4), 'cuts', b['cuts'])"
done
