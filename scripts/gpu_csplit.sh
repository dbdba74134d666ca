#!/bin/bash
# Short-batch candidate levels over slices (launch_cand's cs_* kernels) and the split commit's batch threshold:
# parity tests that run short batches, then C5 at 100k nodes A/B (default, GS_CAND_SPLIT=0, GS_SPEC_SPLIT_MINB=0)
# and one C3 line. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ext.py tests/test_gpu_c5.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > gpurun_out/csplit_pytest.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed" gpurun_out/csplit_pytest.log | tail -2
grep -E "FAILED|Error|assert" gpurun_out/csplit_pytest.log | head -10
[ $rc -eq 0 ] || exit $rc
c5() {   # $1 tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --profile c5 --nodes 100000 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/csplit_c5_$tag.json 2> gpurun_out/csplit_c5_$tag.err
  local r=$?; [ $r -eq 0 ] || { echo "C5 $tag rc=$r"; tail -3 gpurun_out/csplit_c5_$tag.err; return $r; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C5', sys.argv[2], round(d['pods_per_s']), d['breakdown_ms'])" gpurun_out/csplit_c5_$tag.json $tag
}
c5 on GS_X=1 && c5 nocand GS_CAND_SPLIT=0 && c5 splitall GS_SPEC_SPLIT_MINB=0 && c5 on2 GS_X=1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/csplit_c3.json 2> gpurun_out/csplit_c3.err
rc=$?; echo "BENCH rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/csplit_c3.err; exit $rc; }
python -c "import json; d=json.loads(open('gpurun_out/csplit_c3.json').read().strip().splitlines()[-1]); print('C3', round(d['pods_per_s']), d['breakdown_ms'])"
