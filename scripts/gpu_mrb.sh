#!/bin/bash
# Direct batches read back in one copy: C5 at 100k nodes A/B (default, GS_DIRECT_MERGE_RB=0), then the parity, extension
# and C5 GPU tests. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
c5() {   # $1 tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --profile c5 --nodes 100000 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/mrb_c5_$tag.json 2> gpurun_out/mrb_c5_$tag.err
  local r=$?; [ $r -eq 0 ] || { echo "C5 $tag rc=$r"; tail -3 gpurun_out/mrb_c5_$tag.err; return $r; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C5', sys.argv[2], round(d['pods_per_s']), d['breakdown_ms'])" gpurun_out/mrb_c5_$tag.json $tag
}
c5 on GS_X=1 && c5 off GS_DIRECT_MERGE_RB=0 && c5 on2 GS_X=1 && c5 off2 GS_DIRECT_MERGE_RB=0 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ext.py tests/test_gpu_c5.py tests/test_gpu_quota_gate.py tests/test_gpu_sampling.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/mrb_pytest.log 2>&1; rc=$?; echo PYTEST rc=$rc; tail -2 gpurun_out/mrb_pytest.log; exit $rc
