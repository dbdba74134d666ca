#!/bin/bash
# Short batches on one stream (direct_batch): C5 at 100k nodes A/B (default, GS_DIRECT_B=0), then the full GPU suite
# and a C3 line (gpu_suite_bench.sh). Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
c5() {   # $1 tag, then env assignments
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --profile c5 --nodes 100000 --steps 3 --warmup 1 --no-cpu-baseline \
      > gpurun_out/direct_c5_$tag.json 2> gpurun_out/direct_c5_$tag.err
  local r=$?; [ $r -eq 0 ] || { echo "C5 $tag rc=$r"; tail -3 gpurun_out/direct_c5_$tag.err; return $r; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C5', sys.argv[2], round(d['pods_per_s']), d['breakdown_ms'])" gpurun_out/direct_c5_$tag.json $tag
}
c5 on GS_X=1 && c5 off GS_DIRECT_B=0 && c5 on2 GS_X=1 && c5 off2 GS_DIRECT_B=0 || exit 1
bash scripts/gpu_suite_bench.sh
