#!/bin/bash
# Extension-path session: merge diagnostic, the extension GPU tests, the C5 bench at 100k nodes + its kernel trace.
# A failing check (rc 1) does not stop the call; a timeout / fault / abort does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -${TAIL:-6} "gpurun_out/$name.log"
  [ $rc -le 1 ] || exit $rc
}
[ -x tools_bin/diag_merge ] && TAIL=20 step diag_merge 60 ./tools_bin/diag_merge
step gpu_tests 700 python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 200 --timeout-method thread
grep -E "FAILED" gpurun_out/gpu_tests.log | head -20
C5_ARGS="--nodes 100000 --steps 3 --warmup 1" bash scripts/gpu_c5.sh
