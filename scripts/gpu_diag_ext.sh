#!/bin/bash
# Ext-path NUMA diagnostics + the device merge probe test, then the measurement steps. A step that fails its check
# (rc 1) does not stop the call; a timeout / fault / abort does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -12 "gpurun_out/$name.log"
  [ $rc -le 1 ] || exit $rc
}
step diag100 300 python -u scripts/diag_ext_numa.py 100
step diag40 300 python -u scripts/diag_ext_numa.py 40
step mergeprobe 300 python -u -m pytest tests/test_numa_merge_device.py -m gpu -x -q --timeout 200 --timeout-method thread
