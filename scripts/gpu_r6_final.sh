#!/bin/bash
# Round 6 final measurements: smoke, the default bench line (extras and CPU baseline included), the kernel trace and
# the two PMC passes (scripts/gpu_profile.sh), then the commit stamps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/r6_smoke.log 2>&1
rc=$?; echo "SMOKE rc=$rc"; tail -2 gpurun_out/r6_smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_profile.sh || exit 1
bash scripts/gpu_stamps_only.sh > gpurun_out/r6_stamps_summary.txt 2>&1 || exit 1
tail -3 gpurun_out/r6_stamps_summary.txt
