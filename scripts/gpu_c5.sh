#!/bin/bash
# C5 (Reservation + DeviceShare at 100k nodes) on one GPU: the bench line, then a rocprofv3 kernel trace of it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --profile c5 ${C5_ARGS:---steps 3 --warmup 1} > gpurun_out/c5.json 2> gpurun_out/c5.err
rc=$?; echo "C5 rc=$rc"; cat gpurun_out/c5.json; tail -3 gpurun_out/c5.err
[ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PROF:-0}" != 1 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_c5" -o c5 -- \
      python -u bench.py --profile c5 --steps 2 --warmup 1 --no-cpu-baseline ${C5_PROF_ARGS:---nodes 100000} \
      > gpurun_out/prof_c5.log 2>&1
  rc=$?; echo "PROF_C5 rc=$rc"; tail -3 gpurun_out/prof_c5.log
  find gpurun_out/prof_c5 -name "*stats*" | head
fi
