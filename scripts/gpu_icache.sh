#!/bin/bash
# Instruction-cache counters of the commit kernel (one rocprofv3 --pmc pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/ic1
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
    --kernel-include-regex "commit" -d "$PWD/gpurun_out/ic1" -o pmc --output-format csv -- \
    python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ic1.log 2>&1
rc=$?; echo "IC rc=$rc"; tail -2 gpurun_out/ic1.log
[ $rc -eq 0 ] || exit $rc
python scripts/sq_summary.py gpurun_out/ic1
