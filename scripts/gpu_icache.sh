#!/bin/bash
# Instruction-cache and issue counters of the commit kernel, two rocprofv3 --pmc passes (one counter block each).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/ic1 gpurun_out/ic2
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
    --kernel-include-regex "commit" -d "$PWD/gpurun_out/ic1" -o pmc --output-format csv -- \
    python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > gpurun_out/ic1.log 2>&1
rc=$?; echo "IC1 rc=$rc"; tail -2 gpurun_out/ic1.log
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAIT_ANY \
    --kernel-include-regex "commit" -d "$PWD/gpurun_out/ic2" -o pmc --output-format csv -- \
    python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras > gpurun_out/ic2.log 2>&1
rc=$?; echo "IC2 rc=$rc"; tail -2 gpurun_out/ic2.log
[ $rc -eq 0 ] || exit $rc
python scripts/sq_summary.py gpurun_out/ic1; python scripts/sq_summary.py gpurun_out/ic2
