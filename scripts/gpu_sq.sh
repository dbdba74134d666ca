#!/bin/bash
# SQ instruction / wait counters of the commit kernel (one rocprofv3 --pmc pass per counter group).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/sq1 gpurun_out/sq2
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    --kernel-include-regex "commit" -d "$PWD/gpurun_out/sq1" -o pmc --output-format csv -- \
    python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/sq1.log 2>&1
rc=$?; echo "SQ1 rc=$rc"; tail -2 gpurun_out/sq1.log
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS \
    --kernel-include-regex "commit" -d "$PWD/gpurun_out/sq2" -o pmc --output-format csv -- \
    python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/sq2.log 2>&1
rc=$?; echo "SQ2 rc=$rc"; tail -2 gpurun_out/sq2.log
python scripts/sq_summary.py gpurun_out/sq1 gpurun_out/sq2
