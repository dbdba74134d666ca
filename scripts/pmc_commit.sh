#!/bin/bash
# SQ counters of every kernel over a short bench run (one rocprofv3 --pmc pass; no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH} \
    -d "$PWD/gpurun_out/pmc" -o pmc --output-format csv -- python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline \
    > gpurun_out/pmc.log 2>&1
rc=$?; echo "PMC rc=$rc"; tail -3 gpurun_out/pmc.log; find gpurun_out/pmc -name "*.csv" | head
