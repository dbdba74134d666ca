#!/bin/bash
# One profiling session on the GPU box: the default bench line, a rocprofv3 kernel trace (--stats), and two
# PMC passes (FETCH_SIZE, WRITE_SIZE: they cannot share a pass) over a short bench run. Stops at the first
# failure. Outputs under gpurun_out/ (copy the summaries into profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "BENCH rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o bench --output-format csv -- \
    python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?; echo "PROF rc=$rc"; tail -2 gpurun_out/prof.log
[ $rc -eq 0 ] || exit $rc
for ctr in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_$(echo $ctr | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$PWD/$d" -o pmc --output-format csv -- \
      python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-extras ${BENCH_ARGS:-} > $d.log 2>&1
  rc=$?; echo "PMC $ctr rc=$rc"; tail -2 $d.log
  [ $rc -eq 0 ] || exit $rc
done
find gpurun_out/prof gpurun_out/pmc_* -name "*.csv" | head -20
python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_latest.json
