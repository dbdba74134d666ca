#!/bin/bash
# Round-5 measurement session: PMC passes first (the bench line reads profiles/pmc_latest.json for its traffic field),
# the default bench line (CPU baseline included), a kernel trace (--stats), the commit-kernel stamps, smoke(), and
# the C5 bench at 100k nodes. Each step under its own limit; stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
for ctr in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_$(echo $ctr | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$PWD/$d" -o pmc --output-format csv -- \
      python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $d.log 2>&1
  rc=$?; echo "PMC $ctr rc=$rc"; tail -2 $d.log
  [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_latest.json || exit 1
cp gpurun_out/pmc_latest.json profiles/pmc_latest.json
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "BENCH rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof" -o bench --output-format csv -- \
    python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?; echo "PROF rc=$rc"; tail -2 gpurun_out/prof.log
[ $rc -eq 0 ] || exit $rc
GS_COMMIT_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/stamps.json 2> gpurun_out/stamps.err
rc=$?; echo "STAMPS rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "SMOKE rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --profile c5 --nodes 100000 > gpurun_out/c5.json 2> gpurun_out/c5.err
rc=$?; echo "C5 rc=$rc"; cat gpurun_out/c5.json; [ $rc -eq 0 ] || { tail -3 gpurun_out/c5.err; exit $rc; }
