#!/bin/bash
# Selected GPU tests (PYTEST_ARGS: test files), then the default bench line (async submission) and the --sync one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${PYTEST_ARGS} -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_q.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_q.log | tail -2
grep -E "FAILED|Error|assert" gpurun_out/pytest_q.log | head -10
[ $rc -eq 0 ] || exit $rc
for mode in "" "--sync"; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $mode ${BENCH_ARGS} \
      > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err
  rc=$?; echo "BENCH $mode rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_q.err; exit $rc; }
  python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_q.json").read().strip().splitlines()[-1])
print("BENCH", round(d["pods_per_s"]), "pods/s", round(d["ms_per_step"], 3), "ms/step", d["breakdown_ms"], "frac", round(d["roofline"]["frac"], 4))
PY
done
