#!/bin/bash
# Full GPU test suite, then a short bench line and the commit-kernel role stamps. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 950 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -10
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err
rc=$?; echo "BENCH rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_q.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_q.json").read().strip().splitlines()[-1])
print("BENCH", round(d["pods_per_s"]), "pods/s", d["breakdown_ms"], "frac", round(d["roofline"]["frac"], 4))
PY
bash scripts/gpu_stamps_only.sh
