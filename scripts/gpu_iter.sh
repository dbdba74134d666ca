#!/bin/bash
# Iteration loop: selected GPU tests (PYTEST_ARGS), the commit-kernel stamps run, one default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PYTEST_ARGS=${PYTEST_ARGS:-"tests/test_gpu_parity.py tests/test_gpu_numa.py tests/test_gpu_cpuset.py"}
timeout -k 10 600 python -u -m pytest ${PYTEST_ARGS} -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_iter.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_iter.log | tail -2
grep -E "FAILED|Error|assert" gpurun_out/pytest_iter.log | head -10
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_stamps_only.sh || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} \
    > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err
rc=$?; echo "BENCH rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_iter.err; exit $rc; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_iter.json").read().strip().splitlines()[-1])
print("BENCH", round(d["pods_per_s"]), "pods/s", round(d["ms_per_step"], 3), "ms/step", d["breakdown_ms"])
PY
