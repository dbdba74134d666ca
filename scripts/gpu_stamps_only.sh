#!/bin/bash
# Commit-kernel role stamps (GS_COMMIT_STAMPS=1) on a short bench run, no tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
GS_COMMIT_STAMPS=1 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-extras ${BENCH_ARGS} \
    > gpurun_out/stamps.json 2> gpurun_out/stamps.err
rc=$?
grep -A12 gpuscore gpurun_out/stamps.err
python - <<'PY'
import json
d = json.loads(open("gpurun_out/stamps.json").read().strip().splitlines()[-1])
print(round(d["pods_per_s"]), d["breakdown_ms"])
PY
exit $rc
