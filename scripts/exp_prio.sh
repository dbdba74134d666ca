#!/bin/bash
# A/B of the commit kernel's role issue priorities (GS_SPEC_PRIO), default bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for pr in ${PRIOS:-0 32 288 16 96 0}; do
  GS_SPEC_PRIO=$pr timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      > gpurun_out/bench_prio.json 2> gpurun_out/bench_prio.err
  rc=$?; [ $rc -eq 0 ] || { echo "prio $pr rc=$rc"; tail -5 gpurun_out/bench_prio.err; exit $rc; }
  PR=$pr python - <<'PY'
import json, os
d = json.loads(open("gpurun_out/bench_prio.json").read().strip().splitlines()[-1])
print("PRIO", os.environ["PR"], round(d["pods_per_s"]), "pods/s", round(d["ms_per_step"], 3), "ms/step commit", round(d["breakdown_ms"]["commit"], 2))
PY
done
