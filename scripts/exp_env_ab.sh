#!/bin/bash
# A/B of environment settings on the default bench line: ENVS="A=1 B=2,C=3" (comma-separated groups; "-" = none).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for grp in ${ENVS:--}; do
  envs=()
  [ "$grp" = "-" ] || IFS=',' read -ra envs <<< "$grp"
  env "${envs[@]}" timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} \
      > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err
  rc=$?; [ $rc -eq 0 ] || { echo "$grp rc=$rc"; tail -5 gpurun_out/bench_ab.err; exit $rc; }
  G="$grp" python - <<'PY'
import json, os
d = json.loads(open("gpurun_out/bench_ab.json").read().strip().splitlines()[-1])
print("AB", os.environ["G"], round(d["pods_per_s"]), "pods/s", round(d["ms_per_step"], 3), "ms/step", {k: round(v, 2) if isinstance(v, float) else v for k, v in d["breakdown_ms"].items()})
PY
done
