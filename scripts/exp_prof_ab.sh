#!/bin/bash
# rocprofv3 kernel stats of a short bench with $AB_ENV unset / set: per-kernel average durations side by side.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" "$AB_ENV"; do
  d=gpurun_out/pab_$([ -z "$v" ] && echo a || echo b)
  rm -rf $d
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$d" -o x --output-format csv -- \
      python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $d.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 $d.log; exit $rc; }
  echo "== ${v:-default}"; python - "$d" <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if r["Name"].startswith("__amd"): continue
    print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:8.1f} max_us {float(r["MaxNs"])/1e3:8.1f}')
PY
done
