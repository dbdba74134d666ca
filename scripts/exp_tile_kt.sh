#!/bin/bash
# eval_numa tiling variants: kernel durations (rocprofv3 kernel trace) and bench pods/s for GS_NUMA_TILE=1 / 2 / 0
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 2 0; do
  d=gpurun_out/ktt_$v; rm -rf $d
  GS_NUMA_TILE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$d" -o kt --output-format csv -- \
      python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $d.json 2> $d.log
  rc=$?; echo "KT $v rc=$rc"; [ $rc -eq 0 ] || { tail -3 $d.log; exit $rc; }
done
python - <<'PY'
import csv, glob, json
for v in ("1", "2", "0"):
    f = glob.glob(f"gpurun_out/ktt_{v}/**/*kernel_stats.csv", recursive=True)[0]
    d = json.loads(open(f"gpurun_out/ktt_{v}.json").read().strip().splitlines()[-1])
    out = [f"tile={v}", str(round(d["pods_per_s"])), "pods/s"]
    for r in csv.DictReader(open(f)):
        if "eval" in r["Name"] or "commit_spec" in r["Name"]:
            out.append(r["Name"].split("(")[0].replace("void gs::", "") + " " + str(round(float(r["AverageNs"]) / 1e3, 1)))
    print(" | ".join(out))
PY
