#!/bin/bash
# Tiled eval_numa A/B: FETCH_SIZE / WRITE_SIZE per launch of the NUMA eval kernels and the kernel
# durations, tiled (default) and untiled (GS_NUMA_TILE=0), after the NUMA parity tests. Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_numa.py tests/test_gpu_cpuset.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pt_tile.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -2 gpurun_out/pt_tile.log; [ $rc -eq 0 ] || exit $rc
for v in "" "GS_NUMA_TILE=0"; do
  tag=$([ -z "$v" ] && echo tile || echo notile)
  for ctr in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/pmc_${tag}_$(echo $ctr | tr A-Z a-z | cut -d_ -f1)
    rm -rf $d
    env $v timeout -s KILL 240 rocprofv3 --pmc $ctr -d "$PWD/$d" -o pmc --output-format csv -- \
        python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $d.log 2>&1
    rc=$?; echo "PMC $tag $ctr rc=$rc"; [ $rc -eq 0 ] || { tail -3 $d.log; exit $rc; }
  done
  d=gpurun_out/kt_${tag}; rm -rf $d
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/$d" -o kt --output-format csv -- \
      python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $d.log 2>&1
  rc=$?; echo "KT $tag rc=$rc"; [ $rc -eq 0 ] || { tail -3 $d.log; exit $rc; }
done
python - <<'PY'
import csv, glob, collections
for tag in ("tile", "notile"):
    for ctr in ("fetch", "write"):
        f = glob.glob(f"gpurun_out/pmc_{tag}_{ctr}/**/*counter_collection.csv", recursive=True)[0]
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "eval_numa" in k or "gather_numa" in k:
                acc[k.split("(")[0]].append(float(r["Counter_Value"]))
        for k, v in acc.items():
            print(tag, ctr, k, "KiB/launch", round(sum(v) / len(v)), "launches", len(v))
    f = glob.glob(f"gpurun_out/kt_{tag}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "eval" in r["Name"] or "gather" in r["Name"]:
            print(tag, r["Name"][:45], "avg_us", round(float(r["AverageNs"]) / 1e3, 1))
PY
