#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out; export TMPDIR=/tmp
for p in 2 4 8; do
  GS_NUMA_PPT=$p timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ppt$p.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ppt$p.json'));print('PPT $p', round(d['pods_per_s']), 'eval us', round(d['roofline']['kernels']['eval_pass']['avg_launch_us']))"
  GS_NUMA_PPT=$p timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_ppt$p -o p -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
  python3 - <<PY
import csv,glob,collections
f=glob.glob('gpurun_out/pmc_ppt$p/**/*counter_collection.csv',recursive=True)[0]
s=collections.defaultdict(float); n=collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k=r['Kernel_Name']
    if 'eval_numa' in k: s[k]+=float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k in s: print('  ', k[:40], 'FETCH_SIZE KB per launch', round(s[k]/len(n[k])))
PY
done
