#!/bin/bash
# A/B of the commit kernels on the dbg cluster and the quick bench (no tests).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in pipe spec; do
  GS_COMMIT_KERNEL=$k timeout -k 10 200 python -u scripts/dbg_spec.py > gpurun_out/dbg_$k.log 2>&1 || { echo "dbg $k failed"; tail -5 gpurun_out/dbg_$k.log; exit 1; }
  echo "== $k"; grep -E "stats|feasible" gpurun_out/dbg_$k.log | sed -e 's/.eval_pairs.*commit_ms/ commit_ms/' -e 's/, .exchange_ms.*//'
  GS_COMMIT_KERNEL=$k timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$k.json 2> gpurun_out/bench_$k.err || { echo "bench $k failed"; tail -5 gpurun_out/bench_$k.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$k.json'));k=d['roofline']['kernels'];print('$k', round(d['pods_per_s']), 'commit us/pod', round(k['commit_kernel']['us_per_pod'],2), d['breakdown_ms'])"
done
