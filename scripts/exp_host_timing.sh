#!/bin/bash
# Host time per batch (GS_HOST_TIMING=1) on the default bench and the --sync one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "" "--sync"; do
  GS_HOST_TIMING=1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline $v > gpurun_out/ht.json 2> gpurun_out/ht.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/ht.err; exit $rc; }
  python -c "
import json; d=json.loads(open('gpurun_out/ht.json').read().strip().splitlines()[-1])
print('[${v:-default}]', round(d['pods_per_s']), 'pods/s')"
  grep "gpuscore host" gpurun_out/ht.err
done
nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null
