#!/bin/bash
# Side measurements on one GPU (each step under its own time limit, stops at the first failure):
#   gang   — Coscheduling throughput, native gate loop (scripts/bench_gang.py)
#   delta  — incremental snapshot-update throughput at 100k nodes, 1% and 10% of the rows touched per round
#   ranks  — the bench flow at 1 rank and at 2 processes over gloo on the one GPU (a rehearsal of the sharded path)
# STEPS="gang delta ranks" selects them (default: all).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-gang delta ranks}"
run() {   # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.json" 2> "gpurun_out/$name.err"
  local rc=$?
  echo "$name rc=$rc"; tail -1 "gpurun_out/$name.json" | cut -c1-600
  [ $rc -eq 0 ] || { tail -5 "gpurun_out/$name.err"; exit $rc; }
}
for s in $STEPS; do
  case $s in
    gang) run gang_bench 300 python -u scripts/bench_gang.py ;;
    delta)
      run delta_1pct 300 python -u scripts/bench_delta.py --nodes 100000 --frac 0.01
      run delta_10pct 300 python -u scripts/bench_delta.py --nodes 100000 --frac 0.10 ;;
    ranks)
      run b1_gloo 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --sync
      run b2_gloo 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
          --master-port 29511 bench.py --gpus 2 --transport gloo --share-gpu --steps 10 --warmup 2 --no-cpu-baseline ;;
  esac
done
