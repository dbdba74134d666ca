#!/bin/bash
# Round 6: the multi-rank tests (score-row and level exchanges), then the device-transport rehearsal at 1, 2, 4 ranks
# (score rows) and 2, 4 ranks (levels).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "ranks or transport" tests/test_gpu_dist.py \
    tests/test_gpu_numa.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r6_mr_tests.log 2>&1
rc=$?; echo "PYTEST rc=$rc"; tail -3 gpurun_out/r6_mr_tests.log; grep -E "^E |FAILED" gpurun_out/r6_mr_tests.log | head -8
[ $rc -eq 0 ] || exit $rc
for spec in "1:scores" "2:scores" "4:scores" "2:levels" "4:levels"; do
  n=${spec%%:*}; x=${spec##*:}
  GS_XCHG=$x timeout -k 10 300 python -u scripts/bench_local_ranks.py --ranks $n > gpurun_out/lr_${n}_$x.json 2> gpurun_out/lr_${n}_$x.err
  rc=$?; echo "RANKS $n $x rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/lr_${n}_$x.err; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/lr_${n}_$x.json'))
print(d['ranks'], d['exchange'], round(d['pods_per_s']), 'pods/s', 'same', d['identical_placements_on_every_rank'], d['placements_sha1'], [(p['levels_ms_per_batch'], p['commit_ms_per_batch'], p['eval_ms_per_batch'], p['exchange_ms_per_batch']) for p in d['per_rank']])"
done
