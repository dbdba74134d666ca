#!/bin/bash
# Round 6: the device-transport rehearsal (scripts/bench_local_ranks.py) over LR_SPECS "ranks:exchange:hwqueues ..."
# (hwqueues: GPU_MAX_HW_QUEUES for the process, '-' the default 4), submission one step ahead unless LR_SYNC=1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${LR_SPECS:-1:scores:- 2:scores:- 2:scores:8 4:scores:-}; do
  IFS=: read n x q <<< "$spec"
  tag=lr_${n}_${x}_q${q}
  extra=""; [ "${LR_SYNC:-0}" = 1 ] && extra="--sync"
  if [ "$q" = "-" ]; then
    GS_XCHG=$x timeout -k 10 300 python -u scripts/bench_local_ranks.py --ranks $n $extra > gpurun_out/$tag.json 2> gpurun_out/$tag.err
  else
    GPU_MAX_HW_QUEUES=$q GS_XCHG=$x timeout -k 10 300 python -u scripts/bench_local_ranks.py --ranks $n $extra > gpurun_out/$tag.json 2> gpurun_out/$tag.err
  fi
  rc=$?; echo "RANKS $spec rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/$tag.err; exit $rc; }
  python -c "
import json; d=json.load(open('gpurun_out/$tag.json'))
print(d['ranks'], d['exchange'], '$q', round(d['pods_per_s']), 'pods/s', 'same', d['identical_placements_on_every_rank'], d['placements_sha1'], [(p['levels_ms_per_batch'], p['commit_ms_per_batch'], p['eval_ms_per_batch'], p['exchange_ms_per_batch']) for p in d['per_rank']])"
done
