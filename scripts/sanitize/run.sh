#!/bin/bash
# The repository's CPU code under AddressSanitizer + UndefinedBehaviorSanitizer. CPU only, no GPU.
#   san_host (g++ -fsanitize=address,undefined): the oracle replaying recorded C2 / C3 / C5 workloads (placements
#     must equal the unsanitized oracle's), the device cpuset selection compiled for the host against the host takeCPUs
#     (gsx_cpuset_selftest), the ingest decoders over the reference vectors and their mutations, random quota forests,
#     random Coscheduling event sequences.
#   san_merge (amdclang++ host-only, sanitizers on the host compilation): the two-provider topology merge of the
#     extension path against the oracle's permutation scan on random list sets.
# Any sanitizer report aborts (halt_on_error / -fno-sanitize-recover); the script fails on the first.
set -euo pipefail
cd "$(dirname "$0")"
ROOT=../..
OUT=build
mkdir -p $OUT
CS=$ROOT/koordinator_amd/csrc
J=${JOBS:-8}
SAN="-fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer"
export ASAN_OPTIONS=halt_on_error=1:detect_leaks=1:abort_on_error=0
export UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1

echo "== record workloads (unsanitized oracle: the expected placements)"
python3 record.py $OUT

echo "== build san_host (g++ $SAN)"
objs=()
for src in $ROOT/oracle/oracle.cpp $ROOT/oracle/numa.cpp $CS/gs_numa_host.cpp $CS/gs_ingest.cpp $CS/gs_quota.cpp \
           $CS/gs_gang.cpp $CS/gs_reasons.cpp san_host.cpp; do
  o=$OUT/$(basename $src).o
  g++ -std=c++17 -O1 -g $SAN -ffp-contract=off -pthread -c $src -o $o &
  objs+=($o)
  while [ "$(jobs -r | wc -l)" -ge "$J" ]; do sleep 0.2; done
done
wait
g++ $SAN -pthread -o $OUT/san_host "${objs[@]}"

echo "== build san_merge (amdclang++ host-only)"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
HSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all"
$HIPCC -x hip --offload-host-only -std=c++17 -O1 -g $HSAN -ffp-contract=off -fno-omit-frame-pointer \
    -o $OUT/san_merge san_merge.cpp -x c++ $ROOT/oracle/numa.cpp $ROOT/oracle/oracle.cpp -pthread

echo "== build san_merge_msan (MemorySanitizer: uninitialized reads, which ASan + UBSan do not see; linked without the"
echo "   HIP runtime, whose uninstrumented initialisers MSan would report; both the library's copy form of the merge and"
echo "   the round-4 pointer-select form, GS_MERGE_PTR_SELECT)"
MSAN="-fsanitize=memory -fsanitize-memory-track-origins=2 -fno-sanitize-recover=all"
XMSAN="-Xarch_host -fsanitize=memory -Xarch_host -fsanitize-memory-track-origins=2 -Xarch_host -fno-sanitize-recover=all"
for f in numa oracle; do
  /opt/rocm/llvm/bin/clang++ -std=c++17 -O1 -g $MSAN -ffp-contract=off -fno-omit-frame-pointer -c -o $OUT/${f}_msan.o $ROOT/oracle/$f.cpp
done
for v in copy ptr; do
  D=""; [ $v = ptr ] && D="-DGS_MERGE_PTR_SELECT"
  $HIPCC -x hip --offload-host-only $D -std=c++17 -O1 -g $XMSAN -ffp-contract=off -fno-omit-frame-pointer \
      -c -o $OUT/san_merge_msan_$v.o san_merge.cpp
  /opt/rocm/llvm/bin/clang++ -fsanitize=memory -o $OUT/san_merge_msan_$v $OUT/san_merge_msan_$v.o $OUT/numa_msan.o \
      $OUT/oracle_msan.o -pthread
done
export MSAN_OPTIONS=halt_on_error=1

echo "== run"
for w in c2 c3 c5; do $OUT/san_host replay $OUT/$w.bin "$(cat $OUT/$w.bin.expect)"; done
$OUT/san_host ingest $OUT/ingest.corpus
$OUT/san_host quota 1 3000
$OUT/san_host gang 1 1500
for seed in 1 2 3 4; do $OUT/san_host cpuset $seed 40000; done
for seed in 1 2; do $OUT/san_merge $seed 100000; done
for seed in 1 2; do $OUT/san_merge_msan_copy $seed 100000; done
$OUT/san_merge_msan_ptr 3 100000
echo "SANITIZERS CLEAN"
