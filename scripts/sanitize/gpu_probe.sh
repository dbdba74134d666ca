#!/bin/bash
# Builds (here, no GPU needed) or runs (on the GPU box) the merge reproducer in both forms.
#   bash scripts/sanitize/gpu_probe.sh build   |   bash scripts/sanitize/gpu_probe.sh run
cd "$(dirname "$0")"
mkdir -p probe_bin
if [ "$1" = build ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DGS_MERGE_PTR_SELECT -o probe_bin/merge_ptr_probe merge_ptr_probe.hip &&
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o probe_bin/merge_copy_probe merge_ptr_probe.hip &&
  for o in 0 1 2; do   # the pointer form at lower optimisation levels (which pass introduces the wrong result)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O$o -std=c++17 -DGS_MERGE_PTR_SELECT -o probe_bin/merge_ptr_probe_O$o \
        merge_ptr_probe.hip || exit 1
  done
else
  timeout -k 10 60 ./probe_bin/merge_ptr_probe 200000 && timeout -k 10 60 ./probe_bin/merge_copy_probe 200000 &&
  for o in 0 1 2; do echo -n "-O$o "; timeout -k 10 120 ./probe_bin/merge_ptr_probe_O$o 200000 | tail -1 || exit 1; done
fi
