cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
GS_PATCH_TWICE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof2" -o x --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/exp1.log 2>&1; echo rc=$?
