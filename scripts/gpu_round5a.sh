#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PYTEST_ARGS="${PT:-tests/test_gpu_dist.py tests/test_gpu_ext.py tests/test_gpu_fullsize.py::test_c3_bench_config_50k_nodes_replay_parity}" \
  AB_ENV="GS_SPEC_SOLOAD=1" bash scripts/gpu_iter5.sh && bash scripts/sanitize/gpu_probe.sh run && bash scripts/gpu_c4bisect.sh
