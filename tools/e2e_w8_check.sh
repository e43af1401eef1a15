#!/bin/bash
# knn parity tests, then configs[4] with the 4- and 8-wave DP=256 screen, then a FETCH_SIZE pass (GPU box only)
set -eo pipefail
timeout -k 10 300 python -u -m pytest tests/test_knn_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/knn_tests.log 2>&1
for w in 0 1; do
  NRK_SCREEN_W8=$w timeout -k 10 300 python bench.py --workload e2e --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/e2e_w8_$w.json 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc_e2e -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload e2e --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1
