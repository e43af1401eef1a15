#!/bin/bash
# configs[4] retrieve (10M x 256, k = 200): deferred 8-wave screen + pre-pass vs direct; then the e2e bench.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_knn_gpu.py -k "256" > gpurun_out/t_w8.log 2>&1
timeout -k 10 300 python -u tools/bench_screen.py NRK_SCREEN_W8_DEFER=0,1 --nb 10000000 --d 256 --k 200 --rounds 2 > gpurun_out/w8_ablate.log 2>&1
timeout -k 10 300 python -u bench.py --workload e2e --no-cpu-baseline > gpurun_out/e2e.json 2> gpurun_out/e2e.err
