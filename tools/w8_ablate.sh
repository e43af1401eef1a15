#!/bin/bash
# configs[4] retrieve (10M x 256, k = 200) and configs[1] after the merge compaction.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_knn_gpu.py tests/test_pipeline.py > gpurun_out/t_w8.log 2>&1
timeout -k 10 300 python -u tools/bench_screen.py --nb 10000000 --d 256 --k 200 --rounds 2 > gpurun_out/w8_ablate.log 2>&1
timeout -k 10 200 python -u tools/bench_screen.py --rounds 3 >> gpurun_out/w8_ablate.log 2>&1
