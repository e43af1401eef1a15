#!/bin/bash
# Deferred IP main pass: 64- vs 128-item tiles on several shapes.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_screen.py NRK_SCREEN_TI=64,128 --rounds 3 > gpurun_out/screen_ablate2.log 2>&1
timeout -k 10 200 python -u tools/bench_screen.py NRK_SCREEN_TI=64,128 --d 64 --k 10 --rounds 3 >> gpurun_out/screen_ablate2.log 2>&1
timeout -k 10 200 python -u tools/bench_screen.py NRK_SCREEN_TI=64,128 --d 32 --k 1 --rounds 3 >> gpurun_out/screen_ablate2.log 2>&1
timeout -k 10 200 python -u tools/bench_screen.py NRK_SCREEN_TI=64,128 --nb 10000000 --rounds 2 >> gpurun_out/screen_ablate2.log 2>&1
