#!/bin/bash
# Headline screen (configs[1]: 1M x 128, 4096 queries, k = 5) under kernel
# variants, interleaved in one process (tools/bench_screen.py).
#   NRK_SCREEN_DEFER  0: epilogue after each MFMA chain; 1: deferred into the next chain
#   NRK_SCREEN_EPI    0 full epilogue, 2 MFMA only (ablation; selects the non-deferred kernel)
set -e
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/bench_screen.py NRK_SCREEN_DEFER=0,1 NRK_SCREEN_EPI=0,2 --rounds 3 \
  > gpurun_out/screen_ablate.log 2>&1
timeout -k 10 200 python -u tools/bench_screen.py NRK_SCREEN_DEFER=0,1 --nb 10000000 --rounds 2 \
  >> gpurun_out/screen_ablate.log 2>&1
timeout -k 10 200 python -u tools/bench_screen.py NRK_SCREEN_DEFER=0,1 --metric l2 --d 64 --k 10 --rounds 2 \
  >> gpurun_out/screen_ablate.log 2>&1
