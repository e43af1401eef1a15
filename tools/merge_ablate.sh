#!/bin/bash
# configs[1] stage split under pre-pass stride and rescoring-depth (KP) variants.
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/bench_screen.py NRK_PRE_STRIDE=8,16,32 --rounds 3 > gpurun_out/merge_ablate.log 2>&1
timeout -k 10 200 python -u tools/bench_screen.py NRK_PRE_STRIDE=16 NRK_KP=16,32,64,128 --rounds 3 >> gpurun_out/merge_ablate.log 2>&1
[ -f newsrecommend_amd/alt/libnrk.so ] && NRK_LIB=newsrecommend_amd/alt/libnrk.so timeout -k 10 200 python -u tools/bench_screen.py NRK_PRE_STRIDE=16 NRK_KP=16,32,64,128 --rounds 3 >> gpurun_out/merge_ablate.log 2>&1
true
