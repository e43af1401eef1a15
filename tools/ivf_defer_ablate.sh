#!/bin/bash
# configs[3] IVF (10M x 128, nlist 300, nprobe 32, k = 5): deferred-epilogue
# collect / lane-maxima screens (one query tile per wave) vs the direct ones.
#   NRK_IVF_QT     1: one query tile per wave (the deferred variants need it)
#   NRK_IVF_DEFER  1: MODE 3/4 screens with the epilogue deferred into the next MFMA chain
set -e
mkdir -p gpurun_out
NRK_IVF_QT=1 NRK_IVF_DEFER=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ivf_gpu.py > gpurun_out/t_ivf_defer.log 2>&1
timeout -k 10 400 python -u tools/bench_ivf.py NRK_IVF_QT=0,1 NRK_IVF_DEFER=0,1 > gpurun_out/ivf_defer.log 2>&1
