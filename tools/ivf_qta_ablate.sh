#!/bin/bash
# configs[3] IVF: phase A (lane maxima) with one query tile per wave (NRK_IVF_QTA=1,
# default) vs the plan's two (2); phase B keeps two.  Parity first.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ivf_gpu.py > gpurun_out/t_ivf_qta.log 2>&1
NRK_IVF_QTA=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_ivf_gpu.py >> gpurun_out/t_ivf_qta.log 2>&1
timeout -k 10 400 python -u tools/bench_ivf.py NRK_IVF_QTA=1,2 --reps 20 > gpurun_out/ivf_qta.log 2>&1
timeout -k 10 400 python -u tools/bench_ivf.py NRK_IVF_QTA=2,1 --reps 20 >> gpurun_out/ivf_qta.log 2>&1
