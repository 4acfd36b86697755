#!/bin/bash
# unpooled 5x5 dX as a persistent direct conv (whole K resident in LDS, next tile's patch loaded under
# the MFMAs): parity, then A/B against HEAD (libmanette_hip_prev.so) on the LSTM and PWYX-RGB lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "PWYX or LSTM or loss_backward" > gpurun_out/c24_kern.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py tests/test_e2e_gpu.py -k "lstm or pwyx or LSTM or frames" > gpurun_out/c24_e2e.log 2>&1 && \
VARIANTS="base prev" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c24 bash tools/ab_lib.sh
