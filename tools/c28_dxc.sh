#!/bin/bash
# the unpooled 5x5 dX on 8 x 1 waves (one M-tile x both N-tiles): parity, then A/B against the
# 4 x 2 form (libmanette_hip_pre2.so) on the PWYX-RGB and LSTM lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "PWYX or LSTM or loss_backward" > gpurun_out/c28_kern.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py tests/test_e2e_gpu.py -k "lstm or pwyx or LSTM or frames" > gpurun_out/c28_e2e.log 2>&1 && \
VARIANTS="base pre2" CONFIGS="breakout-pwyx-figar-rgb mspacman-lstm-figar" N=2 TAG=c28 bash tools/ab_lib.sh
