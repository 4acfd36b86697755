#!/bin/bash
# the unpooled 64-channel forward (conv4) on 1 x 4 waves: parity, then A/B against the 2 x 4 form
# (libmanette_hip_pre5.so)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "PWYX or LSTM" > gpurun_out/c41_kern.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py tests/test_e2e_gpu.py tests/test_learner_gpu.py -k "lstm or pwyx or LSTM or PWYX or frames" \
  > gpurun_out/c41_e2e.log 2>&1 && \
VARIANTS="base pre5" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c41 bash tools/ab_lib.sh
