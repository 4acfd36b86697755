#!/bin/bash
# stride-1 k-state loaders of the generic backward-data GEMM (LdConvBwdA / LdConvBwdB) + the
# direct-conv weight chunks two ahead: parity, then A/B of base (both) / wpf (the chunks only) /
# base6 (HEAD) on the LSTM, PWYX-RGB and Breakout NATURE lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py > gpurun_out/c20_kern.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py tests/test_e2e_gpu.py > gpurun_out/c20_e2e.log 2>&1 && \
VARIANTS="base wpf base6" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb breakout-nature-figar" N=2 TAG=c20 \
  bash tools/ab_lib.sh
