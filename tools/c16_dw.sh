#!/bin/bash
# row-mapped 5x5 weight-gradient staging: parity of every path that runs it (PWYX / LSTM backward,
# e2e), then A/B against the item-mapped build (libmanette_hip_r05dw.so) on the LSTM and PWYX-RGB lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "loss_backward or rows_then or fused" > gpurun_out/c16_kern.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py "tests/test_e2e_gpu.py" -k "lstm or pwyx or frames or LSTM" > gpurun_out/c16_e2e.log 2>&1 && \
VARIANTS="base r05dw" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c16 bash tools/ab_lib.sh
