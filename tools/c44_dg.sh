#!/bin/bash
# backward-data chunks of 32 for CIN >= 64: parity (kernels, e2e), then A/B against libmanette_hip_pre6.so
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py > gpurun_out/c44_kern.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py tests/test_e2e_gpu.py > gpurun_out/c44_e2e.log 2>&1 && \
VARIANTS="base pre6" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb breakout-nature-figar" N=2 TAG=c44 bash tools/ab_lib.sh
