#!/bin/bash
# direct-conv weight chunks prefetched two ahead: parity of every dconv path, then A/B against HEAD
# (libmanette_hip_base6.so) on the LSTM and PWYX-RGB lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py > gpurun_out/c18_kern.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py tests/test_e2e_gpu.py > gpurun_out/c18_e2e.log 2>&1 && \
VARIANTS="v base6" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c18 bash tools/ab_lib.sh
