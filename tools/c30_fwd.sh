#!/bin/bash
# the 32 -> 32 direct forward on 8 x 1 waves: parity of every forward / trunk path that runs it, then
# A/B against the 4 x 2 form (libmanette_hip_pre3.so)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "PWYX or LSTM" > gpurun_out/c30_kern.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py tests/test_e2e_gpu.py tests/test_learner_gpu.py -k "lstm or pwyx or LSTM or PWYX or frames" \
  > gpurun_out/c30_e2e.log 2>&1 && \
VARIANTS="base pre3" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c30 bash tools/ab_lib.sh
