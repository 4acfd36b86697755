#!/bin/bash
# LSTM rollout steps with the per-frame x-product sum cache: parity (LSTM kernels, learner, e2e), then
# A/B against the build without it (libmanette_hip_pre4.so)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lstm_gpu.py tests/test_e2e_gpu.py tests/test_learner_gpu.py tests/test_dp_gpu.py -k "lstm or LSTM" \
  > gpurun_out/c39_tests.log 2>&1 && \
VARIANTS="base pre4" CONFIGS="mspacman-lstm-figar" N=3 TAG=c39 bash tools/ab_lib.sh
