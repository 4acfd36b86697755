#!/bin/bash
# NATURE / PWYX dense layer in 8 K-splits: parity, then A/B against the per-row build (pre8)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_learner_gpu.py -k "NATURE or nature or PWYX or pwyx or seaquest or breakout" \
  > gpurun_out/c50_tests.log 2>&1 && \
VARIANTS="base pre8" CONFIGS="seaquest-nature breakout-nature-figar breakout-pwyx-figar-rgb" N=2 TAG=c50 bash tools/ab_lib.sh
