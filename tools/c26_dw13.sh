#!/bin/bash
# 5x5 32 -> 32 weight gradient with 13 M-tiles per wave (2 tap groups, 256 splits, 8M-float slab cap):
# parity of the variant library, then A/B against the product on the LSTM and PWYX-RGB lines
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_dw13.so timeout -k 10 600 python -u -m pytest -x -v --timeout 200 \
  --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_e2e_gpu.py -k "PWYX or pwyx or lstm or LSTM" \
  > gpurun_out/c26_tests.log 2>&1 && \
VARIANTS="base dw13" CONFIGS="mspacman-lstm-figar breakout-pwyx-figar-rgb" N=2 TAG=c26 bash tools/ab_lib.sh
