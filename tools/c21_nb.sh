#!/bin/bash
# NIPS conv backward: branch-free conv2 dX epilogue (padding column + dropped buffer stores) — parity,
# then A/B against the build without it (libmanette_hip_pre.so) on the Pong line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "NIPS or nips" > gpurun_out/c21_kern.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_e2e_gpu.py -k "pong" > gpurun_out/c21_e2e.log 2>&1 && \
VARIANTS="base pre" CONFIGS="pong-nips" N=3 TAG=c21 bash tools/ab_lib.sh
