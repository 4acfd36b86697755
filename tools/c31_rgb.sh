#!/bin/bash
# RGB conv1 weight gradient with 10 M-tiles per wave (one tap group, 512 splits): parity of the
# variant library, then A/B against the product on the PWYX-RGB line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_rgb10.so timeout -k 10 600 python -u -m pytest -x -v --timeout 200 \
  --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_e2e_gpu.py -k "PWYX or pwyx" \
  > gpurun_out/c31_tests.log 2>&1 && \
VARIANTS="base rgb10" CONFIGS="breakout-pwyx-figar-rgb" N=3 TAG=c31 bash tools/ab_lib.sh
