#!/bin/bash
# NIPS dense layer in 8 K-splits (256 blocks at E = 32): parity of every NIPS path, then A/B against
# the 9-split build (libmanette_hip_pre7.so) on the driver's Pong line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c48_smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_learner_gpu.py tests/test_probe_gpu.py tests/test_dp_gpu.py \
  -k "NIPS or nips or pong or Pong or probe or infer or stacking or dp or native or runner" > gpurun_out/c48_tests.log 2>&1 && \
VARIANTS="base pre7" CONFIGS="pong-nips" N=4 TAG=c48 bash tools/ab_lib.sh
