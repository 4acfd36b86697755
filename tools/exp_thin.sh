#!/bin/bash
# Experiment: product library vs the MT_THIN_BM=128 variant (parity subset + benches).
set -u
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_learner_gpu.py -x -q --timeout 300 --timeout-method thread -k "native_step" > gpurun_out/t_learner.log 2>&1; echo "t_learner rc=$?"
MANETTE_HIP_LIB=$R/manette_amd/libmanette_hip_bm128.so timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "backward or forward_parity" > gpurun_out/t_bm128.log 2>&1; echo "t_bm128 rc=$?"
for v in base bm128 base2 bm128b; do
  L=$R/manette_amd/libmanette_hip_bm128.so; case $v in base*) L=$R/manette_amd/libmanette_hip.so;; esac
  for c in pong-nips breakout-nature-figar; do
    MANETTE_HIP_LIB=$L timeout -k 10 300 python bench.py --config $c --steps 60 --no_cpu_baseline > gpurun_out/b_${v}_$c.log 2>&1; echo "b_${v}_$c rc=$?"
  done
done
