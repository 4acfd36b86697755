#!/bin/bash
# heads: skip the division by temp when temp == 1 and the repetition softmax when R == 1 (vs sm0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c62_tests.log 2>&1 || { echo tests rc=$?; exit 1; }
echo tests ok
for v in probe probe_sm0; do
  for c in pong-nips seaquest-nature breakout-nature-figar; do
    MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so timeout -k 10 300 python tools/probe.py --config $c --updates 10 > gpurun_out/c62_${v}_$c.txt 2>&1 || { echo probe rc=$?; exit 1; }
  done
done
echo probes ok
VARIANTS="base sm0" CONFIGS="pong-nips" N=3 TAG=c62 bash tools/ab_lib.sh
