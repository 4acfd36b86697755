#!/bin/bash
# heads: the whole head region requested at kernel start for F > 256 (11 quads per thread) vs 8
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c58_tests.log 2>&1 || { echo tests rc=$?; exit 1; }
echo tests ok
for v in probe probe_kq0; do
  for c in seaquest-nature breakout-nature-figar; do
    MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so timeout -k 10 300 python tools/probe.py --config $c --updates 10 > gpurun_out/c58_${v}_$c.txt 2>&1 || { echo probe rc=$?; exit 1; }
  done
done
echo probes ok
VARIANTS="base kq0" CONFIGS="seaquest-nature" N=3 TAG=c58 bash tools/ab_lib.sh
