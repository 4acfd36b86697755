#!/bin/bash
# heads: F > 256 rows on 512 threads (8 waves) vs 256 (nt0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c60_tests.log 2>&1 || { echo tests rc=$?; exit 1; }
echo tests ok
for v in probe probe_nt0; do
  for c in seaquest-nature breakout-nature-figar; do
    MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so timeout -k 10 300 python tools/probe.py --config $c --updates 10 > gpurun_out/c60_${v}_$c.txt 2>&1 || { echo probe rc=$?; exit 1; }
  done
done
echo probes ok
VARIANTS="base nt0" CONFIGS="seaquest-nature breakout-nature-figar" N=3 TAG=c60 bash tools/ab_lib.sh
