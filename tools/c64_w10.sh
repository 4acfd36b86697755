#!/bin/bash
# heads: F > 256 rows with more than 16 outputs (Seaquest's 20) on 10 waves vs 8 (w8)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c64_tests.log 2>&1 || { echo tests rc=$?; exit 1; }
echo tests ok
for v in probe probe_w8; do
  MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so timeout -k 10 300 python tools/probe.py --config seaquest-nature --updates 10 > gpurun_out/c64_${v}_seaquest-nature.txt 2>&1 || { echo probe rc=$?; exit 1; }
done
echo probes ok
VARIANTS="base w8" CONFIGS="seaquest-nature" N=3 TAG=c64 bash tools/ab_lib.sh
