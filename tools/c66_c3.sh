#!/bin/bash
# heads GEMV: passes of three outputs when a wave has more than two (Seaquest on 8 waves) vs pairs (c2)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c66_tests.log 2>&1 || { echo tests rc=$?; exit 1; }
echo tests ok
for v in probe probe_c2; do
  for c in seaquest-nature pong-nips; do
    MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so timeout -k 10 300 python tools/probe.py --config $c --updates 10 > gpurun_out/c66_${v}_$c.txt 2>&1 || { echo probe rc=$?; exit 1; }
  done
done
echo probes ok
VARIANTS="base c2" CONFIGS="seaquest-nature" N=3 TAG=c66 bash tools/ab_lib.sh
