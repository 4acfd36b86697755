#!/bin/bash
# heads: wave 0 stores only after its last arithmetic; H stored by waves 1-3 (vs st0)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c59_tests.log 2>&1 || { echo tests rc=$?; exit 1; }
echo tests ok
for v in probe probe_st0; do
  for c in seaquest-nature pong-nips; do
    MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so timeout -k 10 300 python tools/probe.py --config $c --updates 10 > gpurun_out/c59_${v}_$c.txt 2>&1 || { echo probe rc=$?; exit 1; }
  done
done
echo probes ok
VARIANTS="base st0" CONFIGS="pong-nips seaquest-nature" N=3 TAG=c59 bash tools/ab_lib.sh
