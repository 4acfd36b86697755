#!/bin/bash
# heads GEMV: h read once, two outputs per pass, 24-bit lane offsets, biases fetched with the
# operands. GPU suite (product lib), Seaquest / Pong chain probes (new + hb), A/B vs hb.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c56_tests.log 2>&1 || { echo tests rc=$?; exit 1; }
echo tests ok
for v in probe probe_hb; do
  for c in seaquest-nature pong-nips; do
    MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_$v.so timeout -k 10 300 python tools/probe.py --config $c --updates 10 > gpurun_out/c56_${v}_$c.txt 2>&1 || { echo probe rc=$?; exit 1; }
  done
done
echo probes ok
VARIANTS="base hb" CONFIGS="seaquest-nature pong-nips" N=3 TAG=c56 bash tools/ab_lib.sh
