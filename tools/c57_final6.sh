#!/bin/bash
# closing check at the last code: smoke, GPU suite, heads chain probes, default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c57_smoke.log 2>&1 || { echo smoke rc=$?; exit 1; }
echo smoke ok
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/c57_tests.log 2>&1 || { echo tests rc=$?; exit 1; }
echo tests ok
for c in seaquest-nature pong-nips; do
  MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so timeout -k 10 300 python tools/probe.py --config $c --updates 10 > gpurun_out/c57_probe_$c.txt 2>&1 || { echo probe rc=$?; exit 1; }
done
echo probes ok
timeout -k 10 600 python bench.py > gpurun_out/c57_bench.log 2>&1 || { echo bench rc=$?; exit 1; }
echo bench ok
