#!/bin/bash
# last-code check: smoke and the driver's default bench line (the GPU suite ran at this code in c62)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c63_smoke.log 2>&1 || { echo smoke rc=$?; exit 1; }
echo smoke ok
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/c63_bench.log 2>&1 || { echo bench rc=$?; exit 1; }
echo bench ok
