#!/bin/bash
# phase timeline of nips_conv_bwd_kernel (probe build) at the update's 160 rows
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so timeout -k 10 300 python tools/probe_bwd.py --rows 160 \
  > gpurun_out/c22_probe_bwd.txt 2>&1
