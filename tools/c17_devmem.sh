# round-3 call: host -> GPU frame hand-off latency, pinned host vs host-written device memory
# (the device-address attempt last: a host segfault there ends the call)
set -u
OUT=gpurun_out/c17; mkdir -p $OUT
timeout -k 10 60 tools/bin/devmem_probe host 3000 >> $OUT/devmem.log 2>&1; echo "host rc=$?" >> $OUT/devmem.log
timeout -k 10 60 tools/bin/devmem_probe fine 3000 direct >> $OUT/devmem.log 2>&1; echo "fine-direct rc=$?" >> $OUT/devmem.log
