# round-3 call: one-round-trip tagged staging vs ready word + frame (tools/devmem_probe.hip)
set -u
OUT=gpurun_out/c21; mkdir -p $OUT
for m in host tagged host tagged; do
  timeout -k 10 60 tools/bin/devmem_probe $m 3000 >> $OUT/devmem.log 2>&1; rc=$?
  echo "$m rc=$rc" >> $OUT/devmem.log
  case $rc in 124|137|134|139) exit $rc;; esac
done
