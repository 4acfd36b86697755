#!/bin/bash
# rocprofv3 kernel-trace + stats of every bench config (tools/prof.sh each), then the summaries
set -u
TAG=${1:-prof}
for c in ${CONFIGS:-pong-nips breakout-nature-figar seaquest-nature breakout-pwyx-figar-rgb mspacman-lstm-figar}; do
  bash tools/prof.sh ${TAG}_prof_$c --config $c
  rc=$?
  f=$(ls gpurun_out/${TAG}_prof_$c/*/run_kernel_trace.csv gpurun_out/${TAG}_prof_$c/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python tools/prof_summary.py $f > gpurun_out/${TAG}_prof_$c.summary.txt
  # keep the summary and rocprof's own stats, drop the raw trace (gpurun copies back <= 64 MiB)
  find gpurun_out/${TAG}_prof_$c -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_prof_$c.kernel_stats.csv \; 2>/dev/null
  rm -rf gpurun_out/${TAG}_prof_$c
  [ $rc -ne 0 ] && exit $rc
done
exit 0
