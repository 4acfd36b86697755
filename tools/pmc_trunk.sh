#!/bin/bash
# PMC HBM bytes of the roofline launch alone (tools/trunk_only.py): one rocprofv3 pass per counter
# (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2), each under its own hard limit, then the per-kernel
# summary (tools/pmc_summary.py: gfx950 FETCH_SIZE x2 for 16-B/lane reads).
set -u
NAME=${1:-pmc_trunk}
shift || true
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/$NAME/$C -o run --output-format csv -- \
    python3 $R/tools/trunk_only.py "$@" > $R/gpurun_out/$NAME.$C.log 2>&1
  rc=$?
  echo "pmc $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/$NAME > $R/gpurun_out/$NAME.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${NAME}_trace -o run --output-format csv -- \
  python3 $R/tools/trunk_only.py "$@" > $R/gpurun_out/${NAME}_trace.log 2>&1
rc=$?
echo "trace rc=$rc"
# keep the JSON, the logs and the trace's stats; drop the raw counter / trace files (<= 64 MiB back)
find $R/gpurun_out/${NAME}_trace -name '*kernel_stats.csv' -exec cp {} $R/gpurun_out/${NAME}_trace_stats.csv \; 2>/dev/null
rm -rf $R/gpurun_out/$NAME $R/gpurun_out/${NAME}_trace
exit $rc
