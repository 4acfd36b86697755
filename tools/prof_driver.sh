#!/bin/bash
# rocprofv3 --kernel-trace --stats of the driver's exact bench command (python3 bench.py --gpus 1
# --steps 20 --warmup 5, CPU baseline included), then tools/rocpd_summary.py: the whole-run kernel
# table and the dispatches inside each labelled window of the bench line (`roofline`, `train_pass`,
# ...), so the line's us_per_launch can be read off the profile of the same run.
#   bash tools/prof_driver.sh <name> [extra bench args]   -> gpurun_out/<name>.{log,summary.txt}
set -u
NAME=${1:-prof_driver}
shift || true
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$NAME -o run -- \
  python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 "$@" > $R/gpurun_out/$NAME.log 2>&1
rc=$?
echo "rocprof rc=$rc"
[ $rc -ne 0 ] && exit $rc
db=$(find $R/gpurun_out/$NAME -name '*.db' | head -1)
[ -z "$db" ] && { echo "no rocpd database under gpurun_out/$NAME"; exit 1; }
python3 $R/tools/rocpd_summary.py "$db" --bench $R/gpurun_out/$NAME.log -o $R/gpurun_out/$NAME.summary.txt > /dev/null
rc=$?
echo "summary rc=$rc"
rm -rf $R/gpurun_out/$NAME  # (the summary and the log stay; gpurun copies back <= 64 MiB)
exit $rc
