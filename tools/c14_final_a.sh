# r06 final set, part A: PMC traffic of the roofline launches whose kernels changed this round (NIPS
# conv / fc, the row_fc tiles of the E = 32 layered trunks), then the windowed rocprof of the
# driver's exact command
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in pong-nips seaquest-nature breakout-pwyx-figar-rgb; do
  bash tools/pmc_trunk.sh pmc_trunk_$c --config $c --reps 50 > gpurun_out/r06fa_pmc_$c.log 2>&1 || exit 1
done && \
bash tools/prof_driver.sh r06fa_prof_driver > gpurun_out/r06fa_prof_driver.rc 2>&1
