set -u
OUT=gpurun_out/r04g; mkdir -p $OUT
for c in breakout-nature-figar seaquest-nature; do
  MT_ROLLOUT_AHEAD=1 MANETTE_HIP_LIB=$PWD/manette_amd/libmanette_hip_probe.so timeout -k 10 200 python tools/probe.py --config $c --updates 10 > $OUT/probe_$c.txt 2>&1; rc=$?; echo "probe $c rc=$rc"
  case $rc in 124|137|134|139) exit $rc;; esac
done
