#!/bin/bash
# bench.py on every config (no CPU baseline except pong unless CPU_ALL), one log each:
# gpurun_out/${TAG}_<config>.log. A fault-like exit (timeout, abort, segfault) stops the loop.
set -u
TAG=${TAG:-ball}
for c in ${CONFIGS:-pong-nips breakout-nature-figar seaquest-nature breakout-pwyx-figar-rgb mspacman-lstm-figar}; do
  extra="--no_cpu_baseline"; [ "$c" = pong-nips ] && extra=""
  [ -n "${CPU_ALL:-}" ] && extra=""
  timeout -k 10 400 python bench.py --config $c $extra ${ARGS:-} > gpurun_out/${TAG}_$c.log 2>&1
  rc=$?
  echo "$c rc=$rc"
  case $rc in 124|137|134|139) echo "fault-like exit in $c, stopping"; exit $rc;; esac
  sleep 5  # (the previous line's CPU-baseline worker processes finish exiting before the next timed region)
done
