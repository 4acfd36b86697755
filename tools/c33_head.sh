# round-3 last call: smoke, the whole GPU suite and one default bench at HEAD
set -u
OUT=gpurun_out/c33; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
echo "tests rc=$rc" > $OUT/suite.log
case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || exit $?
