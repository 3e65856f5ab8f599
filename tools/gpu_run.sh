#!/bin/bash
# One GPU-box session (run by gpurun from the repo root); every step under
# its own time limit, stopping at the first failure.  Output under
# gpurun_out/$TAG.  Steps, each optional:
#   TESTS="tests/x.py tests/y.py"  pytest -m gpu over these (ALL = tests/)
#   SMOKE=1                        __graft_entry__.smoke()
#   BENCH="--steps 20 ..."         bench.py with these args (DEFAULT = none)
#   PROF="--steps 5 ..."           rocprofv3 --kernel-trace --stats of bench.py
#   PY="tools/x.py args"           a python probe
set -o pipefail
TAG=${TAG:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -n "$TESTS" ]; then
  [ "$TESTS" = ALL ] && TESTS=tests
  timeout -k 10 ${TESTS_TIMEOUT:-900} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 \
    --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
  tail -3 $O/gpu_tests.txt
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 \
    || { tail -20 $O/smoke.txt; exit 1; }
  tail -1 $O/smoke.txt
fi
if [ -n "$PY" ]; then
  timeout -k 10 ${PY_TIMEOUT:-600} python -u $PY > $O/py.txt 2> $O/py.err || { tail -20 $O/py.err; exit 1; }
  tail -20 $O/py.txt
fi
if [ -n "$BENCH" ]; then
  [ "$BENCH" = DEFAULT ] && BENCH=""
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py $BENCH --supp-out $O/bench_supplementary.json \
    > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -c 1500 $O/bench.json; wc -c $O/bench.json
fi
if [ -n "$PROF" ]; then
  (cd /tmp && timeout -k 10 ${PROF_TIMEOUT:-600} rocprofv3 --kernel-trace --stats -d $O/prof -o run \
    --output-format csv -- python3 $R/bench.py $PROF --supp-out $O/prof_supp.json \
    > $O/prof_bench.json 2> $O/prof_bench.err) || { tail -20 $O/prof_bench.err; exit 1; }
  echo "prof done"
fi
echo "ALL DONE"
