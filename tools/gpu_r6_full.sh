#!/bin/bash
# Round 6: the full GPU suite, smoke and the default bench line (as the driver runs them).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6full
timeout -k 10 1000 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r6full/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6full/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6full/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/r6full/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r6full/bench.json 2> gpurun_out/r6full/bench.err; rc=$?; cat gpurun_out/r6full/bench.json; exit $rc
