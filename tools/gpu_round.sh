#!/bin/bash
# GPU-box helper: GPU tests -> smoke -> bench (1 GPU) -> rocprofv3 kernel-trace stats.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
# step NAME OUTFILE CMD...: CMD's stdout -> OUTFILE (stderr -> OUTFILE.err); the status line goes to the console
step() { local name=$1 out=$2; shift 2; "$@" > "$out" 2> "$out.err"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
if [ -z "$SKIP_TESTS" ]; then
  # no -x: every GPU test reports (a failing test does not stop the smoke / bench / profile steps)
  timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; [ $rc -le 1 ] || exit $rc
  step smoke gpurun_out/smoke.log timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench gpurun_out/bench.json timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 5}
step prof gpurun_out/prof/bench.json timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
  -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --sampler-steps 5 --no-config-e --no-config-d
find gpurun_out/prof -name "*stats*"
