#!/bin/bash
# GPU-box helper: full GPU test suite, then the train bench (no CPU baseline) and the config D probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -rA ${TEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
step bench timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
grep -o '"ms_per_step": [0-9.]*\|"sampler_ms_per_step": [0-9.]*' gpurun_out/bench.json
step d timeout -k 10 300 python -u tools/bench_latent.py ${LATENT_ARGS} > gpurun_out/probe_d.json
cat gpurun_out/probe_d.json
