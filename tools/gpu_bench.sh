#!/bin/bash
# GPU-box helper: bench (1 GPU) then a rocprofv3 kernel-trace summary of a short bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err
echo "bench rc=$?"
