#!/bin/bash
# GPU-box helper: rocprofv3 kernel-trace + stats of a short eager bench run (no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --sampler-steps 5 ${PROF_ARGS} > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err
echo "prof rc=$?"
find gpurun_out/prof -name "*stats*" | head
