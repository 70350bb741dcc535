#!/bin/bash
# GPU-box helper: rocprofv3 kernel trace of config E's 128^3 train step (tools/bench3d.py, graph-captured).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_e
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o e -- \
  python3 tools/bench3d.py --size 128 --graph --steps 3 --warmup 2 > gpurun_out/prof_e/bench3d.log 2>&1
echo "prof_e rc=$?"
