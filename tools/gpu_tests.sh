#!/bin/bash
# GPU-box helper: all GPU tests + smoke, each step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -rA -s > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?"
