#!/bin/bash
# GPU-box helper: GPU tests, then the conv micro-benchmark (each step time-limited, stop at first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${TEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/conv_micro.py > gpurun_out/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; exit $rc
