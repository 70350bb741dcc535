#!/bin/bash
# Round 6: fmd_conv_small parts for the LDS plan (config B's 8^2 concat convs): parity, sampler / D A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6o
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_small.py \
  tests/test_gpu_sampler.py > gpurun_out/r6o/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r6o/tests.log; [ $rc -eq 0 ] || exit $rc
AB="FMD_TUNE=SMALL_CONV_MAX_WORK=32768 FMD_TUNE=SMALL_CONV_MAX_WORK=65536 FMD_TUNE=SMALL_CONV_MAX_WORK=32768 FMD_TUNE=SMALL_CONV_MAX_WORK=65536" ARGS="--no-config-e" timeout -k 10 1000 bash tools/ab_bench.sh || exit $?
