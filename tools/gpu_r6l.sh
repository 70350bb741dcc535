#!/bin/bash
# Round 6: conv_small instances per chunks-per-wave: parity, phases, config D / config B sampler A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6l
V=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_small.py \
  tests/test_gpu_latent.py > gpurun_out/r6l/tests_small.log 2>&1
rc=$?; tail -3 gpurun_out/r6l/tests_small.log; [ $rc -eq 0 ] || exit $rc
FMD_LIB=$V/libfmdiff_ts.so timeout -k 10 300 python tools/small_abl.py > gpurun_out/r6l/abl.txt 2>&1; rc=$?; cat gpurun_out/r6l/abl.txt; [ $rc -eq 0 ] || exit $rc
AB="FMD_TUNE=SMALL_CONV=0 FMD_TUNE=SMALL_CONV=1 FMD_TUNE=SMALL_CONV=1,SMALL_CONV_MAX_HW=256" ARGS="--no-config-e" timeout -k 10 1000 bash tools/ab_bench.sh || exit $?
