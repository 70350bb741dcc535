#!/bin/bash
# Round 6: conv_small phase timestamps + config D / config B sampler A/B of the level caps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6m
V=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_gpu_conv_small.py > gpurun_out/r6m/t.log 2>&1 || { tail -30 gpurun_out/r6m/t.log; exit 1; }
FMD_LIB=$V/libfmdiff_ts.so timeout -k 10 300 python tools/small_abl.py s1_32_cat_skip up_16 s1_16_cat_skip_embadd > gpurun_out/r6m/abl.txt 2>&1; rc=$?; cat gpurun_out/r6m/abl.txt; [ $rc -eq 0 ] || exit $rc
AB="FMD_TUNE=SMALL_CONV=1 FMD_TUNE=SMALL_CONV=1,SMALL_CONV_MAX_WORK=131072 FMD_TUNE=SMALL_CONV=1,SMALL_CONV_MAX_WORK=262144,SMALL_CONV_MAX_HW=1024 FMD_TUNE=SMALL_CONV=1" ARGS="--no-config-e" timeout -k 10 1000 bash tools/ab_bench.sh || exit $?
