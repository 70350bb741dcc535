#!/bin/bash
# GPU-box helper (round 5): head-kernel tests, then config D A/B of the halo split-K chunk floor.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs_de.py tests/test_gpu_latent.py -x -q \
  -k "head or latent or config_d" --timeout 200 --timeout-method thread > gpurun_out/r5c_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5c_tests.log; [ $rc -eq 0 ] || exit $rc
AB="FMD_TUNE=HALO_MIN_CHUNKS=2 FMD_LIB=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants/libfmdiff_oldhead.so FMD_TUNE=HALO_MIN_CHUNKS=1 FMD_TUNE=HALO_MIN_CHUNKS=2 FMD_LIB=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants/libfmdiff_oldhead.so FMD_TUNE=HALO_MIN_CHUNKS=1" bash tools/ab_latent.sh
