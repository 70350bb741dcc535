#!/bin/bash
# Round 6: the GroupNorm fold inside the halo conv: parity, end-to-end tests, config D / B sampler A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread -m gpu tests/test_gpu_halo_fold.py \
  tests/test_gpu_latent.py tests/test_gpu_sampler.py tests/test_gpu_blocks.py tests/test_gpu_configs_de.py \
  > gpurun_out/r6n/tests.log 2>&1
rc=$?; grep "halo fold" gpurun_out/r6n/tests.log; tail -3 gpurun_out/r6n/tests.log; [ $rc -eq 0 ] || exit $rc
AB="FMD_TUNE=HALO_FOLD=0 FMD_TUNE=HALO_FOLD=1 FMD_TUNE=HALO_FOLD=0 FMD_TUNE=HALO_FOLD=1" ARGS="--no-config-e" timeout -k 10 1000 bash tools/ab_bench.sh || exit $?
A="FMD_TUNE=HALO_FOLD=1" B="FMD_TUNE=HALO_FOLD=0" timeout -k 10 650 bash tools/ab_prof_latent.sh || exit $?
