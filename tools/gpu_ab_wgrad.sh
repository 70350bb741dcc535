#!/bin/bash
# GPU-box helper: weight-gradient kernel tests on the product library, then interleaved tools/wgrad_abl.py timings
# of library variants (LIBS: names under fmdiff/lib/variants, "cur" = the product library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${TESTK:-wgrad}" > gpurun_out/abw_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/abw_kernels.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in ${LIBS:-prev cur}; do
    if [ $lib = cur ]; then unset FMD_LIB; else export FMD_LIB=$V/libfmdiff_$lib.so; fi
    timeout -k 10 200 python -u tools/wgrad_abl.py --iters 20 > gpurun_out/abw.txt 2>&1
    rc=$?; echo "wgrad [$lib] rc=$rc"; grep -v amdgpu.ids gpurun_out/abw.txt; [ $rc -eq 0 ] || exit $rc
  done
done
