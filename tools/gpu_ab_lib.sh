#!/bin/bash
# GPU-box helper: halo kernel tests on the product library, then interleaved conv_micro timings of library
# variants (LIBS: names under fmdiff/lib/variants, "cur" = the product library) and optional ablations (DBG flags
# on the dbg variant).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=$PWD/flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "${TESTK:-halo or conv}" > gpurun_out/ab_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/ab_kernels.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for lib in ${LIBS:-prev cur}; do
    if [ $lib = cur ]; then unset FMD_LIB; else export FMD_LIB=$V/libfmdiff_$lib.so; fi
    timeout -k 10 120 python -u tools/conv_micro.py --only ${ONLY:-fwd,dgrad,cat} --iters 50 > gpurun_out/ab_micro.txt 2>&1
    rc=$?; echo "micro [$lib] rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_micro.txt; [ $rc -eq 0 ] || exit $rc
  done
done
unset FMD_LIB
if [ -n "$DBG" ]; then
  FMD_LIB=$V/libfmdiff_dbg.so timeout -k 10 200 python -u tools/conv_micro.py --only ${ONLY:-fwd,dgrad} --iters 50 --dbg $DBG > gpurun_out/ab_dbg.txt 2>&1
  rc=$?; echo "ablation rc=$rc"; grep -v amdgpu.ids gpurun_out/ab_dbg.txt; [ $rc -eq 0 ] || exit $rc
fi
