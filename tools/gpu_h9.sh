#!/bin/bash
# GPU-box helper (round 4): halo v9 kernel tests, then interleaved micro timings of the kernel variants
# (FMD_HALO9 = 0 round-3 kernel, 1 v9 first version, 2 v9 pipelined).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${H9_TEST_VARIANTS:-2}; do
  FMD_HALO9=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "halo or conv" > gpurun_out/h9_kernels_$v.log 2>&1
  rc=$?; echo "kernel tests halo9=$v rc=$rc"; tail -2 gpurun_out/h9_kernels_$v.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for arm in ${H9_ARMS:-0 1 2}; do
    FMD_HALO9=$arm timeout -k 10 120 python -u tools/conv_micro.py --only ${H9_ONLY:-fwd,dgrad,cat} --iters 50 ${MICRO_ARGS} > gpurun_out/h9_micro_$arm.txt 2>&1
    rc=$?; echo "micro halo9=$arm rc=$rc"; grep -v amdgpu.ids gpurun_out/h9_micro_$arm.txt; [ $rc -eq 0 ] || exit $rc
  done
done
