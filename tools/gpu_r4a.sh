#!/bin/bash
# GPU-box helper (round 4): halo conv / weight-gradient kernel tests and micro A/B of the conv generations, full GPU
# suite on the defaults, then train-step A/B of kernel generations and weight-gradient slab caps.  Stops at the first
# failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "halo or conv or wgrad" > gpurun_out/r4a_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/r4a_kernels.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for arm in "FMD_HALO9=1" "FMD_HALO9=3"; do
    env $arm timeout -k 10 120 python -u tools/conv_micro.py --only fwd,dgrad,cat,wgrad --iters 50 > gpurun_out/r4a_micro.txt 2>&1
    rc=$?; echo "micro [$arm] rc=$rc"; grep -v amdgpu.ids gpurun_out/r4a_micro.txt; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4a_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4a_tests.log; [ $rc -eq 0 ] || exit $rc
AB="${AB:-FMD_HALO9=0 FMD_HALO9=3 FMD_WGRAD_SLAB_MB=32 FMD_WGRAD_SLAB_MB=16 FMD_HALO9=0 FMD_HALO9=3}" bash tools/ab_env.sh
