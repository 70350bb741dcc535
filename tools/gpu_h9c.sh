#!/bin/bash
# GPU-box helper (round 4): halo kernel tests under FMD_HALO9=$H9C_ARM (default 4 = v9c), then interleaved micro
# timings of FMD_HALO9 arms (H9_ARMS, default "3 4").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
FMD_HALO9=${H9C_ARM:-4} timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "halo or conv" > gpurun_out/h9c_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -2 gpurun_out/h9c_kernels.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for arm in ${H9_ARMS:-3 4}; do
    FMD_HALO9=$arm timeout -k 10 120 python -u tools/conv_micro.py --only ${H9_ONLY:-fwd,dgrad,cat} --iters 50 > gpurun_out/h9c_micro_$arm.txt 2>&1
    rc=$?; echo "micro halo9=$arm rc=$rc"; grep -v amdgpu.ids gpurun_out/h9c_micro_$arm.txt; [ $rc -eq 0 ] || exit $rc
  done
done
