#!/bin/bash
# GPU-box helper (round 4): halo v9 kernel tests, then interleaved micro timings v9 vs the round-3 kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "halo or conv" > gpurun_out/h9_kernels.log 2>&1
rc=$?; echo "kernel tests rc=$rc"; tail -3 gpurun_out/h9_kernels.log; [ $rc -eq 0 ] || exit $rc
for arm in 1 0 1 0; do
  FMD_HALO9=$arm timeout -k 10 120 python -u tools/conv_micro.py --only fwd,dgrad,cat --iters 50 ${MICRO_ARGS} > gpurun_out/h9_micro_$arm.txt 2>&1
  rc=$?; echo "micro halo9=$arm rc=$rc"; cat gpurun_out/h9_micro_$arm.txt; [ $rc -eq 0 ] || exit $rc
done
