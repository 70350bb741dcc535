#!/bin/bash
# GPU-box helper: weight-gradient combine variants (FMD_WGRAD_REDUCE 0/1/2): wgrad tests per variant, then
# train-step A/B.  Stops at the first failing step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in 0 1 2; do
  FMD_WGRAD_REDUCE=$m timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/wred_t$m.log 2>&1
  rc=$?; echo "wgrad tests mode $m rc=$rc $(tail -1 gpurun_out/wred_t$m.log)"; [ $rc -eq 0 ] || exit $rc
done
AB="${AB:-FMD_WGRAD_REDUCE=0 FMD_WGRAD_REDUCE=1 FMD_WGRAD_REDUCE=2 FMD_WGRAD_REDUCE=0 FMD_WGRAD_REDUCE=1 FMD_WGRAD_REDUCE=2}" bash tools/ab_env.sh
