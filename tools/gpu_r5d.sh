#!/bin/bash
# GPU-box helper (round 5): linear-backward kernel tests + train-step goldens, train-step A/B against the committed
# misc kernels (variant "oldmisc"), then a kernel-trace of the train step for the per-kernel durations.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_d
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q -k "linear or grouped or train or golden or unet" \
  --timeout 200 --timeout-method thread > gpurun_out/r5d_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5d_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_libs_step.sh product ${AB_VARIANT:-oldmisc} || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_d -o run -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-sampler --no-config-e --no-config-d \
  > gpurun_out/prof_d/bench.json 2> gpurun_out/prof_d/bench.err
echo "prof rc=$?"
