#!/bin/bash
# GPU-box helper: A/B of train-step env switches.  usage: AB="FMD_TUNE=HALO_MIN_WG=32 FMD_TUNE=HALO_MIN_WG=64 ..." bash tools/ab_env.sh
# Runs the wgrad / train-step GPU tests once, then one bench per setting (train only, no CPU baseline).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -k "$AB_TESTS" \
    > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
for setting in $AB; do
  env ${setting//,/ } timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-sampler --no-roofline --no-config-e --no-config-d \
    > gpurun_out/ab_$setting.json 2> gpurun_out/ab_$setting.err
  rc=$?; echo "$setting rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_$setting.json)"; [ $rc -eq 0 ] || exit $rc
done
