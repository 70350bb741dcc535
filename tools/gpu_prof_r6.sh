#!/bin/bash
# GPU-box helper (round 6): rocprofv3 kernel traces of the train step and of the config B sampler on the current tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6p_train gpurun_out/r6p_samp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6p_train -o run -- \
  python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-sampler --no-roofline --no-config-e --no-config-d \
  > gpurun_out/r6p_train/bench.json 2> gpurun_out/r6p_train/bench.err
rc=$?; echo "train prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6p_samp -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-config-e --no-config-d \
  > gpurun_out/r6p_samp/bench.json 2> gpurun_out/r6p_samp/bench.err
rc=$?; echo "sampler prof rc=$rc"; exit $rc
