#!/bin/bash
# GPU-box helper: rocprofv3 kernel traces of a short train bench under two env settings (this tree).
# usage: A="FMD_TUNE=CONV_GN=1" B="FMD_TUNE=CONV_GN=0" bash tools/ab_prof_env.sh   -> gpurun_out/abpe_A, gpurun_out/abpe_B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for tag in A B; do
  setting=${!tag}
  mkdir -p gpurun_out/abpe_$tag
  env $setting timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abpe_$tag -o run -- \
    python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-sampler > gpurun_out/abpe_$tag/bench.json \
    2> gpurun_out/abpe_$tag/bench.err
  rc=$?; echo "$tag ($setting) prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
