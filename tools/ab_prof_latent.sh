#!/bin/bash
# GPU-box helper: rocprofv3 kernel stats of the config D probe under two env settings.
# usage: A="FMD_TUNE=CONV_GN=1" B="FMD_TUNE=CONV_GN=0" bash tools/ab_prof_latent.sh   -> gpurun_out/abpl_A, gpurun_out/abpl_B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for tag in A B; do
  setting=${!tag}
  mkdir -p gpurun_out/abpl_$tag
  env $setting timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abpl_$tag -o run -- \
    python3 tools/bench_latent.py --reps 2 > gpurun_out/abpl_$tag/bench.json 2> gpurun_out/abpl_$tag/bench.err
  rc=$?; echo "$tag ($setting) prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
