#!/bin/bash
# GPU-box helper: config D probe per env setting.  usage: AB="FMD_TUNE=CONV_GN=0 FMD_TUNE=CONV_GN=1" bash tools/ab_latent.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for setting in $AB; do
  i=$((i + 1))
  env ${setting//;/ } timeout -k 10 200 python tools/bench_latent.py ${LATENT_ARGS} > gpurun_out/abl_$i.json 2> gpurun_out/abl_$i.err
  rc=$?; echo "$setting rc=$rc $(grep -o '"images_per_sec": [0-9.]*\|"sample": [0-9.]*' gpurun_out/abl_$i.json | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
