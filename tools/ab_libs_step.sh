#!/bin/bash
# interleaved train-step A/B of variant libraries: bash ab_libs_step.sh name...  ("product" = in-tree library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = product ]; then lib=""; else lib="FMD_LIB=$V/libfmdiff_$v.so"; fi
    env $lib timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-sampler --no-config-e --no-config-d \
      > gpurun_out/abl_${v}_$r.json 2> gpurun_out/abl_${v}_$r.err
    rc=$?; echo "$v $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abl_${v}_$r.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
