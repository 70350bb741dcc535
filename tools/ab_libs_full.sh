#!/bin/bash
# interleaved A/B of variant libraries on the train step AND the 50-step sampler: bash ab_libs_full.sh name...
# ("product" = in-tree library)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = product ]; then lib=""; else lib="FMD_LIB=$V/libfmdiff_$v.so"; fi
    env $lib timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-config-e --no-config-d \
      > gpurun_out/abf_${v}_$r.json 2> gpurun_out/abf_${v}_$r.err
    rc=$?
    echo "$v $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abf_${v}_$r.json) $(grep -o '"sampler_ms_per_step": [0-9.]*' gpurun_out/abf_${v}_$r.json)"
    [ $rc -eq 0 ] || exit $rc
  done
done
