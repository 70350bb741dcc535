#!/bin/bash
# interleaved config D A/B of the in-tree library against a variant (tools/build_variant.sh NAME) on the GPU box:
#   bash tools/ab_config_d_libs.sh NAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
mkdir -p gpurun_out
for r in 1 2; do for v in product "$1"; do
  if [ "$v" = product ]; then lib=""; else lib="FMD_LIB=$V/libfmdiff_$v.so"; fi
  env $lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config-e --no-sampler \
    > gpurun_out/abd_${v}_$r.json 2> gpurun_out/abd_${v}_$r.err || exit $?
  echo "$v $r $(grep -o '"images_per_sec": [0-9.]*' gpurun_out/abd_${v}_$r.json)"
done; done
