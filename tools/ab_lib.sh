#!/bin/bash
# GPU-box helper: interleaved conv micro A/B of the product library vs variant libraries.
#   tools/ab_lib.sh "fwd,dgrad" variantA [variantB ...]   (variants under fmdiff/lib/variants/libfmdiff_<name>.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
only=$1; shift
V=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
for r in 1 2; do
  echo "== product $r"; timeout -k 10 150 python tools/conv_micro.py --iters 30 --only $only || exit 1
  for v in "$@"; do
    echo "== $v $r"; FMD_LIB=$V/libfmdiff_$v.so timeout -k 10 150 python tools/conv_micro.py --iters 30 --only $only || exit 1
  done
done
