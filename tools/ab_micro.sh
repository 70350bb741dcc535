#!/bin/bash
# GPU-box helper: A/B the conv micro-benchmark between the product library and variant libraries
# in ONE call (same box, same clocks), interleaved twice.  Usage: bash tools/ab_micro.sh B.so [C.so ...]
# (paths relative to flow-matching-and-diffusion-models_amd/fmdiff/lib/); MICRO_ARGS passes through.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBDIR=$PWD/flow-matching-and-diffusion-models_amd/fmdiff/lib
out=gpurun_out/ab.log
: > $out
for round in 1 2; do
  for lib in libfmdiff_hip.so "$@"; do
    echo "== $lib (round $round)" >> $out
    FMD_LIB=$LIBDIR/$lib timeout -k 10 120 python tools/conv_micro.py ${MICRO_ARGS} >> $out 2>&1 || { echo "micro failed for $lib"; exit 1; }
  done
done
grep -v "^/opt" $out
