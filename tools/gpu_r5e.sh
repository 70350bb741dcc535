#!/bin/bash
# GPU-box helper (round 5): 3-D weight-gradient tests + config E goldens, then an interleaved config E A/B of the
# product library against a variant (AB_VARIANT), then a kernel trace of the product's config E step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_e
export TMPDIR=/tmp
V=flow-matching-and-diffusion-models_amd/fmdiff/lib/variants
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q -k "wgrad3d or conv3d or config_e or 3d or golden_e" \
  --timeout 300 --timeout-method thread > gpurun_out/r5e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5e_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in product ${AB_VARIANT}; do
    if [ "$v" = product ]; then lib=""; else lib="FMD_LIB=$V/libfmdiff_$v.so"; fi
    env $lib timeout -k 10 300 python tools/bench3d.py --size 128 --graph --steps 5 --warmup 2 \
      > gpurun_out/r5e_${v}_$r.json 2> gpurun_out/r5e_${v}_$r.err
    rc=$?; echo "$v $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5e_${v}_$r.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o e -- \
  python3 tools/bench3d.py --size 128 --graph --steps 3 --warmup 2 > gpurun_out/prof_e/bench3d.log 2>&1
echo "prof_e rc=$?"
