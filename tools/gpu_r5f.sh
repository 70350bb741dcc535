#!/bin/bash
# GPU-box helper (round 5): 3-D stride-2 halo tests + config E goldens, then an interleaved config E A/B of the
# default against FMD_TUNE=$AB_TUNE, then a kernel trace of the default config E step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_e
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q -k "s2d or d2s or 3d or config_e or golden_e" \
  --timeout 300 --timeout-method thread > gpurun_out/r5f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5f_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in default alt; do
    if [ "$v" = default ]; then tune=""; else tune="$AB_TUNE"; fi
    FMD_TUNE="$tune" timeout -k 10 300 python tools/bench3d.py --size 128 --graph --steps 5 --warmup 2 \
      > gpurun_out/r5f_${v}_$r.json 2> gpurun_out/r5f_${v}_$r.err
    rc=$?; echo "$v $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5f_${v}_$r.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o e -- \
  python3 tools/bench3d.py --size 128 --graph --steps 3 --warmup 2 > gpurun_out/prof_e/bench3d.log 2>&1
echo "prof_e rc=$?"
