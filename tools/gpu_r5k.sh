#!/bin/bash
# GPU-box helper (round 5): halo-conv tests (8-row tiles on the small grids), then interleaved A/Bs of the default
# against FMD_TUNE=$AB_TUNE: bench.py train step + sampler + config D, then config E (tools/bench3d.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q -k "halo or conv3d or golden or unet or train or latent or config" \
  --timeout 300 --timeout-method thread > gpurun_out/r5k_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5k_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in default alt; do
    if [ "$v" = default ]; then tune=""; else tune="$AB_TUNE"; fi
    FMD_TUNE="$tune" timeout -k 10 400 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-config-e \
      > gpurun_out/r5k_b_${v}_$r.json 2> gpurun_out/r5k_b_${v}_$r.err
    rc=$?
    echo "B $v $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5k_b_${v}_$r.json) $(grep -o '"sampler_ms_per_step": [0-9.]*' gpurun_out/r5k_b_${v}_$r.json) $(grep -o '"images_per_sec": [0-9.]*' gpurun_out/r5k_b_${v}_$r.json)"
    [ $rc -eq 0 ] || exit $rc
  done
done
for v in default alt; do
  if [ "$v" = default ]; then tune=""; else tune="$AB_TUNE"; fi
  FMD_TUNE="$tune" timeout -k 10 300 python tools/bench3d.py --size 128 --graph --steps 5 --warmup 2 \
    > gpurun_out/r5k_e_${v}.json 2> gpurun_out/r5k_e_${v}.err
  rc=$?; echo "E $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5k_e_${v}.json)"; [ $rc -eq 0 ] || exit $rc
done
