#!/bin/bash
# GPU-box helper (round 5): stride-2 halo weight-gradient tests + goldens, the stride-2 weight-gradient micro timings
# (halo vs FMD_TUNE=WGRAD_S2D=0), then interleaved config B train-step and config E A/Bs of the same switch.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q -k "wgrad or golden or train_step or s2d or 3d" \
  --timeout 300 --timeout-method thread > gpurun_out/r5g_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/wgrad_s2_micro.py > gpurun_out/r5g_micro_halo.txt 2>&1 || exit $?
FMD_TUNE=WGRAD_S2D=0 timeout -k 10 200 python tools/wgrad_s2_micro.py > gpurun_out/r5g_micro_generic.txt 2>&1 || exit $?
paste gpurun_out/r5g_micro_halo.txt gpurun_out/r5g_micro_generic.txt | cut -c1-120
for r in 1 2; do
  for v in default alt; do
    if [ "$v" = default ]; then tune=""; else tune="WGRAD_S2D=0"; fi
    FMD_TUNE="$tune" timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-sampler \
      --no-config-e --no-config-d > gpurun_out/r5g_b_${v}_$r.json 2> gpurun_out/r5g_b_${v}_$r.err
    rc=$?; echo "B $v $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5g_b_${v}_$r.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
for r in 1 2; do
  for v in default alt; do
    if [ "$v" = default ]; then tune=""; else tune="WGRAD_S2D=0"; fi
    FMD_TUNE="$tune" timeout -k 10 300 python tools/bench3d.py --size 128 --graph --steps 5 --warmup 2 \
      > gpurun_out/r5g_e_${v}_$r.json 2> gpurun_out/r5g_e_${v}_$r.err
    rc=$?; echo "E $v $r rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r5g_e_${v}_$r.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
