#!/bin/bash
# GPU-box helper: bench.py legs per env setting (';' joins several assignments in one setting).
# usage: AB="FMD_TUNE=SMALL_CONV=0 FMD_TUNE=SMALL_CONV=1,SMALL_CONV_MAX_HW=64" ARGS="--no-config-e" bash tools/ab_bench.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abb
i=0
for setting in $AB; do
  i=$((i + 1))
  env ${setting//;/ } timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-roofline $ARGS \
    > gpurun_out/abb/$i.json 2> gpurun_out/abb/$i.err
  rc=$?
  echo "$setting rc=$rc $(python3 -c "import json,sys; d=json.load(open('gpurun_out/abb/$i.json')); print('train', round(d['value'],1), 'sampler', round(d.get('sampler_images_per_sec') or 0,2), 'D', round((d.get('config_d') or {}).get('images_per_sec') or 0,1), 'E', round(d.get('config_e_ms_per_step') or 0,1))" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
