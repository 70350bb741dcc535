#!/bin/bash
# GPU-box helper: the default bench.py line (roofline and CPU-baseline legs included) per env setting.
# usage: AB="FMD_TUNE=X=0 FMD_TUNE=X=1" bash tools/ab_bench_default.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/abd
i=0
for setting in $AB; do
  i=$((i + 1))
  env ${setting//;/ } timeout -k 10 600 python bench.py > gpurun_out/abd/$i.json 2> gpurun_out/abd/$i.err
  rc=$?
  echo "$setting rc=$rc $(python3 -c "import json; d=json.load(open('gpurun_out/abd/$i.json')); print('train', round(d['value'],1), 'sampler', round(d.get('sampler_images_per_sec') or 0,2), 'D', round((d.get('config_d') or {}).get('images_per_sec') or 0,1), 'E', round(d.get('config_e_ms_per_step') or 0,1))" 2>/dev/null)"
  [ $rc -eq 0 ] || exit $rc
done
