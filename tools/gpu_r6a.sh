#!/bin/bash
# Round 6, first GPU call: the rewritten halo-vs-generic statistics test + the in-flight-bucket hazard test, the
# round-5 dgrad_ep failure reproduced on the v10 development tree (abref = fdb9787, built here), and the SQ counter
# passes of the shipped halo forward / data-gradient instances.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6a
ok_or_fail() {   # a test failure (1) is a result; anything else (timeout, abort, fault) ends the call
  local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ] || { echo "step failed rc=$rc"; exit $rc; }
}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "halo_conv_matches_generic or 8_row_tiles or inflight_bucket" tests/test_gpu_exchange_hazard.py \
  > gpurun_out/r6a/tests.log 2>&1
rc=$?; tail -5 gpurun_out/r6a/tests.log; ok_or_fail $rc
if [ -d abref/t_old ]; then
  for v in 1 0; do
    (cd abref && FMD_HALO10=$v timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
       t_old/test_gpu_kernels.py -k "halo_conv_matches_generic" > ../gpurun_out/r6a/v10_repro_$v.log 2>&1)
    rc=$?; tail -3 gpurun_out/r6a/v10_repro_$v.log; ok_or_fail $rc
  done
fi
PMC_ONLY=fwd,dgrad PMC_PASSES="1 2" timeout -k 10 700 bash tools/gpu_pmc.sh > gpurun_out/r6a/pmc.log 2>&1
rc=$?; tail -3 gpurun_out/r6a/pmc.log; [ $rc -eq 0 ] || exit $rc
cp -r gpurun_out/pmc gpurun_out/r6a/pmc_csv
