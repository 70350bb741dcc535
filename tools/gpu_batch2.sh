#!/bin/bash
# GPU-box helper: 3-D conv checks (parity-class transposed gather), 3-D conv micro A/B vs ./abref, PMC of the 3-D wgrad.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -k "3d or transposed or data_gradient or weight_cache" tests/test_gpu_unet.py -k "unet3d or 3d" -q --timeout 200 --timeout-method thread -rf > gpurun_out/b2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/b2_tests.log; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for tree in . abref; do
    echo "== $tree $r"
    (cd $tree && timeout -k 10 200 python tools/conv3d_micro.py) || exit 1
  done
done
OUT=gpurun_out/pmc3
mkdir -p $OUT
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o run -- \
    python tools/conv3d_micro.py --only wgrad,fwd --iters 3 --warm 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
