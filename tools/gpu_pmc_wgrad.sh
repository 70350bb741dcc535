#!/bin/bash
# GPU-box helper: PMC counter passes (one rocprofv3 --pmc run per pass) over tools/wgrad_abl.py (config E problem).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmcw
mkdir -p $OUT
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
            "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "WRITE_SIZE"; do
  i=$((i+1))
  case " ${PASSES:-1 2 3 4 5} " in *" $i "*) ;; *) continue ;; esac
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o run -- \
    python tools/wgrad_abl.py --only ${WONLY:-e} --iters 5 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
