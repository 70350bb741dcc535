#!/bin/bash
# GPU-box helper: PMC counter passes (one rocprofv3 --pmc run per pass, kernel dispatch counters only)
# over tools/conv_micro.py.  Usage: PMC_ONLY=fwd,wgrad bash tools/gpu_pmc.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
mkdir -p $OUT
ONLY=${PMC_ONLY:-fwd,wgrad}
timeout -k 10 120 python tools/conv_micro.py --only $ONLY --iters 20 --variants ${PMC_VARIANTS:-1} > $OUT/plain.txt 2>&1 || exit 1
cat $OUT/plain.txt
PASSES=${PMC_PASSES:-1 2 3 4}
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  case " $PASSES " in *" $i "*) ;; *) continue ;; esac
  timeout -k 10 300 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o run -- \
    python tools/conv_micro.py --only $ONLY --iters 20 --warm 300 --variants ${PMC_VARIANTS:-1} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done
