#!/bin/bash
# GPU-box helper: PMC passes over fmd_conv_small on latent shapes (tools/small_abl.py with the product library).
# One rocprofv3 --pmc run per pass, dispatch counters only.  Usage: CASES="s1_2_cat s1_32_cat_skip" bash tools/gpu_pmc_small.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_small
mkdir -p $OUT
CASES=${CASES:-s1_2_cat s1_32_cat_skip}
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
            "SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_MISC" \
            "SQ_IFETCH SQ_IFETCH_LEVEL SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT" \
            "SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_DCACHE_MISSES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $OUT/p$i -o run -- \
    python tools/small_abl.py $CASES > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; continue; }
  echo "pass $i ok"
done
exit 0
