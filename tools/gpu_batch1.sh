#!/bin/bash
# GPU-box helper: 3-D checks + config E profile, then the PMC passes of the halo fwd / dgrad / wgrad kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/e_check.sh || exit $?
PMC_ONLY=fwd,wgrad,dgrad timeout -k 10 800 bash tools/gpu_pmc.sh > gpurun_out/pmc_run.log 2>&1
echo "pmc rc=$?"
