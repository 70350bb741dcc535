#!/bin/bash
# GPU-box helper: kernel-level numerics tests (each step under its own time limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/dev.txt 2>&1
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -rA > gpurun_out/kernels.log 2>&1
echo "kernels rc=$?"
