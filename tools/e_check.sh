#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_unet.py -k "unet3d or forward_vs_golden or train_step_gradients" tests/test_gpu_kernels.py -v --timeout 200 --timeout-method thread -rA > gpurun_out/e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/e_tests.log | tail -1; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/bench3d.py --size 128 --steps 3 > gpurun_out/probe_e128.json || exit 1
cat gpurun_out/probe_e128.json | grep -v warmup
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o e -- python3 tools/bench3d.py --size 128 --steps 1 --warmup 1 > gpurun_out/prof_e.log 2>&1
