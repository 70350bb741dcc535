#!/bin/bash
# GPU-box helper: halo-conv correctness tests on this tree, then interleaved conv micro-benchmarks and train-step
# benches of this tree vs ./abref (a git worktree of an older commit with its own built library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "halo" tests/test_gpu_unet.py -k "halo or b256 or golden" -v --timeout 200 --timeout-method thread -rA > gpurun_out/abc_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/abc_tests.log | tail -1; [ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for tree in . abref; do
    (cd $tree && timeout -k 10 120 python tools/conv_micro.py --only ${ONLY:-fwd,dgrad,cat,fwd0} --iters 50 --warm ${WARM:-1000}) > gpurun_out/abc_micro_$(basename $(cd $tree && pwd))_$r.txt 2>&1 || exit 1
    echo "== $tree $r"; grep -E "us/call" gpurun_out/abc_micro_$(basename $(cd $tree && pwd))_$r.txt
  done
done
REPS=${REPS:-1} bash tools/ab_tree.sh
