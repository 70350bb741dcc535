#!/bin/bash
# GPU-box helper (round 5): split-combine tests -> full bench -> config D probe + latent kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_d
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
step tests timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "split or wgrad or conv_gn" \
  --timeout 200 --timeout-method thread > gpurun_out/r5b_tests.log 2>&1
step bench timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/r5b_bench.json 2> gpurun_out/r5b_bench.err
step d timeout -k 10 300 python -u tools/bench_latent.py > gpurun_out/probe_d.json 2> gpurun_out/probe_d.err
step dprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_d -o d -- \
  python3 tools/bench_latent.py --reps 1 > gpurun_out/prof_d.log 2>&1
