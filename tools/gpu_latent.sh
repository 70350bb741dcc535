#!/bin/bash
# GPU-box helper: config D (VAE latent) probe line + a kernel trace of one latent sampling run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_d
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step d timeout -k 10 300 python -u tools/bench_latent.py ${LATENT_ARGS} > gpurun_out/probe_d.json
step dprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_d -o d -- \
  python3 tools/bench_latent.py --reps 1 ${LATENT_ARGS} > gpurun_out/prof_d.log 2>&1
