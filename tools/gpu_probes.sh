#!/bin/bash
# GPU-box helper: bench.py (config B train + FM / DDPM samplers), config E (3-D, eager and graph-captured) and
# config D (VAE latent) probes, and the config E kernel profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1; shift; "$@"; local rc=$?; echo "$name rc=$rc" >&2; [ $rc -eq 0 ] || exit $rc; }
step bench timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/probe_bench.json 2> gpurun_out/probe_bench.err
step e128g timeout -k 10 300 python -u tools/bench3d.py --size 128 --steps 3 --graph > gpurun_out/probe_e128_graph.json
step e128 timeout -k 10 300 python -u tools/bench3d.py --size 128 --steps 3 > gpurun_out/probe_e128.json
step d timeout -k 10 300 python -u tools/bench_latent.py > gpurun_out/probe_d.json
step eprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_e -o e -- \
  python3 tools/bench3d.py --size 128 --steps 1 --warmup 1 > gpurun_out/prof_e.log 2>&1
