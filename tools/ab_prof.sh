#!/bin/bash
# GPU-box helper: rocprofv3 kernel traces of a short train bench in this tree and in a reference tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
REF=${REF:-abref}
ROOT=$(pwd)
for tree in . $REF; do
  tag=$(basename $(cd $tree && pwd))
  mkdir -p $ROOT/gpurun_out/abp_$tag
  (cd $tree && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/abp_$tag -o run -- \
    python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-sampler > $ROOT/gpurun_out/abp_$tag/bench.json \
    2> $ROOT/gpurun_out/abp_$tag/bench.err)
  rc=$?; echo "$tree prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
