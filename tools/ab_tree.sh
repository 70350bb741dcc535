#!/bin/bash
# GPU-box helper: interleaved train-step bench of this tree vs a reference tree (default ./abref, a git
# worktree of an older commit with its own built library).  usage: REPS=2 bash tools/ab_tree.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
REF=${REF:-abref}
for r in $(seq 1 ${REPS:-2}); do
  for tree in . $REF; do
    tag=$(basename $(cd $tree && pwd))_$r
    (cd $tree && timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:---no-sampler}) \
      > gpurun_out/abt_$tag.json 2> gpurun_out/abt_$tag.err
    rc=$?; echo "$tree rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"sampler_ms_per_step": [0-9.]*' gpurun_out/abt_$tag.json | tr '\n' ' ')"
    [ $rc -eq 0 ] || exit $rc
  done
done
