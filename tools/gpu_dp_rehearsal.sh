#!/bin/bash
# GPU-box helper: rehearse bench.py's N-rank path on ONE GPU (ranks share the device, gloo carries the
# gradient buckets): split graph captures, overlapped per-bucket all-reduces, 1/world AdamW, max-over-ranks
# timing.  RCCL itself needs one GPU per rank and is exercised only by the driver's multi-GPU runs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FMD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus ${NPROC:-2} --steps 10 --warmup 3 --sampler-steps 10 \
  > gpurun_out/dp_rehearsal.json 2> gpurun_out/dp_rehearsal.err
rc=$?; echo "dp rehearsal rc=$rc"; grep "\[bench\]" gpurun_out/dp_rehearsal.err; exit $rc
