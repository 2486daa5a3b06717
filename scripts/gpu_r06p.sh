#!/bin/bash
# Round 6 (p): the driver's N > 1 launch shape rehearsed on the one-GPU box: two ranks (torch.distributed.run, gloo
# barriers) sharing device 0 through PFMPE_BENCH_DEVICE; each rank runs its own C5 stream.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out/r06; export TMPDIR=/tmp
PFMPE_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29617 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r06/dist2_rehearsal.log 2>&1 || { tail -30 gpurun_out/r06/dist2_rehearsal.log; exit 1; }
grep '^{"metric"' gpurun_out/r06/dist2_rehearsal.log | cut -c1-900
