#!/bin/bash
# tuning round 2 + a 2-rank RCCL rehearsal on one GPU (two processes share device 0)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 ./tools/tune_transpose 10 > gpurun_out/tune3.log 2>&1; rc=$?; echo "tune rc=$rc"
grep -v verify gpurun_out/tune3.log; grep FAIL gpurun_out/tune3.log
[ $rc -le 1 ] || exit $rc
NCCL_DEBUG=WARN timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --edge 4096 \
    > gpurun_out/bench2.log 2>&1; rc=$?; echo "bench2 rc=$rc"; tail -30 gpurun_out/bench2.log
