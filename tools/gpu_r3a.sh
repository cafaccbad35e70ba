#!/bin/bash
# r3 first GPU pass: full -m gpu suite, the system-RCCL test with its log, the bench (N=1),
# the multi-GPU entries rehearsed on one GPU with the new position checks, cfg 5 'T'
set -o pipefail
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 240 python -u -m pytest tests/test_gpu_rccl_system.py -s -v --timeout 200 --timeout-method thread > $O/rccl_system.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python bench.py --extra cfg3,cfg4:32768,cfg5:N --steps 5 --no-cpu-baseline --no-e2e > $O/bench_extra.json 2> $O/bench_extra.err &&
timeout -k 10 200 python bench.py --workload cfg5 --cfg5-op T --steps 10 --no-cpu-baseline > $O/bench_c5T.json 2> $O/bench_c5T.err
