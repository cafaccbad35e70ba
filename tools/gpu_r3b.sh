#!/bin/bash
# r3: parity after the Annex G complex products (+ specials goldens, 3-cycle relabel case)
set -o pipefail
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --workload cfg4 --steps 10 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/bench.json 2> $O/bench.err
