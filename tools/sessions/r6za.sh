#!/bin/bash
# r6 final check (re-run after the GPU group builder, the 16-group chunks, the pieces in the
# group launch and the skew ops in groups), part a: tools/gpu_full.sh without its cfg 3 / 4 / 5 PMC tails (-m gpu, smoke,
# bench N = 1, cfg 5 'N' / 'T' lines, rocprofv3 kernel trace of the bench and its FETCH_SIZE /
# WRITE_SIZE passes) -> profiles/r6z (tools/save_full.py)
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op N --steps 10 --no-cpu-baseline > $O/c5N.json 2> $O/c5N.err || exit 1
timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op T --steps 10 --no-cpu-baseline > $O/c5T.json 2> $O/c5T.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o trace --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-extra > $O/prof.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_$c -o p --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/pmc_$c.log 2>&1 || exit 1
done
