#!/bin/bash
# A/B of environment settings (tuning knobs) on bench workloads, alternating, twice:
#   tools/env_ab.sh TAG "ENV_A" "ENV_B" ... -- workloads (c5N c5T c2)
set -o pipefail
O=gpurun_out/$1
shift
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
shift
W=${@:-c5N c5T}
mkdir -p $O
for rep in 1 2; do
  for w in $W; do
    case $w in
      c5T) a="--workload cfg5 --cfg5-op T --steps 10" ;;
      c5N) a="--workload cfg5 --cfg5-op N --steps 10" ;;
      c2) a="--steps 20" ;;
    esac
    for i in "${!envs[@]}"; do
      env ${envs[$i]} timeout -k 10 300 python3 bench.py $a --no-cpu-baseline --no-e2e --no-extra >> $O/e${i}_$w.json 2>> $O/e${i}_$w.err || exit 1
    done
  done
done
for i in "${!envs[@]}"; do echo "e$i: ${envs[$i]}" >> $O/envs.txt; done
