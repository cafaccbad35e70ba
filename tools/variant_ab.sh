#!/bin/bash
# A/B of the shipped library against the tuning builds under build/variants on cfg 5 'T' / 'N'
# (a variant directory's `env` file: environment for its runs, e.g. COSTA_TINY_LDS=8192)
# (and cfg 2), alternating, twice; first the -m gpu suite on the shipped library
#   tools/variant_ab.sh TAG [workloads...]   (default workloads: c5T c5N)
set -o pipefail
O=gpurun_out/${1:-vab}
shift
W=${@:-c5T c5N}
mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
fi
run() {  # name lib workload
  local a
  case $3 in
    c5T) a="--workload cfg5 --cfg5-op T --steps 10" ;;
    c5N) a="--workload cfg5 --cfg5-op N --steps 10" ;;
    c2) a="--steps 20" ;;
  esac
  local e=""
  [ -n "$2" ] && [ -f $(dirname $2)/env ] && e=$(cat $(dirname $2)/env)
  env $e COSTA_LIB=$2 timeout -k 10 300 python3 bench.py $a --no-cpu-baseline --no-e2e --no-extra >> $O/$1_$3.json 2>> $O/$1_$3.err || exit 1
}
for rep in 1 2; do
  for w in $W; do
    run shipped "" $w || exit 1
    for v in build/variants/*/; do
      run $(basename $v) $v/libcosta_amd.so $w || exit 1
    done
  done
done
