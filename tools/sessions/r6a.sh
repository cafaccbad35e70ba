#!/bin/bash
# r6 session a: FETCH_SIZE / WRITE_SIZE calibration by access width (tools/fetch_calib.hip); cfg 5
# destination-block groups in XCD column bands (COSTA_CB_BANDS=1) against the shipped maps and
# against the wavefront path (COSTA_CBLOCK=0): tests on the bands, A/B, PMC of the bands
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1
timeout -k 10 60 ./tools/fetch_calib 5 > $O/calib.json 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
  timeout -s KILL 60 rocprofv3 --pmc $c -d $O/calib_$c -o p --output-format csv -- ./tools/fetch_calib 3 > $O/calib_$c.log 2>&1 || exit 1
done
COSTA_TUNING=1 COSTA_CB_BANDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_bands.txt 2>&1 || exit 1
L="shipped: bands:COSTA_TUNING=1,COSTA_CB_BANDS=1 wave:COSTA_TUNING=1,COSTA_CBLOCK=0"
for op in N T; do
  timeout -k 10 500 python3 tools/ab_bench.py $O/c5$op 2 $L \
    -- --workload cfg5 --cfg5-op $op --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
done
for op in N T; do
  alg=$([ $op = N ] && echo 2147483648 || echo 3221225472)
  for c in FETCH_SIZE WRITE_SIZE; do
    for v in shipped bands; do
      if [ $v = bands ]; then export COSTA_TUNING=1 COSTA_CB_BANDS=1; else unset COSTA_TUNING COSTA_CB_BANDS; fi
      timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_${op}_${v}_$c -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op $op --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/pmc_${op}_${v}_$c.log 2>&1 || exit 1
      echo "$op $v" >> $O/pmc_summary.txt
      python3 tools/pmc_brief.py $O/pmc_${op}_${v}_$c $alg >> $O/pmc_summary.txt 2>&1
    done
  done
done
