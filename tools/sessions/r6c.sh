#!/bin/bash
# r6 session c: HBM read bytes by request size (TCC_EA0_RDREQ_128B / _64B / _32B, tools/pmc_bytes.py)
# on the calibration kernels, cfg 5 and the headline; cfg 5 destination-block groups reading their
# sources as aligned 16-byte chunks (tuning build gpuvar/cbv, COSTA_CB_VLOAD), with and without the
# XCD column bands, against the shipped groups and the wavefront path
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
export TMPDIR=/tmp
P="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
timeout -s KILL 60 rocprofv3 --pmc $P -d $O/calib_bytes -o p --output-format csv -- ./tools/fetch_calib 3 > $O/calib_bytes.log 2>&1 || exit 1
python3 tools/pmc_bytes.py $O/calib_bytes --all > $O/calib_bytes.txt 2>&1
CBV=gpuvar/cbv/lib/libcosta_amd.so
COSTA_LIB=$CBV timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_cbv.txt 2>&1 || exit 1
L="shipped: wave:COSTA_TUNING=1,COSTA_CBLOCK=0 cbv:COSTA_LIB=$CBV cbv_bands:COSTA_LIB=$CBV,COSTA_TUNING=1,COSTA_CB_BANDS=1"
timeout -k 10 600 python3 tools/ab_bench.py $O/c5N 2 $L \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
L="shipped: cbv:COSTA_LIB=$CBV"
timeout -k 10 400 python3 tools/ab_bench.py $O/c5T 2 $L \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
B="--steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra"
for v in N_shipped N_wave N_bands N_cbv T_shipped T_cbv; do
  op=${v%%_*}
  case $v in
    *_wave) E="COSTA_TUNING=1 COSTA_CBLOCK=0";;
    *_bands) E="COSTA_TUNING=1 COSTA_CB_BANDS=1";;
    *_cbv) E="COSTA_LIB=$CBV";;
    *) E="";;
  esac
  env $E timeout -s KILL 200 rocprofv3 --pmc $P -d $O/bytes_$v -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op $op $B > $O/bytes_$v.log 2>&1 || exit 1
  echo "== $v" >> $O/bytes_summary.txt
  python3 tools/pmc_bytes.py $O/bytes_$v $([ $op = N ] && echo 1073741824 || echo 2147483648) >> $O/bytes_summary.txt 2>&1
done
timeout -s KILL 200 rocprofv3 --pmc $P -d $O/bytes_cfg2 -o p --output-format csv -- python3 bench.py $B > $O/bytes_cfg2.log 2>&1 || exit 1
echo "== cfg2" >> $O/bytes_summary.txt
python3 tools/pmc_bytes.py $O/bytes_cfg2 2147483648 >> $O/bytes_summary.txt 2>&1
