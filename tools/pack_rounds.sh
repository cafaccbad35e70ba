set -o pipefail
O=gpurun_out/pk1; mkdir -p $O
for r in 1 4; do for op in N T; do
  COSTA_EXCHANGE_ROUNDS=$r COSTA_LOOPBACK=1 timeout -k 10 300 python3 tools/c5_sort_probe.py $op 10 2>&1 | grep "^sort" | sed "s/^/rounds=$r /" >> $O/lb.txt || exit 1
  COSTA_EXCHANGE_ROUNDS=$r COSTA_LOOPBACK=1 timeout -k 10 120 python3 tools/order_probe.py f64 16384 256 0 10 2>/dev/null | grep "^f64" | sed "s/^/rounds=$r /" >> $O/lb.txt || exit 1
done; done
