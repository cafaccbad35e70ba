set -o pipefail
O=gpurun_out/xb3; mkdir -p $O
for rep in 1 2; do for b in 0 1; do for op in N T; do
  COSTA_XCD_BANDS=$b COSTA_LOOPBACK=1 timeout -k 10 300 python3 tools/c5_sort_probe.py $op 10 2>&1 | grep -v amdgpu.ids | sed "s/^/bands=$b /" >> $O/loopback.txt || exit 1
done; done; done
