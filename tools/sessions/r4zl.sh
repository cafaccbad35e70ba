#!/bin/bash
# r4 session zl: staged loads of the transposing tiles pipelined into LDS, G loads in flight per
# thread (tile_kernels.hip kStagePipe, tuning builds pipe2 / pipe4) against all at once
set -o pipefail
O=gpurun_out/r4zl
mkdir -p $O
for rep in 1 2 3; do
  for v in default pipe2 pipe4; do
    lib=""; [ $v != default ] && lib=gpuvar/$v/lib/libcosta_amd.so
    for a in "f64 16384 256 0.0 20" "f64 32768 256 0.0 10" "f32 16384 256 0.0 20" "c64 16384 256 0.0 20"; do
      echo -n "$v " >> $O/pipe.txt
      COSTA_LIB=$lib timeout -k 10 200 python3 tools/order_probe.py $a >> $O/pipe.txt 2>> $O/err.txt || exit 1
    done
  done
done
COSTA_LIB=gpuvar/pipe2/lib/libcosta_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py -x -q > $O/pytest_pipe2.log 2>&1 || exit 1
