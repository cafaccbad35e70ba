set -o pipefail
O=gpurun_out/vd1; mkdir -p $O
COSTA_LIB=build/variants/vecdst/libcosta_amd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_cfg5.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_vecdst.log 2>&1 || exit 1
NO_TESTS=1 bash tools/variant_ab.sh vd1 c5T || exit 1
