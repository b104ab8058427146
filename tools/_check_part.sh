set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3zl; export TMPDIR=/tmp
# diagnostics of the tiled-partition mismatch: default tree, then the tiled
# variant with the device cache on / off and with the overlap off
timeout -k 10 240 python -u tools/diag_partition.py 12 2>&1 | grep -v amdgpu.ids | cut -c1-140 || exit 1
echo "== tp cache on"; PFDR_LIB_PATH=scratch/tp.so timeout -k 10 240 python -u tools/diag_partition.py 12 2>&1 | grep -v amdgpu.ids | cut -c1-140 || exit 1
echo "== tp cache off"; PFDR_DEVICE_CACHE_MB=0 PFDR_LIB_PATH=scratch/tp.so timeout -k 10 240 python -u tools/diag_partition.py 12 2>&1 | grep -v amdgpu.ids | cut -c1-140 || exit 1
echo "== tp no overlap"; PFDR_LIB_PATH=scratch/tpno.so timeout -k 10 240 python -u tools/diag_partition.py 12 2>&1 | grep -v amdgpu.ids | cut -c1-140 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_fullsize_gpu.py tests/test_partition_gpu.py tests/test_bench_ranks_gpu.py tests/test_tiled_gpu.py tests/test_fullsize_pin_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zl/pytest.log 2>&1; rc=$?
tail -n 3 gpurun_out/r3zl/pytest.log; exit $rc
