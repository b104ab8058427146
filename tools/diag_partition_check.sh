set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3zn; export TMPDIR=/tmp
# tiled-partition diagnostic: setup-array hashes per rank over repeated setups
# (scratch/tpd.so: tools/setup_dump.patch applied, -DPFDR_TILED_PARTITIONS=1 -DPFDR_SETUP_DUMP=1)
PFDR_LIB_PATH=scratch/tpd.so timeout -k 10 300 python -u tools/diag_partition.py 6 > gpurun_out/r3zn/dump.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r3zn/dump.log | cut -c1-150 | grep -v "^\[dump\]"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zn/pytest_gpu.log 2>&1; rc=$?
tail -n 3 gpurun_out/r3zn/pytest_gpu.log; exit $rc
