set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r3zm; export TMPDIR=/tmp
# tiled-partition diagnostic: tiled ranks without Z-direct
echo "== tp no zd"; PFDR_LIB_PATH=scratch/tpnz.so timeout -k 10 240 python -u tools/diag_partition.py 12 2>&1 | grep -v amdgpu.ids | cut -c1-140 || exit 1
echo "== tp no zd, no overlap"; PFDR_LIB_PATH=scratch/tpno.so timeout -k 10 240 python -u tools/diag_partition.py 6 2>&1 | grep -v amdgpu.ids | cut -c1-140 || exit 1
TAG=r3zm PMC="headline:60000000:10000000 c2:50135040:16777216 c5:785203200:262144000" bash tools/round_check.sh
