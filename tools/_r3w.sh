set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3w; mkdir -p $O
S=60x60,120x120,240x240,480x480
timeout -k 10 300 python -u tools/exp_sx_lifecycle.py $S > $O/nt256.log 2>&1 || exit $?
PFDR_SX_NT=64 timeout -k 10 300 python -u tools/exp_sx_lifecycle.py $S > $O/nt64.log 2>&1 || exit $?
grep graph=1 $O/nt256.log; echo ---; grep graph=1 $O/nt64.log
