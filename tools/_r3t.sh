set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3t; mkdir -p $O
timeout -k 10 600 python tools/cp_time.py --shapes 256x256,512x512 > $O/cp_time_l1.log 2>&1 || exit $?
cut -c1-400 $O/cp_time_l1.log | tail -2
timeout -k 10 600 python tools/cp_time.py --shapes 128x128,256x256 --kind simplex > $O/cp_time_simplex.log 2>&1 || exit $?
cut -c1-400 $O/cp_time_simplex.log | tail -2
