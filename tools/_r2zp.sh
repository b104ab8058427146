set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r2zp; mkdir -p $O
timeout -k 10 300 python tools/exp_pad.py > $O/exp_pad.log 2>&1; rc=$?; cat $O/exp_pad.log; exit $rc
