set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r2zd}; mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests/test_fused_gpu.py tests/test_tiny_gpu.py tests/test_parity_gpu.py tests/test_edge_cases_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
fi
for f in 1 0 1 0; do PFDR_FUSE=$f timeout -k 10 120 python bench.py --workload ${WL:-c1} --no-cpu-baseline --no-kernel-events > $O/c1_f$f.log 2>&1 || exit $?; echo "fuse=$f $(grep -o '"ms_per_step": [0-9.]*' $O/c1_f$f.log)"; done
