set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4i; mkdir -p $OUT; export TMPDIR=/tmp
TAG=r4i tools/gpu_tests.sh "tests/test_seqdif_gpu.py" || exit 1
for arm in new:"" graph:scratch/specgraph.so; do
  n=${arm%%:*}; L=${arm#*:}
  PFDR_LIB_PATH=$L timeout -k 10 300 python bench.py --workload headline_conv --no-cpu-baseline > $OUT/conv_$n.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads([l for l in open('$OUT/conv_$n.log') if l.startswith('{')][-1]); print('$n', d['ms_per_step'], d['converged_iterations'], d['time_to_tolerance_s'])"
done
TAG=r4i WL="c1 c2 c3 c3_ata c4 c5 headline_shuffled headline_slab8" tools/measure.sh wl
