# Host CPU description and the reference's CPU baseline at 1 / 8 / 16 cores
# (affinity mask: the reference sizes its OpenMP teams from
# omp_get_num_procs, which honours it; OMP_NUM_THREADS is ignored).
#   TAG=r2d WL=headline bash tools/cpu_sweep.sh
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-cpu}; mkdir -p $OUT
lscpu > $OUT/lscpu.txt 2>&1 || true
for c in ${CORES:-1 8 16}; do
  timeout -k 10 600 python bench.py --cpu-baseline-child --workload ${WL:-headline} --cpu-cores $c > $OUT/cpu_${WL:-headline}_$c.json 2>&1 || exit $?
  echo "$c cores: $(tail -c 400 $OUT/cpu_${WL:-headline}_$c.json)"
done
