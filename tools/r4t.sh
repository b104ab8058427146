set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-r4t}; mkdir -p $OUT; export TMPDIR=/tmp
TAG=${TAG:-r4t} tools/gpu_tests.sh "tests/test_gram_gpu.py" || exit 1
for v in wg2 wg4; do
  if [ $v = wg4 ]; then export PFDR_LIB_PATH=scratch/gram4.so; else unset PFDR_LIB_PATH; fi
  TAG=${TAG:-r4t}_c3_$v WL=c3 KSEL="k_gram_v" bash tools/profile_mfma.sh > $OUT/mfma_c3_$v.log 2>&1 || { tail -5 $OUT/mfma_c3_$v.log; exit 1; }
  echo "$v c3"; grep -h "Mfma\|gram_kernel_s\|frac" $OUT/mfma_c3_$v.log
  TAG=${TAG:-r4t}_ata_$v WL=c3_ata KSEL="k_gram_v" bash tools/profile_mfma.sh > $OUT/mfma_ata_$v.log 2>&1 || { tail -5 $OUT/mfma_ata_$v.log; exit 1; }
  echo "$v c3_ata"; grep -h "Mfma\|gram_kernel_s\|frac" $OUT/mfma_ata_$v.log
done
