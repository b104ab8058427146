set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r4x; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python tools/rec_check.py rec || exit 1
PFDR_LIB_PATH=scratch/norec.so timeout -k 10 300 python tools/rec_check.py norec || exit 1
python - <<'PY'
import numpy as np
for k in ("single", "k2"):
    a = np.load("gpurun_out/rec_%s.npy" % k); b = np.load("gpurun_out/norec_%s.npy" % k)
    d = np.nonzero(a != b)[0]
    print(k, "differs at", d.size, "entries", d[:5], d[-5:] if d.size else "")
a = np.load("gpurun_out/norec_single.npy"); b = np.load("gpurun_out/norec_k2.npy")
print("norec single vs k2 differ:", int((a != b).sum()))
a = np.load("gpurun_out/rec_single.npy"); b = np.load("gpurun_out/rec_k2.npy")
print("rec single vs k2 differ:", int((a != b).sum()))
PY
TAG=r4x tools/gpu_tests.sh "tests/test_tiled_gpu.py tests/test_partition_tiled_gpu.py" || exit 1
