set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; O=gpurun_out/r3c; mkdir -p $O
cat > $O/one.py <<'PY'
import os, sys, time, numpy as np
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import torch
from cp_pfdr_graph_d1_amd import pfdr
from cp_pfdr_graph_d1_amd.graphs import grid_graph
shape, K, dt = (40, 40), 4, np.float32
Eu, Ev = grid_graph(shape, 8); V = 1600
rng = np.random.default_rng(V); Q = rng.random((V, K)); Q = (Q / Q.sum(axis=1, keepdims=True)).reshape(-1).astype(dt)
for f in (os.environ.get("FUSE", "1"),):
    os.environ["PFDR_FUSE"] = f
    s = pfdr.Session(pfdr.PFDR_KIND_SIMPLEX, dt, V, Eu.size, Eu, Ev, np.full(Eu.size, 0.05, dt), Q.copy(), Q, K=K, al=0.1, rho=1.0, condMin=0.1, difRcd=0.0, difTol=1e-12, itMax=700)
    s.run(100); torch.cuda.synchronize(); t = time.perf_counter(); s.run(500); torch.cuda.synchronize()
    print(f, (time.perf_counter() - t) / 500 * 1e6, s.result()[1]); s.close()
PY
for f in 1 0; do
FUSE=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$f -o run --output-format csv -- python $O/one.py > $O/one$f.log 2>&1 || exit $?
grep -v "^[WE]2" $O/one$f.log | tail -1
python tools/trace_gaps.py $O/prof$f/run_kernel_trace.csv 1500 > $O/gaps$f.txt
cat $O/gaps$f.txt
done
