"""Benchmark of the MI355X PFDR hot path (BASELINE.json metric).

Workload (SURVEY.md §8(d) 'Headline'): PFDR_graph_quadratic_d1_l1<float>,
identity A, La_d1 = 0.1, La_l1 = 0.01, rho = 1.5, on the jittered
250x200x200 grid where every vertex emits its 6 nearest 26-neighbours:
V = 10,000,000 vertices, E = 60,000,000 edges.  One "step" = one PFDR
iteration over the whole graph (edge sweep + vertex sweep), inputs resident
in HBM, difTol = difRcd = 0 and Obj = Dif = NULL as in the reference's
per-iteration timing methodology (setup excluded, reported separately).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 (launched by torch.distributed.run, one process per GPU): weak
scaling — every rank owns a 10M-vertex slab;
``value`` = all ranks' edge updates / max-over-ranks time.

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel
(edge sweep, HIP events on the session stream over the timed region) and the
reference CPU path timed on this host (bounded sample, its own process).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SHAPE = (250, 200, 200)
KNN = 6
GRAPH_SEED, Y_SEED = 6, 2
LA_D1, LA_L1, RHO, COND_MIN = 0.1, 0.01, 1.5, 1e-3
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# algorithmic bytes: per edge Eu, Ev (8) + Zu, Zv read and
# write (16) + W_d1u, W_d1v, Th_d1 (12) + Wu, Wv (8) = 44 B; per vertex X,
# Y, Ga, Th_l1 read + X write = 20 B (fp32)
EDGE_BYTES, VERTEX_BYTES = 44, 20
METRIC = "PFDR iter/s and Medge-updates/s, 10M-vertex 6-NN graph, 1/2/4/8 MI355X"


def headline_inputs(rank, nranks, dtype=np.float32):
    """Rank r's slab of the weak-scaled headline graph: the global jittered
    grid is 250 x 200 x (200 * nranks), rank r owns the vertices of
    z in [200 r, 200 r + 200) (10M) and the 60M edges they emit; edges
    reaching the next slab are its halo.  nranks = 1: the headline graph."""
    from cp_pfdr_graph_d1_amd import pfdr
    nx, ny, nz = SHAPE
    gshape = (nx, ny, nz * nranks)
    V = nx * ny * nz
    v0 = rank * V
    Eu, Ev = pfdr.gen_knn_jitter_grid(gshape, KNN, GRAPH_SEED, 0.25, (v0, v0 + V))
    Y = pfdr.gen_piecewise(nx, V * nranks, Y_SEED, dtype, 0.2, (v0, v0 + V))
    return gshape, V, Eu, Ev, Y


# ------------------------------------------------------------ CPU baseline --
def cpu_baseline_child(args):
    """Runs in its own process: time the reference CPU path (oracle/_ref
    OpenMP build if present, else the restatement) on this host."""
    avail = sorted(os.sched_getaffinity(0))
    cores = avail[: min(len(avail), args.cpu_cores)]
    os.sched_setaffinity(0, cores)  # omp_get_num_procs honours the mask
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    kind = "reference" if oracle.available("ref_omp") else "port"
    lib = oracle.Oracle("ref_omp" if kind == "reference" else "port")
    _, V, Eu, Ev, Y = headline_inputs(0, 1)
    Eu, Ev = Eu.astype(np.int32), Ev.astype(np.int32)
    La = np.full(Eu.size, LA_D1, np.float32)
    L1 = np.full(V, LA_L1, np.float32)
    times = {}
    for k in (args.cpu_k0, args.cpu_k1):
        t = time.perf_counter()
        lib.quadratic_d1_l1(np.zeros(V, np.float32), Y, None, 0, Eu, Ev, La, L1, 0, 0, None,
                            RHO, COND_MIN, 0.0, 0.0, k)
        times[k] = time.perf_counter() - t
    per_it = (times[args.cpu_k1] - times[args.cpu_k0]) / (args.cpu_k1 - args.cpu_k0)
    print(json.dumps({
        "value": Eu.size / per_it / 1e6, "unit": "Medge-updates/s",
        "cores": len(cores) if kind == "reference" else 1, "kind": kind,
        "iter_per_s": 1.0 / per_it,
        "sample": "full headline graph (V=%d, E=%d) fp32, per-iteration time = "
                  "(T(%d it) - T(%d it)) / %d, setup excluded" % (
                      V, Eu.size, args.cpu_k1, args.cpu_k0, args.cpu_k1 - args.cpu_k0),
        "setup_s": times[args.cpu_k0] - args.cpu_k0 * per_it}))


def run_cpu_baseline(args):
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child",
           "--cpu-k0", str(args.cpu_k0), "--cpu-k1", str(args.cpu_k1),
           "--cpu-cores", str(args.cpu_cores)]
    try:
        out = subprocess.run(cmd, check=True, capture_output=True, text=True,
                             timeout=900).stdout
        return json.loads(out.strip().splitlines()[-1])
    except Exception as ex:  # reported, never fatal for the GPU number
        return {"value": None, "error": repr(ex)[:300]}


def pmc_traffic():
    """Per-launch HBM bytes of the edge sweep from the committed rocprofv3
    PMC summary (profiles/pmc_traffic.json, written by tools/pmc_traffic.py),
    when it matches this workload; else None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
        k = d["kernels"]["k_edge_sweep"]
        if d.get("workload_E") == KNN * SHAPE[0] * SHAPE[1] * SHAPE[2]:
            return k["hbm_bytes_per_launch"]
    except Exception:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-child", action="store_true")
    ap.add_argument("--cpu-k0", type=int, default=2)
    ap.add_argument("--cpu-k1", type=int, default=12)
    ap.add_argument("--cpu-cores", type=int, default=16)
    args = ap.parse_args()
    if args.cpu_baseline_child:
        cpu_baseline_child(args)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # CPU baseline first, in its own process, before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = run_cpu_baseline(args)

    import torch
    import torch.distributed as dist
    from cp_pfdr_graph_d1_amd import pfdr

    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if world > 1:
            dist.barrier()

    gshape, V, Eu, Ev, Y = headline_inputs(rank, world)
    E = Eu.size
    dist_kw = {}
    if world > 1:  # 1-D vertex-range partition, RCCL halo exchange over xGMI
        from cp_pfdr_graph_d1_amd import partition
        comm = partition.comm_init(world, rank, lambda t: dist.broadcast(t, 0))
        dist_kw = dict(nranks=world, rank=rank, comm=comm, comm_kind=partition.COMM_RCCL,
                       vtx_begin=rank * V, V_global=world * V, e_offset=rank * E)
    t = time.perf_counter()
    sess = pfdr.Session(pfdr.PFDR_KIND_L1, np.float32, V, E, Eu, Ev,
                        np.full(E, LA_D1, np.float32), np.zeros(V, np.float32), Y,
                        La_l1=np.full(V, LA_L1, np.float32), rho=RHO, condMin=COND_MIN,
                        difTol=0.0, difRcd=0.0, itMax=args.warmup + args.steps, **dist_kw)
    setup_s = time.perf_counter() - t
    del Eu, Ev
    sess.run(args.warmup)
    sess.profile(True)
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    it = sess.run(args.steps)
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    assert it == args.warmup + args.steps, it
    el_max = el
    if world > 1:
        tt = torch.tensor([el], device="cuda", dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el_max = float(tt.item())
    n_e, ms_e = sess.kernel_stats("edge_sweep")
    n_v, ms_v = sess.kernel_stats("vertex_sweep")
    halo = {k: sess.kernel_stats(k)[1] for k in ("halo_pull", "halo_push")} if world > 1 else {}
    X, _, _, _ = sess.result()
    finite = bool(np.all(np.isfinite(X)))
    dev_bytes = sess.device_bytes()
    sess.close()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    total_edges = E * world
    ms_step = el_max / args.steps * 1e3
    value = total_edges * args.steps / el_max / 1e6
    achieved = EDGE_BYTES * E / (ms_e * 1e-3) / 1e9 if ms_e > 0 else None
    traffic = pmc_traffic()
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Medge-updates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "iter_per_s": round(1e3 / ms_step, 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": "PFDR_graph_quadratic_d1_l1<float>, identity A, l1 + TV, "
                        "jittered %dx%dx%d grid, %d-NN (V=%d, E=%d per GPU)" % (
                            SHAPE + (KNN, V, E)),
            "global_graph": "%dx%dx%d" % gshape,
            "V_per_gpu": V, "E_per_gpu": E,
            "parallelism": "vertex-partition%d (RCCL halo)" % world if world > 1 else "single",
            "average": os.environ.get("PFDR_AVERAGE", "split"),
            "setup_s": round(setup_s, 3),
            "device_bytes": dev_bytes,
            "finite": finite,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_edge_sweep",
            "achieved": None if achieved is None else round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": None if achieved is None else round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": EDGE_BYTES * E,
            "launches": n_e,
            "mean_ms": round(ms_e, 5),
            "vertex_sweep_mean_ms": round(ms_v, 5),
            "halo_mean_ms": {k: round(v, 5) for k, v in halo.items()},
            "iteration_algorithmic_GBps": round(
                (EDGE_BYTES * E + VERTEX_BYTES * V) / (ms_step * 1e-3) / 1e9, 1),
        },
        "cpu_baseline": cpu,
    }
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
