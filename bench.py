"""Benchmark of the MI355X PFDR hot path (BASELINE.json metric).

Default workload (SURVEY.md §8(d) 'Headline'): PFDR_graph_quadratic_d1_l1<float>,
identity A, La_d1 = 0.1, La_l1 = 0.01, rho = 1.5, on the jittered
250x200x200 grid where every vertex emits its 6 nearest 26-neighbours:
V = 10,000,000 vertices, E = 60,000,000 edges.  One "step" = one PFDR
iteration over the whole graph (halo pull, edge sweep, halo push, vertex
sweep), inputs resident in HBM, difTol = difRcd = 0 and Obj = Dif = NULL as
in the reference's per-iteration timing methodology (setup excluded,
reported separately).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload NAME]

N > 1 (launched by torch.distributed.run, one process per GPU): every rank
owns a z-slab of the graph (1-D vertex-range partition, RCCL halo exchange,
DESIGN.md §6).  Default ``--scaling strong``: the metric's fixed 10M-vertex
graph is split across the N GPUs; ``--scaling weak`` gives every GPU a
10M-vertex slab of an N-times taller grid.  ``value`` = all ranks' edge
updates / max-over-ranks time.  The ranks bootstrap over a gloo (host)
process group; the one RCCL communicator of the process is the library's
(halo exchanges, scalar all-reduces, the max-over-ranks timing reduction).

Prints ONE JSON line (rank 0) with the roofline of the dominant kernel and
of every sweep beside it (HIP events on the session stream over the timed
region; SURVEY.md §8(d)'s bytes split per sweep as tools/workloads.py states;
PMC traffic from profiles/pmc/<workload>.json), the whole iteration's
fraction, and the reference CPU path timed on this host (bounded sample, its
own process, before this process touches the GPU).
`--workload c1..c5` selects the other BASELINE.json configs
(tools/workloads.py), measured for DESIGN.md; the driver's line is the
default headline.
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
sys.path.insert(0, os.path.join(ROOT, "tools"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
CPU_PAIRS = 5          # CPU baseline: paired (T(k0), T(k1)) estimates, median reported
CORE_GBS = 25.0        # one host core's streaming rate, upper bound (baseline floor)


# ------------------------------------------------------------ CPU baseline --
def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline_child(args):
    """Runs in its own process: time the reference CPU path (oracle/_ref
    OpenMP build if present, else the restatement) on this host."""
    avail = sorted(os.sched_getaffinity(0))
    cores = avail[: min(len(avail), args.cpu_cores)]
    os.sched_setaffinity(0, cores)  # omp_get_num_procs honours the mask
    host = {"cpu_model": cpu_model(), "host_cpus": os.cpu_count(), "affinity_cpus": len(avail)}
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from workloads import WORKLOADS
    kind = "reference" if oracle.available("ref_omp") else "port"
    lib = oracle.Oracle("ref_omp" if kind == "reference" else "port")
    if args.workload in ("c1", "headline_conv"):  # time to tolerance, whole solve
        inp = WORKLOADS[args.workload].inputs(0, 1)
        kw = inp["kw"]
        Eu, Ev = kw["Eu"].astype(np.int32), kw["Ev"].astype(np.int32)
        t = time.perf_counter()
        X, it, _, _ = lib.quadratic_d1_l1(kw["X0"].copy(), kw["Y"], None, 0, Eu, Ev, kw["La_d1"],
                                          kw["La_l1"], 0, int(kw.get("Ltype", 0)), None,
                                          kw["rho"], kw["condMin"], 0.0, kw["difTol"], 10000)
        el = time.perf_counter() - t
        print(json.dumps({
            "value": Eu.size * it / el / 1e6, "unit": "Medge-updates/s",
            "cores": len(cores) if kind == "reference" else 1, "kind": kind,
            "converged_iterations": it, "time_to_tolerance_s": el,
            "sample": "whole %s solve to difTol %g (setup included), same inputs" % (
                args.workload, kw["difTol"]), **host}))
        return
    name = args.workload if args.workload in ("c2", "c3", "c4", "c5") else "headline"
    sample = "full %s graph" % name
    if name == "c3":  # host-generated A (the pinned law of tests/fullsize_cases.py)
        from cp_pfdr_graph_d1_amd import pfdr
        N, nx, ny = 1024, 2000, 1000
        V = nx * ny
        h = (3.0 / N) ** 0.5
        A = pfdr.gen_uniform(3, N * V, -h, h, np.float32)
        x0 = np.zeros(V, np.float32)
        x0[: V // 3], x0[V // 3: 2 * V // 3] = 1.0, -0.5
        Eu, Ev = pfdr.gen_grid_edges((nx, ny), 4)
        L = np.array([(1.0 + (V / N) ** 0.5) ** 2], np.float32)  # ||A||^2 of U(-h, h), N x V
        kw = dict(Y=pfdr.gen_matvec(A, N, V, x0), A=A, N=N, La_d1=np.full(Eu.size, 0.05, np.float32),
                  La_l1=np.full(V, 0.005, np.float32), X0=np.zeros(V, np.float32), rho=1.5,
                  condMin=1e-3, L=L)
        sample = "C3 direct N=1024 x V=2M (A 8.2 GB host-generated)"
    elif name == "c5":  # a 640x640x80 6-NN grid: the size of one GPU's slab at N = 8
        from cp_pfdr_graph_d1_amd import pfdr
        Eu, Ev = pfdr.gen_grid_edges((640, 640, 80), 6)
        V = 640 * 640 * 80
        kw = dict(X0=np.zeros(V, np.float32), Y=pfdr.gen_piecewise(640, V, 5, np.float32, 0.2),
                  La_d1=np.full(Eu.size, 0.1, np.float32), lo=0.0, hi=1.0, rho=1.5, condMin=1e-3)
        sample = "C5 law on a 640x640x80 6-NN grid (1/8 of 640^3: one GPU's share at N=8)"
    else:
        inp = WORKLOADS[name].inputs(0, 1)
        kw, V = inp["kw"], inp["V"]
        Eu, Ev = kw["Eu"], kw["Ev"]
    Eu, Ev = Eu.astype(np.int32), Ev.astype(np.int32)
    # per-iteration time = (T(k1) - T(k0)) / (k1 - k0): the median of CPU_PAIRS
    # paired estimates (T(k0) then T(k1), back to back) over a span of 40
    # iterations (10 for the slow dense / simplex configurations), the OpenMP
    # threads bound one per core (OMP_PROC_BIND / OMP_PLACES, set by the
    # parent): a difference of two independently noisy minima over 10
    # iterations had spread 0.55 (round 4's driver line)
    args.cpu_k0, args.cpu_k1 = {"c3": (1, 11), "c4": (1, 11)}.get(name, (2, 42))

    def call(k):
        if name == "c4":
            lib.loss_d1_simplex(kw["X0"].copy(), kw["Y"], kw["K"], Eu, Ev, kw["La_d1"],
                                al=kw["al"], La_f=None, rho=kw["rho"], condMin=kw["condMin"],
                                difRcd=0.0, difTol=0.0, itMax=k)
        elif name == "c5":
            lib.quadratic_d1_bounds(kw["X0"].copy(), kw["Y"], None, 0, Eu, Ev, kw["La_d1"],
                                    kw["lo"], kw["hi"], 0, None, kw["rho"], kw["condMin"], 0.0,
                                    0.0, k)
        elif name == "c3":
            lib.quadratic_d1_l1(kw["X0"].copy(), kw["Y"], kw["A"], kw["N"], Eu, Ev, kw["La_d1"],
                                kw["La_l1"], 0, 0, kw["L"], kw["rho"], kw["condMin"], 0.0, 0.0, k)
        else:
            lib.quadratic_d1_l1(kw["X0"].copy(), kw["Y"], None, 0, Eu, Ev, kw["La_d1"],
                                kw["La_l1"], 0, 0, None, kw["rho"], kw["condMin"], 0.0, 0.0, k)
    span = args.cpu_k1 - args.cpu_k0
    call(args.cpu_k0)  # warm: page-in of the inputs and the library, thread pool start
    runs = {args.cpu_k0: [], args.cpu_k1: []}
    for rep in range(CPU_PAIRS):
        for k in (args.cpu_k0, args.cpu_k1):
            t = time.perf_counter()
            call(k)
            runs[k].append(time.perf_counter() - t)
    pairs = [(b - a) / span for a, b in zip(runs[args.cpu_k0], runs[args.cpu_k1])]
    per_it = float(np.median(pairs))
    t0 = float(np.median(runs[args.cpu_k0]))
    # floor: the reference's DR average is a serial scatter over 2E ends
    # (src/PFDR_graph_quadratic_d1_l1.cpp:492-497; simplex per label,
    # src/PFDR_graph_loss_d1_simplex.cpp:636-648): one core reads W and Z and
    # read-modify-writes X for each, >= 16 B per edge (x K labels) at no more
    # than CORE_GBS -- a faster iteration means the timing failed
    K = int(kw.get("K", 1)) if name == "c4" else 1
    floor = 16.0 * Eu.size * K / (CORE_GBS * 1e9)
    out = {"unit": "Medge-updates/s", "cores": len(cores) if kind == "reference" else 1,
           "kind": kind,
           "sample": "%s (V=%d, E=%d) fp32, per-iteration time = median over %d back-to-back "
                     "pairs of (T(%d it) - T(%d it)) / %d, OpenMP threads bound to cores, "
                     "setup excluded" % (sample, V, Eu.size, CPU_PAIRS, args.cpu_k1, args.cpu_k0,
                                         span),
           "per_iteration_s": per_it,
           "spread": {"pair_per_iteration_s": [round(x, 6) for x in pairs],
                      "rel": round((max(pairs) - min(pairs)) / per_it, 4) if per_it > 0 else None,
                      "omp": {k: os.environ.get(k) for k in ("OMP_PROC_BIND", "OMP_PLACES")}},
           "bandwidth_floor_s": floor, **host}
    if per_it < floor:
        out.update(value=None, error="per-iteration time %.4g s below the serial-scatter floor "
                                     "%.4g s: timing rejected" % (per_it, floor))
    else:
        out.update(value=Eu.size / per_it / 1e6, iter_per_s=1.0 / per_it,
                   setup_s=t0 - args.cpu_k0 * per_it)
    print(json.dumps(out))


def run_cpu_baseline(args):
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-baseline-child",
           "--cpu-k0", str(args.cpu_k0), "--cpu-k1", str(args.cpu_k1),
           "--cpu-cores", str(args.cpu_cores), "--workload", args.workload]
    # one OpenMP thread per core, kept there (the reference sets its thread
    # count through num_threads clauses, src/PFDR_graph_quadratic_d1_l1.cpp:31-41;
    # libgomp still honours the binding variables)
    env = dict(os.environ, OMP_PROC_BIND="close", OMP_PLACES="cores")
    try:
        out = subprocess.run(cmd, check=True, capture_output=True, text=True,
                             timeout=900, env=env).stdout
        return json.loads(out.strip().splitlines()[-1])
    except Exception as ex:  # reported, never fatal for the GPU number
        return {"value": None, "error": repr(ex)[:300]}


def launch_ranks(n):
    """python -m torch.distributed.run ... bench.py <same arguments>: one
    process per GPU, as the driver launches N > 1; returns its exit status"""
    import socket
    with socket.socket() as so:  # a free rendezvous port on the loopback address
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def pmc_summary(wl, E):
    """The committed rocprofv3 PMC summary of this workload
    (profiles/pmc/<workload>.json, written by tools/pmc_traffic.py) when it
    was taken on this size AND on the kernel sources built into this library
    (sha256 of the solver's csrc sources); else (None, reason)."""
    try:
        from kernel_hash import kernel_source_sha256
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc", wl.name + ".json")))
        if d.get("workload_E") != E:
            return None, "PMC summary taken on another size"
        if d.get("kernel_source_sha256") != kernel_source_sha256(wl.pmc):
            return None, "stale: PMC summary taken on other kernel sources"
        return d["kernels"], None
    except Exception as ex:
        return None, "no PMC summary (%s)" % type(ex).__name__


# every launch of a kernel family once per iteration: a partitioned session's
# boundary launches (edge_sweep_b, vertex_sweep_b) complete the interior ones
FAMILIES = {"edge_sweep": ("edge_sweep", "edge_sweep_b"),
            "vertex_sweep": ("vertex_sweep", "vertex_sweep_b"),
            "sx_edge_sweep": ("sx_edge_sweep",),
            "sx_vertex_sweep": ("sx_vertex_sweep", "sx_vertex_wide"),  # K <= 64 / K > 64
            "gemv_cols": ("gemv_cols",), "gemv_rows": ("gemv_rows",), "symv": ("symv",)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="headline")
    ap.add_argument("--scaling", default="strong", choices=("strong", "weak"),
                    help="N > 1: split the configuration's graph (strong) or one slab per GPU (weak)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-inputs", action="store_true",
                    help="hand the session host arrays (pinned for their copies during the "
                         "setup) instead of device-resident inputs (A/B runs)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="time the steps without per-kernel HIP events (A/B runs)")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="one rank through the whole distributed path (gloo bootstrap, RCCL "
                         "communicator, partitioned session): a one-GPU rehearsal of N > 1")
    ap.add_argument("--check-ranks", action="store_true",
                    help="only form the process group of --gpus ranks (gloo) and report it")
    ap.add_argument("--cpu-baseline-child", action="store_true")
    ap.add_argument("--cpu-k0", type=int, default=2)
    ap.add_argument("--cpu-k1", type=int, default=12)
    ap.add_argument("--cpu-cores", type=int, default=16)
    args = ap.parse_args()
    if args.cpu_baseline_child:
        cpu_baseline_child(args)
        return
    if args.gpus < 1:
        sys.exit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # not launched per rank: start one process per GPU as a CHILD (this
        # process never touches the GPU) and exit with its status
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit("bench.py: --gpus %d but %d ranks were launched (WORLD_SIZE)" % (args.gpus, world))
    if args.check_ranks:  # launch check only (CPU): form the group, report it
        import torch.distributed as dist
        dist.init_process_group("gloo")
        n = dist.get_world_size()
        if dist.get_rank() == 0:
            print(json.dumps({"ranks": n}))
        dist.destroy_process_group()
        sys.exit(0 if n == args.gpus else 1)
    from workloads import WORKLOADS
    wl = WORKLOADS[args.workload]
    steps = args.steps if args.steps is not None else wl.steps

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist_on = world > 1 or args.dist_selftest
    # CPU baseline first, in its own process, before this process touches the GPU
    cpu = None
    if rank == 0 and world == 1 and wl.name in ("headline", "headline_conv", "c1", "c2", "c3",
                                                 "c4", "c5") and \
            not args.no_cpu_baseline:
        cpu = run_cpu_baseline(args)

    import torch
    import torch.distributed as dist
    from cp_pfdr_graph_d1_amd import pfdr

    torch.cuda.set_device(local)
    if dist_on:  # host bootstrap only: the data path uses the library's RCCL communicator
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29517")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("gloo")

    def barrier():
        if dist_on:
            dist.barrier()

    strong = args.scaling == "strong" or wl.scaling == "strong"
    t = time.perf_counter()
    inp = wl.inputs(rank, world, strong)
    gen_s = time.perf_counter() - t
    V, E = inp["V"], inp["E"]
    converge = bool(inp.get("converge", False))
    kw = inp["kw"]
    if not kw.get("device") and not args.host_inputs and not dist_on:
        # inputs resident in HBM before the session is built (the metric's
        # premise): the setup then copies device to device and pins no host
        # memory -- unpinning ~0.8 GB of caller arrays at its end left the
        # GPU idle for ~30 ms, enough for its clock to drop before the
        # iterations
        dev_kw = dict(kw, device=True)
        for k in ("Eu", "Ev", "La_d1", "X0", "Y", "La_l1", "A", "L"):
            a = kw.get(k)
            if a is not None:  # (the dtypes the host path converts to)
                a = np.ascontiguousarray(a, np.int32 if k in ("Eu", "Ev") else wl.dtype)
                dev_kw[k] = torch.from_numpy(a).to("cuda:%d" % local)
        kw = inp["kw"] = dev_kw
        torch.cuda.synchronize()
    dev_inputs = bool(kw.get("device"))
    dist_kw, parallelism, comm = {}, "single", None
    if dist_on and wl.partitionable:  # 1-D vertex-range partition, RCCL halo over xGMI
        from cp_pfdr_graph_d1_amd import partition
        comm = partition.comm_init(world, rank, lambda x: dist.broadcast(x, 0))
        dist_kw = dict(nranks=world, rank=rank, comm=comm, comm_kind=partition.COMM_RCCL,
                       vtx_begin=inp["vtx_begin"], e_offset=inp["e_offset"],
                       e_global=inp.get("e_global"), vtx_label=inp.get("vtx_label"))
        parallelism = "vertex-partition x%d (RCCL halo), %s scaling" % (
            world, "strong" if strong else "weak")
    elif world > 1:
        strong = False
        parallelism = "independent replicas x%d" % world
    warm = 0 if converge else args.warmup
    # the timed steps run unprofiled, so the session replays its captured
    # chunks (one hipGraph launch per 32 iterations; RCCL partitions with the
    # pull, sweeps and push inside): the production launch path.  The kernel
    # means come from a second, profiled pass of the same length.
    post_events = not converge and not args.no_kernel_events
    itMax = steps if converge else warm + steps + (steps if post_events else 0)
    t = time.perf_counter()
    sess = pfdr.Session(wl.kind, wl.dtype, V, E, itMax=itMax, **kw, **dist_kw)
    setup_s = time.perf_counter() - t
    desc, graph, extra = inp["desc"], inp["graph"], inp.get("extra")
    del inp
    if not converge:
        del kw
    # the timed run replays hipGraphs captured here, BEFORE the warmup: the
    # GPU idles while the host captures them, and the warmup steps then bring
    # its clocks back up ahead of the timed ones
    sess.profile(False)
    sess.prepare(steps)
    if warm:
        sess.run(warm)
        sess.prepare(steps)  # (a speculative session's graphs follow the start's parity)
    # per-kernel HIP events in the timed region, on the dominant kernels only
    # and on every PERIOD-th launch (an event pair costs ~6-9 us of GPU time,
    # profiles/r2/r2d_launch_gap.log); a small solve timed to tolerance is
    # timed bare and a second, profiled solve gives the kernel means
    timed = sorted({wl.dominant, "edge_sweep", "vertex_sweep", "sx_edge_sweep",
                    "sx_vertex_sweep", "sx_vertex_wide", "gemv_cols", "gemv_rows"})
    period = 4 if world == 1 else 8
    torch.cuda.synchronize()
    barrier()
    t0 = time.perf_counter()
    it = sess.run(steps)
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    done = it - warm
    assert converge or done == steps, (it, warm, steps)
    el_max, E_all = el, E * world
    if dist_on:  # host reductions (gloo): max time, total edges
        tmax = torch.tensor([el], dtype=torch.float64)
        tsum = torch.tensor([E], dtype=torch.int64)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        el_max, E_all = float(tmax[0]), int(tsum[0])
    if post_events:
        sess.profile(True, period=period, only=timed)
        sess.run(steps)
        torch.cuda.synchronize()
        barrier()
    if converge:
        res_timed = sess.result()
        sess.close()
        sess = pfdr.Session(wl.kind, wl.dtype, V, E, itMax=itMax, **kw, **dist_kw)
        sess.profile(True, only=timed)
        sess.run(steps)
        torch.cuda.synchronize()
        del kw
    names = (wl.dominant, "edge_sweep", "edge_sweep_b", "vertex_sweep", "vertex_sweep_b",
             "sx_edge_sweep", "sx_vertex_sweep", "sx_vertex_wide", "gemv_rows",
             "gemv_cols", "halo_pull", "halo_push", "seq_evolution")
    stats = {k: sess.kernel_stats(k) for k in names}
    res = res_timed if converge else sess.result()
    finite = bool(np.all(np.isfinite(res[0])))
    dev_bytes = sess.device_bytes()
    reordered = bool(sess.query("reordered"))
    quad = wl.kind != pfdr.PFDR_KIND_SIMPLEX
    split_blocks = sess.query("split_blocks") if quad else 0
    tiled_blocks = sess.query("tiled_blocks")  # (simplex: edges in tile order)
    record_blocks = sess.query("record_blocks")  # (simplex: tile blocks staged from their runs)
    try:  # (tiled quadratic: distinct run slot patterns; a library before round 6 has no key)
        slot_patterns = sess.query("slot_patterns")
    except pfdr.PFDRError:
        slot_patterns = None
    symv = sess.query("symv") if quad else 0  # A^tA from its block upper triangle
    seqdif = sess.query("seqdif")
    # which speculative mode ran (PFDR_SPEC / pfdr_problem.spec): the decision
    # on t beside t + 1 on its own stream (a partition: over a split
    # communicator), serially on the session stream, or none
    spec_ran = {0: "none", 1: "overlapped (second stream%s)" % (
        ", split communicator" if dist_kw else ""), 2: "serial (session stream, one communicator)"}[
        sess.query("speculative")]
    # kernel names behind each family (rocprof / PMC summaries)
    knames = {f: ["k_" + f] for f in FAMILIES}
    if quad and sess.query("ustaged"):  # u ends staged in LDS for u-sorted edges
        knames["edge_sweep"] = ["k_edge_sweep_us"]
    if quad and sess.query("tiled_blocks"):  # tile-ordered edges (large single-GPU graphs)
        knames["edge_sweep"] = ["k_edge_sweep_tl"]
    try:  # two record blocks per workgroup (regular f32 grids; a library before round 6 has no key)
        vpair = quad and sess.query("vertex_pair") > 0
    except pfdr.PFDRError:
        vpair = False
    if vpair:  # (an odd last block runs in a k_vertex_sweep launch of its own)
        knames["vertex_sweep"] = ["k_vertex_sweep_pair", "k_vertex_sweep"]
    if symv:
        knames["symv"] = ["k_symv_tiles", "k_symv_finish"]
    # the dense direct products (N > 0): the column dots and the row partials
    # with their fixed-order finish
    knames["gemv_cols"] = ["k_col_dot"]
    knames["gemv_rows"] = ["k_rows_partial", "k_rows_finish"]
    if not quad and 0 < getattr(wl, "K", 0) <= 64:  # workgroups of M vertex blocks (default),
        # or the one-block sweep (PFDR_SX_M=1)
        knames["sx_vertex_sweep"] = ["k_sx_vertex_tile", "k_sx_vertex_sweep"]
    if not quad and getattr(wl, "K", 0) > 64:  # group sweep (LDS columns), or a wave per vertex
        knames["sx_vertex_sweep"] = ["k_sx_vertex_group", "k_sx_vertex_wide"]
        knames["sx_vertex_wide"] = ["k_sx_vertex_group", "k_sx_vertex_wide"]
    sess.close()
    if comm:
        from cp_pfdr_graph_d1_amd import partition
        partition.comm_destroy(comm)
    if dist_on:
        dist.destroy_process_group()
    if rank != 0:
        return
    ms_step = el_max / max(done, 1) * 1e3
    # per kernel family: SURVEY.md 8(d)'s bytes of that sweep (tools/workloads.py
    # kernel_bytes) over its mean time per iteration (HIP events, timed region)
    pmc, pmc_note = pmc_summary(wl, E)
    kbytes = wl.kernel_bytes(V, E)
    kernels = {}
    for fam, alg_b in kbytes.items():
        ms = sum(stats[k][1] for k in FAMILIES[fam] if k in stats and stats[k][0])
        if ms <= 0:
            continue
        gbs = alg_b / (ms * 1e-3) / 1e9
        # effective_*: SURVEY 8(d)'s bytes of the reference loop this sweep
        # replaces.  The layout moves fewer (Z-direct: no W*Z stores), so that
        # figure can pass 1; frac is the kernel's own measured HBM bytes (PMC,
        # when a summary taken on these sources exists) over time and peak.
        # the family's kernels that ran in the profiled pass (a K > 64
        # simplex runs the group sweep or, past the LDS, the wide one)
        ks = [k for k in knames[fam] if pmc is None or k in pmc] or knames[fam]
        row = {"kernel": "+".join(ks), "algorithmic_bytes": int(alg_b),
               "mean_ms": round(ms, 5), "effective_GBps": round(gbs, 1),
               "effective_frac": round(gbs / HBM_PEAK_GBS, 4)}
        if pmc is not None and all(k in pmc for k in ks):
            t = sum(pmc[k]["hbm_bytes_per_launch"] for k in ks)
            row["pmc_bytes"] = int(t)
            row["pmc_over_algorithmic"] = round(t / alg_b, 3)
            row["achieved_GBps"] = round(t / (ms * 1e-3) / 1e9, 1)
            row["frac"] = round(row["achieved_GBps"] / HBM_PEAK_GBS, 4)
            row["frac_basis"] = "pmc"
        else:
            row["achieved_GBps"] = row["effective_GBps"]
            row["frac"] = row["effective_frac"]
            row["frac_basis"] = "algorithmic (no PMC summary on these sources)"
        kernels[fam] = row
    # the roofline prices the kernel that takes longest per iteration (the C4
    # simplex vertex sweep outlasts its edge sweep; the workload's nominal
    # dominant when no kernel was timed)
    dom_name = max(kernels, key=lambda f: kernels[f]["mean_ms"]) if kernels else wl.dominant
    dom = kernels.get(dom_name, {})
    it_bytes = wl.iteration_bytes(V, E)
    it_gbs = it_bytes / (ms_step * 1e-3) / 1e9
    out = {
        "metric": wl.metric,
        "value": round(E_all * done / el_max / 1e6, 2),
        "unit": "Medge-updates/s",
        "n_gpus": world,
        "steps": done,
        "warmup": warm,
        "ms_per_step": round(ms_step, 4),
        "iter_per_s": round(1e3 / ms_step, 2),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64" if wl.dtype == np.float64 else "f32",
        "data": "synthetic",
        "config": {
            "workload": desc,
            "global_graph": graph,
            "V_per_gpu": V, "E_per_gpu": E,
            "parallelism": parallelism,
            "setup_s": round(setup_s, 3),
            "device_inputs": dev_inputs,
            "input_generation_s": round(gen_s, 3),
            "device_bytes": dev_bytes,
            "relabelled": reordered,
            "split_incidence_blocks": split_blocks,
            "tiled_blocks": tiled_blocks,
            "record_blocks": record_blocks,
            "slot_patterns": slot_patterns,
            "sequential_evolution": bool(seqdif),
            "speculation": spec_ran,
            **({"symv_upper_triangle": bool(symv)} if wl.dominant == "symv" else {}),
            "finite": finite,
        },
        "roofline": {
            "bound": "hbm",
            "kernel": dom.get("kernel"),
            "achieved": dom.get("achieved_GBps"),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": dom.get("frac"),
            "frac_basis": dom.get("frac_basis"),
            "traffic": dom.get("pmc_bytes"),
            "effective_achieved": dom.get("effective_GBps"),
            "effective_frac": dom.get("effective_frac"),
            **({"traffic_note": pmc_note} if pmc_note else {}),
            "algorithmic_bytes_per_launch": dom.get("algorithmic_bytes"),
            "timed_launches": "every %d-th launch of %s%s" % (period, ", ".join(
                k for k in timed if stats.get(k, (0,))[0]),
                ", in a profiled pass of the same length after the unprofiled (graph-replayed) "
                "timed steps" if post_events else ", inside the timed steps"),
            "launches": stats[dom_name][0] if dom_name in stats else 0,
            "dominant_rule": "the kernel family with the longest mean time per iteration",
            "mean_ms": dom.get("mean_ms"),
            "kernels": kernels,
            "kernels_mean_ms": {k: round(v[1], 5) for k, v in stats.items() if v[0]},
            "iteration": {"algorithmic_bytes": int(it_bytes), "achieved_GBps": round(it_gbs, 1),
                          "frac": round(it_gbs / HBM_PEAK_GBS, 4)},
        },
        "cpu_baseline": cpu,
    }
    if extra:
        out["extra"] = extra
    if converge:
        out["converged_iterations"] = it
        out["time_to_tolerance_s"] = round(el_max, 4)
        out["final_dif"] = None if res[3] is None or res[1] < 1 else float(res[3][res[1] - 1])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
