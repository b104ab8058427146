"""Benchmark workloads of bench.py: the headline graph and the five configs of
BASELINE.json, restated concretely in SURVEY.md §8(d).

Each workload builds the session arguments of one rank (inputs generated
deterministically, natively where large) and states its algorithmic bytes
 so bench.py can price each kernel against the HBM
roofline.  SURVEY.md §8(d)'s per-iteration figure is split between the two
sweeps by the reference loop each replaces: the edge sweep owns the TV prox
loop's arrays (ref src/PFDR_graph_quadratic_d1_l1.cpp:466-489: Eu, Ev, Zu and
Zv read and written, W_d1u, W_d1v, Th_d1), the vertex sweep the DR average's
splitting weights (:491-497: Wu, Wv) and the per-vertex arrays; the
simplex the same per (edge, label) (src/PFDR_graph_loss_d1_simplex.cpp:589-648).
Only `headline` is the driver's bench line; the others are run with
`python bench.py --workload cN` for DESIGN.md.
"""
import numpy as np

from cp_pfdr_graph_d1_amd import pfdr


class Workload:
    name = ""
    metric = ""
    kind = pfdr.PFDR_KIND_L1
    dtype = np.float32
    scaling = "weak"
    partitionable = True      # identity/diagonal quadratic: vertex partition
    dominant = "edge_sweep"
    edge_bytes = 44           # algorithmic bytes per edge per iteration
    vertex_bytes = 20
    steps = 50
    itMax_extra = 0
    pmc = "quadratic"         # kernel sources whose hash keys its PMC summary

    def inputs(self, rank, world, strong=True):
        """-> dict(V, E, kw (pfdr.Session kwargs), vtx_begin, e_offset, desc,
        graph[, converge]) of this rank.  strong: the configuration's graph
        is split across the ranks (z- or row-slabs); weak: every rank owns a
        copy-sized slab of a graph stacked `world` times."""
        raise NotImplementedError

    def real_bytes(self):
        return np.dtype(self.dtype).itemsize

    def kernel_bytes(self, V, E):
        """algorithmic HBM bytes of one launch of each sweep: SURVEY.md
        §8(d)'s iteration bytes split as the module docstring says (quadratic:
        edge sweep 8 + 7 s per edge, vertex sweep 2 s per edge + the vertex
        term; they add up to iteration_bytes)"""
        s = self.real_bytes()
        e_edge = 8 + 7 * s
        return {"edge_sweep": e_edge * E,
                "vertex_sweep": (self.edge_bytes - e_edge) * E + self.vertex_bytes * V}

    def dominant_bytes(self, V, E):
        """algorithmic HBM bytes of one launch of the dominant kernel"""
        return self.kernel_bytes(V, E)[self.dominant]

    def iteration_bytes(self, V, E):
        """algorithmic HBM bytes of one whole iteration"""
        return self.edge_bytes * E + self.vertex_bytes * V


def _grid_slab(shape3, rank, world, conn, strong):
    """z-slab of a 3-D grid: weak scaling stacks `world` copies along z,
    strong scaling splits the given grid."""
    nx, ny, nz = shape3
    if strong:
        V_all = nx * ny * nz
        g = (nx, ny, nz)
        z0, z1 = (nz * rank) // world, (nz * (rank + 1)) // world
    else:
        g = (nx, ny, nz * world)
        z0, z1 = nz * rank, nz * (rank + 1)
        V_all = nx * ny * nz * world
    v0, v1 = nx * ny * z0, nx * ny * z1
    Eu, Ev = pfdr.gen_grid_edges(g, conn, (v0, v1))
    return g, V_all, v0, v1, Eu, Ev


class Headline(Workload):
    """The 10M-vertex / 60M-edge 6-NN graph.  Strong scaling (default): the
    fixed graph split into z-slabs of 200/N planes (1.25M vertices per GPU
    at N = 8); weak: a 10M-vertex slab per GPU of a 250x200x(200 N) grid."""
    name = "headline"
    metric = "PFDR iter/s and Medge-updates/s, 10M-vertex 6-NN graph, 1/2/4/8 MI355X"
    SHAPE = (250, 200, 200)

    def inputs(self, rank, world, strong=True):
        nx, ny, nz = self.SHAPE
        if strong:
            g = (nx, ny, nz)
            z0, z1 = (nz * rank) // world, (nz * (rank + 1)) // world
        else:
            g = (nx, ny, nz * world)
            z0, z1 = nz * rank, nz * (rank + 1)
        v0, v1 = nx * ny * z0, nx * ny * z1
        V, V_all = v1 - v0, nx * ny * g[2]
        Eu, Ev = pfdr.gen_knn_jitter_grid(g, 6, 6, 0.25, (v0, v1))
        Y = pfdr.gen_piecewise(nx, V_all, 2, np.float32, 0.2, (v0, v1))
        E = Eu.size
        kw = dict(Eu=Eu, Ev=Ev, La_d1=np.full(E, 0.1, np.float32), X0=np.zeros(V, np.float32),
                  Y=Y, La_l1=np.full(V, 0.01, np.float32), rho=1.5, condMin=1e-3)
        return dict(V=V, E=E, kw=kw, vtx_begin=v0, e_offset=6 * v0,
                    desc="PFDR_graph_quadratic_d1_l1<float>, identity A, l1 + TV, jittered "
                         "%dx%dx%d grid, 6-NN (V=%d, E=%d%s)" % (
                             g[0], g[1], g[2], V_all, 6 * V_all,
                             "" if world == 1 else ", z-slab of %d vertices on this GPU" % V),
                    graph="%dx%dx%d" % g)


class HeadlineConv(Headline):
    """The headline solved to difTol 1e-5 (the parity run):
    time to tolerance and the converged iteration count; the evolution sums
    round as the reference's (PFDR_EVOLUTION_AUTO -> sequential at this size),
    so the count is the reference's (248, tests/golden/fullsize/headline_conv).
    N > 1 (or --dist-selftest): z-slabs as the headline, the evolution summed
    rank to rank (ChainSum) and decided speculatively beside the next
    iteration's halo exchanges."""
    name = "headline_conv"
    steps = 10000

    def inputs(self, rank, world, strong=True):
        d = Headline.inputs(self, rank, world, strong)
        d["kw"].update(difTol=1e-5, record_dif=True)
        d["converge"] = True
        d["desc"] += ", solved to difTol 1e-5"
        return d


class HeadlineSlab8(Headline):
    """Rehearsal of one rank of the 8-GPU strong split on one GPU: the
    250x200x25 graph (1.25M vertices, 7.5M edges) every rank owns at N = 8,
    as a standalone single-GPU problem (no halo): the compute floor of an
    8-GPU iteration."""
    name = "headline_slab8"
    partitionable = False
    SHAPE = (250, 200, 25)


class HeadlineShuffled(Headline):
    """SURVEY.md §8(d) headline ordering (ii): the same graph and data with a
    random vertex relabelling and an edge shuffle (seed 7).  One GPU: the
    session relabels it internally.  N > 1: every rank computes the
    library's locality order of the whole graph (pfdr_locality_order, the
    same on every rank) and owns a range of it (random
    labels must be reordered before the split, or every edge is a halo
    edge); the sums keep the original edge ids and the caller's labels."""
    name = "headline_shuffled"

    def inputs(self, rank, world, strong=True):
        from cp_pfdr_graph_d1_amd.graphs import uniform
        d = Headline.inputs(self, 0, 1)
        kw, V, E = d["kw"], d["V"], d["E"]
        new_of = np.empty(V, np.int64)
        new_of[np.argsort(uniform(7, np.arange(V)), kind="stable")] = np.arange(V)
        eperm = np.argsort(uniform(7 * 0x9E3779B9, np.arange(E)), kind="stable")
        kw["Eu"] = new_of[kw["Eu"][eperm]].astype(np.int32)
        kw["Ev"] = new_of[kw["Ev"][eperm]].astype(np.int32)
        Y = np.empty_like(kw["Y"])
        Y[new_of] = kw["Y"]
        kw["Y"] = Y
        d["desc"] = d["desc"].replace("6-NN", "6-NN, random vertex labels + edge shuffle (seed 7)")
        if world == 1:
            return d
        from cp_pfdr_graph_d1_amd import partition as P
        order, _ = P.locality_order(V, kw["Eu"], kw["Ev"])
        off = P.vertex_offsets(V, world)
        _, nEu, nEv, parts = P.relabelled_split(order, off, kw["Eu"], kw["Ev"])
        e = parts[rank]
        v0, v1 = int(off[rank]), int(off[rank + 1])
        oi = np.asarray(order, np.int64)[v0:v1]
        kw.update(Eu=nEu[e], Ev=nEv[e], La_d1=kw["La_d1"][e], X0=kw["X0"][oi], Y=kw["Y"][oi],
                  La_l1=kw["La_l1"][oi])
        d.update(V=v1 - v0, E=e.size, kw=kw, vtx_begin=v0, e_offset=0, e_global=e,
                 vtx_label=oi)
        d["desc"] += ", locality order split into %d ranges" % world
        return d


class C1(Workload):
    """config 1: 256x256 4-NN, identity A (l22), fp64; time to tolerance"""
    name = "c1"
    metric = "PFDR_graph_quadratic_d1_l1<double> 256x256 4-NN l22: iterations/s to difTol 1e-6"
    dtype = np.float64
    edge_bytes, vertex_bytes = 80, 40
    steps = 10000
    partitionable = False

    def inputs(self, rank, world, strong=True):
        from cp_pfdr_graph_d1_amd.graphs import grid_graph, uniform
        Eu, Ev = grid_graph((256, 256), 4)
        V = 65536
        x = np.arange(V) % 256
        Y = (np.where(x < 128, 1.0, -0.5) + (2 * uniform(1, np.arange(V)) - 1) * 0.2)
        E = Eu.size
        kw = dict(Eu=Eu, Ev=Ev, La_d1=np.full(E, 0.1), X0=np.zeros(V), Y=Y,
                  La_l1=np.full(V, 0.01), rho=1.5, condMin=1e-3, difTol=1e-6,
                  Ltype=pfdr.DIAG, record_dif=True)
        return dict(V=V, E=E, kw=kw, vtx_begin=0, e_offset=0, converge=True,
                    desc="C1: 256x256 4-NN, identity A, fp64, difTol 1e-6", graph="256x256")


class C2(Workload):
    """config 2: 256^3 6-NN grid, identity A, fp32 (strong: z-slabs of the
    grid; weak: one 256^3 per GPU)"""
    name = "c2"
    metric = "PFDR_graph_quadratic_d1_l1<float> 256^3 6-NN: Medge-updates/s"
    SHAPE = (256, 256, 256)

    def inputs(self, rank, world, strong=True):
        g, V_all, v0, v1, Eu, Ev = _grid_slab(self.SHAPE, rank, world, 6, strong=strong)
        V = v1 - v0
        Y = pfdr.gen_piecewise(self.SHAPE[0], V_all, 2, np.float32, 0.2, (v0, v1))
        E = Eu.size
        kw = dict(Eu=Eu, Ev=Ev, La_d1=np.full(E, 0.1, np.float32), X0=np.zeros(V, np.float32),
                  Y=Y, La_l1=np.full(V, 0.01, np.float32), rho=1.5, condMin=1e-3)
        # edges are emitted per vertex in order: global ids are contiguous per rank
        e0 = pfdr.grid_edge_count(g, 6, v0)
        return dict(V=V, E=E, kw=kw, vtx_begin=v0, e_offset=e0,
                    desc="C2: 256^3 6-NN grid (V=%d, E=%d per GPU), identity A, fp32" % (V, E),
                    graph="%dx%dx%d" % g)


class C3(Workload):
    """config 3: dense A (N = 1024, V = 2M), fp32, single GPU (inputs on device)"""
    name = "c3"
    metric = "PFDR_graph_quadratic_d1_l1<float> dense A N=1024 V=2M: iterations/s"
    partitionable = False
    dominant = "gemv_cols"
    steps = 20

    def inputs(self, rank, world, strong=True):
        import torch
        N, nx, ny = 1024, 2000, 1000
        V = nx * ny
        g = torch.Generator(device="cuda")
        g.manual_seed(3 + rank)
        A = ((torch.rand((V, N), generator=g, device="cuda") - 0.5) * (12.0 / N) ** 0.5)
        x0 = torch.zeros(V, device="cuda")
        x0[: V // 3] = 1.0
        x0[V // 3: 2 * V // 3] = -0.5
        Y = torch.mv(A.t(), x0)
        # the caller's L = ||A||^2 with CP's settings (nTol 1e-3, 100 its,
        # 10 starts): A A^t (1024 x 1024) on the matrix cores, then the
        # batched power method (csrc/pfdr_gram.hip)
        import time
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n2, gram_ms = pfdr.operator_norm(A, nTol=1e-3, itMax=100, nbInit=10, device=True)
        norm_s = time.perf_counter() - t0
        L = torch.tensor([n2], dtype=torch.float32, device="cuda")
        Eu, Ev = pfdr.gen_grid_edges((nx, ny), 4)
        E = Eu.size
        dev = lambda a, t=torch.float32: torch.as_tensor(a, dtype=t, device="cuda")
        kw = dict(Eu=dev(Eu, torch.int32), Ev=dev(Ev, torch.int32),
                  La_d1=torch.full((E,), 0.05, device="cuda"), X0=torch.zeros(V, device="cuda"),
                  Y=Y.contiguous(), A=A.contiguous(), N=N,
                  La_l1=torch.full((V,), 0.005, device="cuda"), L=L, Ltype=pfdr.SCAL,
                  rho=1.5, condMin=1e-3, device=True)
        self._keep = (A, Y, L, kw)
        self.N = N
        gram_flop = 2.0 * N * N * V  # full product N x N
        nbt = (N + 127) // 128     # 128 x 128 MFMA block tiles, upper triangle computed
        gram_exec = 2.0 * V * 128 * 128 * nbt * (nbt + 1) // 2
        return dict(V=V, E=E, kw=kw, vtx_begin=0, e_offset=0,
                    desc="C3: dense A N=1024 x V=2M fp32 (8.2 GB), 2000x1000 4-NN, direct (N>0) "
                         "path (A^tA precomputed is V^2 = 4e12 entries: infeasible at V=2M)",
                    graph="2000x1000",
                    extra={"operator_norm": {"L": n2, "seconds": round(norm_s, 4),
                                             "gram_kernel_ms": round(gram_ms, 3),
                                             # MFMA work actually issued (triangle of tiles)
                                             "gram_TFLOPs_executed": round(gram_exec / (gram_ms * 1e-3) / 1e12, 1)
                                             if gram_ms > 0 else None,
                                             "gram_mfma_frac": round(gram_exec / (gram_ms * 1e-3) / 157.3e12, 3)
                                             if gram_ms > 0 else None,
                                             # 2 N^2 V / time: the rate a full GEMM would need
                                             "gram_TFLOPs_full_product_equiv": round(gram_flop / (gram_ms * 1e-3) / 1e12, 1)
                                             if gram_ms > 0 else None,
                                             "gram_peak_TFLOPs_f32_mfma": 157.3}})

    def kernel_bytes(self, V, E):
        # one pass over A each (R = Y - A X; P = -A^t R), + X, Ga, R; the graph
        d = Workload.kernel_bytes(self, V, E)
        d.update(gemv_cols=4 * self.N * V + 12 * V, gemv_rows=4 * self.N * V + 8 * V)
        return d

    def iteration_bytes(self, V, E):
        # two passes over A (R = Y - A X, then P = -A^t R) + the graph
        return 2 * 4 * self.N * V + self.edge_bytes * E + self.vertex_bytes * V


class C4(Workload):
    """config 4: simplex K = 10, KL al = 0.1, 2236^2 8-neighbour grid, fp32;
    N > 1: row slabs of the grid (strong) or a 2236^2 slab per GPU (weak),
    K-wide halos"""
    name = "c4"
    metric = "PFDR_graph_loss_d1_simplex<float> K=10 KL 5M-vertex 8-NN: Medge-updates/s"
    kind = pfdr.PFDR_KIND_SIMPLEX
    dominant = "sx_edge_sweep"
    pmc = "simplex"
    K = 10
    SIDE = 2236
    edge_bytes = 8 + 9 * 10 * 4
    vertex_bytes = 10 * 4 * 4
    steps = 20

    def kernel_bytes(self, V, E):
        # per (edge, label): the prox loop's 7 arrays (ref :589-634) in the
        # edge sweep, the average's Wu, Wv (ref :636-648) with the per-vertex
        # K-wide arrays in the fused vertex sweep
        s, K = self.real_bytes(), self.K
        return {"sx_edge_sweep": (8 + 7 * K * s) * E,
                "sx_vertex_sweep": 2 * K * s * E + self.vertex_bytes * V}

    def inputs(self, rank, world, strong=True):
        from cp_pfdr_graph_d1_amd.graphs import simplex_observation
        n = self.SIDE
        if strong:
            g = (n, n)
            r0, r1 = (n * rank) // world, (n * (rank + 1)) // world
        else:
            g = (n, n * world)
            r0, r1 = n * rank, n * (rank + 1)
        v0 = n * r0
        V = n * (r1 - r0)
        Eu, Ev = pfdr.gen_grid_edges(g, 8, (v0, v0 + V))
        v = np.arange(V) + (v0 if strong else 0)
        lab = ((v % n) * 4 // n) + 4 * (((v // n) % n) * 3 // n)
        Q = simplex_observation(V, self.K, 4, lab, np.float32, v0=v0)
        E = Eu.size
        kw = dict(Eu=Eu, Ev=Ev, La_d1=np.full(E, 0.05, np.float32), X0=Q.copy(), Y=Q,
                  K=self.K, al=0.1, rho=1.0, condMin=0.1)
        return dict(V=V, E=E, kw=kw, vtx_begin=v0, e_offset=pfdr.grid_edge_count(g, 8, v0),
                    desc="C4: 2236^2 8-neighbour grid (V=%d, E=%d on this GPU), K=10, KL al=0.1, "
                         "fp32" % (V, E),
                    graph="%dx%d" % g)


class C4K100(C4):
    """C4's law at K = 100 labels (one wave per vertex, k_sx_vertex_wide) on
    a 1000^2 8-neighbour grid (V = 1M, E = 4M, 400M (edge, label) entries):
    the wide simplex path's throughput, for DESIGN.md"""
    name = "c4k100"
    metric = "PFDR_graph_loss_d1_simplex<float> K=100 KL 1M-vertex 8-NN: Medge-updates/s"
    K = 100
    SIDE = 1000
    edge_bytes = 8 + 9 * 100 * 4
    vertex_bytes = 100 * 4 * 4

    def inputs(self, rank, world, strong=True):
        d = C4.inputs(self, rank, world, strong)
        d["desc"] = d["desc"].replace("2236^2", "1000^2").replace("K=10", "K=100")
        return d


class C5(Workload):
    """config 5: bounds [0,1], 640^3 6-NN, fp32, split across the GPUs
    (strong scaling: the 262M-vertex graph is fixed)"""
    name = "c5"
    metric = "PFDR_graph_quadratic_d1_bounds<float> 640^3 6-NN (1.6B directed edges): Medge-updates/s"
    kind = pfdr.PFDR_KIND_BOUNDS
    scaling = "strong"
    vertex_bytes = 16
    steps = 10
    SHAPE = (640, 640, 640)

    def inputs(self, rank, world, strong=True):
        g, V_all, v0, v1, Eu, Ev = _grid_slab(self.SHAPE, rank, world, 6, strong=True)
        V = v1 - v0
        Y = pfdr.gen_piecewise(self.SHAPE[0], V_all, 5, np.float32, 0.2, (v0, v1))
        E = Eu.size
        e0 = pfdr.grid_edge_count(g, 6, v0)
        kw = dict(Eu=Eu, Ev=Ev, La_d1=np.full(E, 0.1, np.float32), X0=np.zeros(V, np.float32),
                  Y=Y, lo=0.0, hi=1.0, rho=1.5, condMin=1e-3)
        return dict(V=V, E=E, kw=kw, vtx_begin=v0, e_offset=e0,
                    desc="C5: 640^3 6-NN grid (V=262,144,000, E=785,203,200), bounds [0,1], fp32, "
                         "%d GPU slab(s)" % world, graph="640x640x640")


class C3AtA(Workload):
    """config 3, A^tA variant ("The A^tA (N<0) variant
    runs at V=32,768"): A (N = 1024 x V = 32,768, f32) random on the device,
    A^tA = 32,768^2 f32 (4.3 GB) formed on the matrix cores (k_gram_v, the
    only MFMA-shaped step), then PFDR with N = -V; the per-iteration product
    reads the block upper triangle of the exactly symmetric matrix
    (k_symv_tiles + k_symv_finish, priced at SURVEY's V(V+1)/2 unique entries)."""
    name = "c3_ata"
    metric = "PFDR_graph_quadratic_d1_l1<float> A^tA N=-32768 (from A 1024x32768): iterations/s"
    partitionable = False
    dominant = "symv"
    steps = 50

    def inputs(self, rank, world, strong=True):
        import time
        import torch
        N, nx, ny = 1024, 256, 128
        V = nx * ny
        g = torch.Generator(device="cuda")
        g.manual_seed(3 + rank)
        # column-major N x V matrix A = (V, N) contiguous tensor
        At = ((torch.rand((V, N), generator=g, device="cuda") - 0.5) * (12.0 / N) ** 0.5)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        AtA, gram_ms = pfdr.gram(At, which=0, device=True)  # V x V, exactly symmetric
        torch.cuda.synchronize()
        gram_s = time.perf_counter() - t0
        x0 = torch.zeros(V, device="cuda")
        x0[: V // 3] = 1.0
        x0[V // 3: 2 * V // 3] = -0.5
        AtY = torch.mv(At, torch.mv(At.t(), x0))
        n2, _ = pfdr.operator_norm(At, nTol=1e-3, itMax=100, nbInit=10, device=True)
        L = torch.tensor([n2], dtype=torch.float32, device="cuda")
        Eu, Ev = pfdr.gen_grid_edges((nx, ny), 4)
        E = Eu.size
        dev = lambda a, t=torch.float32: torch.as_tensor(a, dtype=t, device="cuda")
        kw = dict(Eu=dev(Eu, torch.int32), Ev=dev(Ev, torch.int32),
                  La_d1=torch.full((E,), 0.05, device="cuda"), X0=torch.zeros(V, device="cuda"),
                  Y=AtY.contiguous(), A=AtA, N=-V,
                  La_l1=torch.full((V,), 0.005, device="cuda"), L=L, Ltype=pfdr.SCAL,
                  rho=1.5, condMin=1e-3, device=True)
        self._keep = (At, AtA, AtY, L, kw)
        nbt = (V + 127) // 128  # 128 x 128 MFMA block tiles, upper triangle computed
        gram_exec = 2.0 * N * 128 * 128 * nbt * (nbt + 1) // 2
        return dict(V=V, E=E, kw=kw, vtx_begin=0, e_offset=0,
                    desc="C3 A^tA: A 1024x32768 fp32 -> A^tA 32768^2 fp32 (4.3 GB) on the matrix "
                         "cores, 256x128 4-NN, N=-V path",
                    graph="256x128",
                    extra={"gram": {"kernel_ms": round(gram_ms, 3), "wall_s": round(gram_s, 4),
                                    "TFLOPs_executed": round(gram_exec / (gram_ms * 1e-3) / 1e12, 1)
                                    if gram_ms > 0 else None,
                                    "mfma_frac": round(gram_exec / (gram_ms * 1e-3) / 157.3e12, 3)
                                    if gram_ms > 0 else None,
                                    "full_product_TFLOP": round(2.0 * N * V * V / 1e12, 3),
                                    "peak_TFLOPs_f32_mfma": 157.3}})

    def kernel_bytes(self, V, E):
        # A^tA adds V(V+1)/2 unique entries per iteration
        d = Workload.kernel_bytes(self, V, E)
        d["symv"] = 4 * V * (V + 1) // 2 + 12 * V
        return d

    def iteration_bytes(self, V, E):
        return 4 * V * (V + 1) // 2 + self.edge_bytes * E + self.vertex_bytes * V


WORKLOADS = {w.name: w for w in (Headline(), HeadlineConv(), HeadlineSlab8(), HeadlineShuffled(),
                                  C1(), C2(), C3(),
                                  C3AtA(), C4(), C4K100(), C5())}
