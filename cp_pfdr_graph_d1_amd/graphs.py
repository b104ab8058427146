"""Seeded synthetic inputs for the PFDR solvers.

The reference ships no datasets (data/EEG.mat is missing,
/root/reference/.MISSING_LARGE_BLOBS:1), so every test and benchmark input is
generated here, deterministically, from a counter-based splitmix64 stream:

* ``grid_graph(shape, conn)``: 2-D 4/8-neighbour or 3-D 6/26-neighbour grids,
  vertex ``v = x + nx*(y + ny*z)``, edges emitted per vertex in lexicographic
  order (+x, +y, +z, then diagonals) — the layout the CP drivers hand to PFDR
  (undirected, each edge once, ``Eu < Ev`` not required by the solver);
* ``knn_jitter_grid(shape, k)``: the headline graph — a jittered grid where
  each vertex emits its k nearest neighbours inside its 26-neighbourhood as
  (v, nn) pairs, so E = k·V exactly, mirrored duplicates kept (the reference
  accepts multi-edges);
* ``piecewise_observation``: Y = (x < nx/2 ? 1 : -0.5) + U(-0.2, 0.2).

The large headline graph is produced by the native generator of the C-ABI
library (``pfdr_gen_knn_jitter_grid``), which implements the same law; tests
check the two agree on small shapes.
"""
import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_SEEDMUL = np.uint64(0xD1B54A32D192ED03)


def splitmix64(x):
    """Vectorised splitmix64 finaliser on uint64 arrays (wrapping)."""
    with np.errstate(over="ignore"):
        z = (np.asarray(x, np.uint64) + _GOLD)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform(seed, index):
    """U[0,1) float64 for counter ``index`` of stream ``seed``."""
    with np.errstate(over="ignore"):
        x = np.uint64(seed) * _SEEDMUL + np.asarray(index, np.uint64)
    return (splitmix64(x) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def _offsets(ndim, conn):
    if ndim == 2 and conn == 4:
        return [(1, 0), (0, 1)]
    if ndim == 2 and conn == 8:
        return [(1, 0), (0, 1), (1, 1), (-1, 1)]
    if ndim == 3 and conn == 6:
        return [(1, 0, 0), (0, 1, 0), (0, 0, 1)]
    if ndim == 3 and conn == 26:
        offs = []
        for dz in (-1, 0, 1):
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    o = (dx, dy, dz)
                    # keep one of each +-pair: lexicographically positive
                    if (dz, dy, dx) > (0, 0, 0):
                        offs.append(o)
        return offs
    raise ValueError("unsupported grid connectivity %s for %d-D" % (conn, ndim))


def grid_graph(shape, conn):
    """Edges (Eu, Ev) int32 of a 2-D/3-D grid, emitted per vertex, in the
    order of ``_offsets``; vertex index x fastest."""
    shape = tuple(int(s) for s in shape)
    ndim = len(shape)
    offs = _offsets(ndim, conn)
    coords = np.indices(shape[::-1]).reshape(ndim, -1)[::-1]  # x, y, (z)
    V = int(np.prod(shape))
    vid = np.arange(V, dtype=np.int64)
    strides = [1]
    for s in shape[:-1]:
        strides.append(strides[-1] * s)
    Eu_l, Ev_l, ok_l = [], [], []
    for o in offs:
        ok = np.ones(V, bool)
        nb = vid.copy()
        for d in range(ndim):
            c = coords[d] + o[d]
            ok &= (c >= 0) & (c < shape[d])
            nb += o[d] * strides[d]
        Eu_l.append(vid)
        Ev_l.append(nb)
        ok_l.append(ok)
    Eu = np.stack(Eu_l, 1).ravel()
    Ev = np.stack(Ev_l, 1).ravel()
    ok = np.stack(ok_l, 1).ravel()
    return Eu[ok].astype(np.int32), Ev[ok].astype(np.int32)


def _nbr26():
    offs = []
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                if (dx, dy, dz) != (0, 0, 0):
                    offs.append((dx, dy, dz))
    return offs


def knn_jitter_grid(shape, k=6, seed=6, jitter=0.25, vertex_range=None):
    """Headline k-NN graph (SURVEY.md §8(d) 'Headline').

    Points p_v = grid(v) + U(-jitter, jitter)^3 with U drawn from stream
    ``seed`` at counters 3v, 3v+1, 3v+2.  Vertex v emits (v, nn) for its k
    nearest 26-neighbours (Euclidean in float64; ties broken by the
    neighbour enumeration order dz, dy, dx ascending).  Edge e = k*v + j.
    ``vertex_range=(v0, v1)`` returns only the edges of those emitters.
    """
    nx, ny, nz = (int(s) for s in shape)
    V = nx * ny * nz
    v0, v1 = (0, V) if vertex_range is None else vertex_range
    v = np.arange(v0, v1, dtype=np.int64)
    x, y, z = v % nx, (v // nx) % ny, v // (nx * ny)

    def point(vv, xx, yy, zz):
        base = 3 * vv
        px = xx + (2.0 * uniform(seed, base) - 1.0) * jitter
        py = yy + (2.0 * uniform(seed, base + 1) - 1.0) * jitter
        pz = zz + (2.0 * uniform(seed, base + 2) - 1.0) * jitter
        return px, py, pz

    px, py, pz = point(v, x, y, z)
    offs = _nbr26()
    dist = np.full((v.size, 26), np.inf)
    nbr = np.zeros((v.size, 26), np.int64)
    for j, (dx, dy, dz) in enumerate(offs):
        xx, yy, zz = x + dx, y + dy, z + dz
        ok = (xx >= 0) & (xx < nx) & (yy >= 0) & (yy < ny) & (zz >= 0) & (zz < nz)
        w = xx + nx * (yy + ny * zz)
        qx, qy, qz = point(w, xx, yy, zz)
        d = (px - qx) ** 2 + (py - qy) ** 2 + (pz - qz) ** 2
        dist[:, j] = np.where(ok, d, np.inf)
        nbr[:, j] = w
    order = np.argsort(dist, axis=1, kind="stable")[:, :k]
    Ev = np.take_along_axis(nbr, order, 1)
    Eu = np.repeat(v, k)
    return Eu.astype(np.int32), Ev.ravel().astype(np.int32)


def piecewise_observation(shape, seed, dtype=np.float64, noise=0.2):
    """Y = (x < nx/2 ? 1.0 : -0.5) + U(-noise, noise) at counter v."""
    V = int(np.prod(shape))
    v = np.arange(V, dtype=np.int64)
    x = v % int(shape[0])
    base = np.where(x < int(shape[0]) // 2, 1.0, -0.5)
    return (base + (2.0 * uniform(seed, v) - 1.0) * noise).astype(dtype)


def simplex_observation(V, K, seed, block_labels, dtype=np.float64, v0=0):
    """Q = normalise(U(0,1) + 3*onehot(label)), column v = Q[v*K:(v+1)*K];
    v0: first global vertex (the draws of a partition slab)."""
    idx = int(v0) * K + np.arange(V * K, dtype=np.int64)
    Q = uniform(seed, idx).reshape(V, K)
    Q[np.arange(V), np.asarray(block_labels) % K] += 3.0
    Q /= Q.sum(1, keepdims=True)
    return Q.ravel().astype(dtype)
