"""Load the golden fixtures and replay them through any back-end that has
the oracle's calling convention (oracle.Oracle or cp_pfdr_graph_d1_amd.pfdr.Lib)."""
import glob
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXED_K = 25


def names(prefix=""):
    out = []
    for p in sorted(glob.glob(os.path.join(GOLD, "*.npz"))):
        n = os.path.basename(p)[:-4]
        if n.startswith("cp_"):  # CP graph-step fixtures: test_cp_graph_*.py
            continue
        if n.startswith(prefix):
            out.append(n)
    return out


def load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    inp, out = {}, {}
    for k in z.files:
        v = z[k]
        if k.startswith("in_"):
            inp[k[3:]] = v.item() if v.ndim == 0 and k[3:] not in ("X0", "P0") else v
        else:
            out[k] = v
    for k in ("La_l1", "A", "L", "La_f"):
        inp.setdefault(k, None)
    return inp, out


def replay(lib, c, fixed, obj=True, dif=True):
    kw = dict(difTol=0.0, difRcd=0.0, itMax=FIXED_K) if fixed else {}
    a = dict(c, **kw)
    s = str(a["solver"])
    if s == "l1":
        return lib.quadratic_d1_l1(
            a["X0"], a["Y"], a["A"], int(a["N"]), a["Eu"], a["Ev"], a["La_d1"],
            a["La_l1"], int(a["positivity"]), int(a["Ltype"]), a["L"],
            float(a["rho"]), float(a["condMin"]), float(a["difRcd"]),
            float(a["difTol"]), int(a["itMax"]), obj=obj, dif=dif)
    if s == "bounds":
        return lib.quadratic_d1_bounds(
            a["X0"], a["Y"], a["A"], int(a["N"]), a["Eu"], a["Ev"], a["La_d1"],
            float(a["lo"]), float(a["hi"]), int(a["Ltype"]), a["L"],
            float(a["rho"]), float(a["condMin"]), float(a["difRcd"]),
            float(a["difTol"]), int(a["itMax"]), obj=obj, dif=dif)
    if s == "simplex":
        return lib.loss_d1_simplex(
            a["P0"], a["Q"], int(a["K"]), a["Eu"], a["Ev"], a["La_d1"],
            float(a["al"]), a["La_f"], float(a["rho"]), float(a["condMin"]),
            float(a["difRcd"]), float(a["difTol"]), int(a["itMax"]), obj=obj,
            dif=dif)
    raise ValueError(s)


def rel_l2(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)
