"""End-to-end cut-pursuit timing: one of the reference's CP drivers
(src/CP_PFDR_graph_*.cpp, compiled unchanged by oracle/Makefile)
linked with the reference PFDR (CPU, sequential PFDR objects as in the parity
test) and with libpfdr_mi355x.so (the drop-in).  Prints one JSON line per
problem: CP wall times of both builds, whether the CP outputs are
identical, and (PFDR_TRACE=1) the drop-in's per-call setup / iterate /
copy-back split.

    python tools/cp_time.py [--shapes 256x256,512x512] [--dtype f32] [--kind l1 --mode diag]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
REF = os.path.join(ROOT, "oracle", "_ref")


def write_problem(path, shape, dt, kind="l1", mode="diag"):
    """in.bin of oracle/harness/cp_drivers.cpp (tests/cp_problems.py)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cp_problems as P
    p = P.problem(kind, mode, dt, nx=shape[0], ny=shape[1])
    P.write(path, p)
    return p["V"], p["E"]


def run(drv, inp, out, env=None):
    p = subprocess.run([drv, inp, out], capture_output=True, text=True, timeout=900,
                       env=dict(os.environ, **(env or {})))
    if p.returncode:
        raise RuntimeError("%s failed: %s" % (drv, p.stderr[-2000:]))
    m = re.search(r"cp_time_s=([0-9.]+) rV=(\d+) CP_it=(\d+)", p.stderr)
    calls = [dict(re.findall(r"(\w+)=([0-9.]+)", l)) for l in p.stderr.splitlines()
             if l.startswith("[pfdr]")]
    return float(m.group(1)), int(m.group(2)), int(m.group(3)), calls, open(out, "rb").read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="256x256,512x512,1024x1024")
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--kind", default="l1", help="l1, duplex, bounds or simplex")
    ap.add_argument("--mode", default="diag", help="diag, identity, direct, AtA")
    args = ap.parse_args()
    dt = np.float64 if args.dtype == "f64" else np.float32
    tmp = tempfile.mkdtemp()
    for sh in args.shapes.split(","):
        shape = tuple(int(x) for x in sh.split("x"))
        inp = os.path.join(tmp, "in.bin")
        V, E = write_problem(inp, shape, dt, args.kind, args.mode)
        t_ref, rv, it, _, o_ref = run(os.path.join(REF, "cp_%s_ref" % args.kind), inp,
                                      os.path.join(tmp, "o1"))
        t_gpu, rv2, it2, calls, o_gpu = run(os.path.join(REF, "cp_%s_mi355x" % args.kind), inp,
                                            os.path.join(tmp, "o2"), {"PFDR_TRACE": "1"})
        s = lambda k: round(sum(float(c[k]) for c in calls), 3)
        print(json.dumps({
            "shape": sh, "kind": args.kind, "mode": args.mode, "dtype": args.dtype, "V": V, "E": E, "rV": rv, "CP_it": it,
            "identical": o_ref == o_gpu and (rv, it) == (rv2, it2),
            "cp_ref_cpu_s": t_ref, "cp_mi355x_s": t_gpu,
            "pfdr_calls": len(calls),
            "pfdr_calls_detail": [{k: c[k] for k in ("V", "E", "it", "total_ms")} for c in calls],
            "pfdr_setup_ms": s("setup_ms"), "pfdr_run_ms": s("run_ms"),
            "pfdr_copy_ms": s("copy_ms"), "pfdr_total_ms": s("total_ms")}), flush=True)


if __name__ == "__main__":
    main()
