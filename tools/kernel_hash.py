"""sha256 over the HIP sources a solver's kernels are compiled from, sorted by
name: "quadratic" (the headline and C1/C2/C3/C5 workloads: edge / vertex
sweeps, reductions, setup kernels) -- pfdr_quadratic.hip and every header it
includes, plus the incidence (pfdr_graph.hip), relabelling (pfdr_order.hip)
and sequential-sum (pfdr_monosum.hip) translation units its setup launches;
"simplex" (C4) -- pfdr_simplex.hip with the same shared units.
Recorded by tools/pmc_traffic.py next to the PMC traffic it summarises and
compared by bench.py before it reports that traffic (a summary taken on
other kernel sources reports null).  Sources of unrelated kernels (CP graph
steps, Gram, simplex, halo transport) and the C ABI declarations
(include/pfdr_mi355x.h, no device code) do not enter: changing them leaves
the headline's kernels, and so their traffic, as they were."""
import hashlib
import os

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
COMMON = ("pfdr_dev.hpp", "pfdr_graph.hip", "pfdr_graph.hpp", "pfdr_halo.hpp",
          "pfdr_monosum.hip", "pfdr_monosum.hpp", "pfdr_session.hpp")
SOURCES = {
    "quadratic": COMMON + ("pfdr_order.hip", "pfdr_order.hpp", "pfdr_quadratic.hip",
                           "pfdr_quadratic_kernels.hpp"),
    "simplex": COMMON + ("pfdr_simplex.hip",),
}


def kernel_source_sha256(solver="quadratic"):
    h = hashlib.sha256()
    for name in sorted(SOURCES[solver]):
        h.update(name.encode())
        h.update(open(os.path.join(ROOT, "cp_pfdr_graph_d1_amd", "csrc", name), "rb").read())
    return h.hexdigest()


if __name__ == "__main__":
    import sys
    print(kernel_source_sha256(*sys.argv[1:2]))
