"""sha256 over the HIP sources the bench's kernels are compiled from
(cp_pfdr_graph_d1_amd/csrc/*.hip, *.hpp, sorted by name): recorded by
tools/pmc_traffic.py next to the PMC traffic it summarises, compared by
bench.py before it reports that traffic (a stale summary reports null)."""
import glob
import hashlib
import os

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def kernel_source_sha256():
    h = hashlib.sha256()
    for f in sorted(glob.glob(os.path.join(ROOT, "cp_pfdr_graph_d1_amd", "csrc", "*.hip")) +
                    glob.glob(os.path.join(ROOT, "cp_pfdr_graph_d1_amd", "csrc", "*.hpp"))):
        h.update(os.path.basename(f).encode())
        h.update(open(f, "rb").read())
    return h.hexdigest()


if __name__ == "__main__":
    print(kernel_source_sha256())
