"""GPU: the workgroup sum of nonnegative terms (pfdr_monosum.hpp) rounds
exactly as the one-thread loop of the reference's amplitude sum
(src/PFDR_graph_quadratic_d1_l1.cpp:146-152): compared bit for bit with
numpy's cumulative sum (strictly sequential) and with the one-lane kernel,
on inputs built to hit every rounding case — exact halves with both
parities, runs that stall the sum (x + 1 = x at 2^24), subnormals, zeros,
terms far above the running sum, overflow to inf, tile and binade
boundaries, a nonzero seed (the running sum of the lower ranks)."""
import numpy as np
import pytest

from cp_pfdr_graph_d1_amd import pfdr

pytestmark = pytest.mark.gpu


def _seq(a, seed):
    a = np.asarray(a)
    if a.size == 0:
        return a.dtype.type(seed)
    return np.cumsum(np.concatenate([np.array([seed], a.dtype), a]))[-1]


def _cases(dt):
    rng = np.random.default_rng(7)
    f = np.dtype(dt).type
    p = 24 if dt == np.float32 else 53
    out = {
        "empty": np.zeros(0, dt),
        "one": np.array([3.25], dt),
        "zeros": np.zeros(70000, dt),
        "uniform_1k": rng.random(1000).astype(dt),
        "uniform_3M": rng.random(3_000_001).astype(dt),
        "lognormal": np.exp(rng.normal(0, 8, 500_000)).astype(dt),
        "halves": (rng.integers(0, 8, 400_000) * 0.5 + 2.0 ** -3).astype(dt),
        "ints_past_2p": np.full(2 ** 20 + 3, 2.0 ** (p - 20), dt),  # reaches 2^p, stalls
        "ties_both_parities": np.tile(np.array([1.0, 0.5, 1.5, 2.5, 0.25], dt), 100_000),
        "subnormal": np.full(50_000, np.finfo(dt).smallest_subnormal, dt),
        "mixed_scales": np.concatenate([np.full(1000, 1e-30, dt), np.full(1000, 1.0, dt),
                                        np.full(1000, 1e-30, dt), np.array([1e20], dt),
                                        rng.random(5000).astype(dt)]),
        "big_first": np.concatenate([np.array([1e25], dt), rng.random(100_000).astype(dt)]),
        "overflow": np.concatenate([rng.random(1000).astype(dt),
                                    np.full(4, np.finfo(dt).max / 3, dt),
                                    rng.random(1000).astype(dt)]),
        "tile_edges": rng.random(8192 * 3 + 17).astype(dt) * f(2.0 ** 10),
        # more tiles than one chain step of the walk holds (512), and a
        # binade crossing in almost every tile (geometric growth)
        "uniform_6M": rng.random(6_000_003).astype(dt),
        "geometric": np.geomspace(1e-20, 1e10, 3_000_000).astype(dt),
        "loguniform_wide": np.exp(rng.uniform(np.log(1e-30), 0.0, 2_000_000)).astype(dt),
    }
    if dt == np.float32:
        out["stall_2p24"] = np.ones(2 ** 24 + 1000, dt)
    return out


@pytest.mark.parametrize("dt", [np.float32, np.float64], ids=["f32", "f64"])
def test_sequential_sum_bitexact(gpu_lib, dt):
    for name, a in _cases(dt).items():
        for seed in (0.0, 1234.5):
            want = _seq(a, seed)
            got, _ = pfdr.sequential_sum(a, seed, method=0)
            lane, _ = pfdr.sequential_sum(a, seed, method=1) if a.size < 4_000_000 else (want, 0)
            assert (np.isinf(want) and got == want) or got == want, (name, seed, got, want)
            assert lane == want or (np.isinf(want) and lane == want), (name, seed, lane, want)
