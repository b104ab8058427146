"""CPU: the numerics the split Gram tile (k_gram_b, csrc/pfdr_gram.hip) rests
on, restated in numpy with the kernel's bit operations: every f32 x splits
EXACTLY into three bf16 pieces x = h + m + l (h = x truncated to 8
significant bits, m = x - h rounded to nearest even at 8, l = x - h - m), and
a product x y formed from the six pieces hh, hm, mh, hl, lh, mm -- each exact
in f32 -- differs from the exact product by the three pieces left out (ml,
lm, ll), at most ~2^-21 of |x y|: at the f32 rounding of the Gram's sums,
which the GPU test (tests/test_gram_gpu.py) holds to 2e-6 relative
Frobenius."""
import numpy as np


def bf16_rne(x):
    """the kernel's bf16_rne: round the f32 bit pattern to its top 16 bits,
    to nearest even"""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFFFFFF) >> 16
    return u.astype(np.uint32)


def bf16_val(h):
    return (h.astype(np.uint32) << 16).view(np.float32)


def bf16_trunc(x):
    """the kernel's leading piece: the top 16 bits of x"""
    return (np.asarray(x, np.float32).view(np.uint32) >> 16).astype(np.uint32)


def split3(x):
    x = np.asarray(x, np.float32)
    h = bf16_val(bf16_trunc(x))
    r1 = (x - h).astype(np.float32)
    m = bf16_val(bf16_rne(r1))
    r2 = (r1 - m).astype(np.float32)
    l = bf16_val(bf16_rne(r2))
    return h, m, l, r2


def _samples(n=200000, seed=11):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal(n).astype(np.float32)
    x *= np.float32(2.0) ** rng.integers(-60, 60, n).astype(np.float32)
    edge = np.array([1.0, -1.0, 0.0, 3.4028235e38, -3.4028235e38, 1.1754944e-38 * 2 ** 24,
                     np.nextafter(np.float32(1), np.float32(2)), 0.1, -0.3, 1 / 3],
                    np.float32)
    return np.concatenate([x, edge])


def test_split_is_exact():
    x = _samples()
    h, m, l, r2 = split3(x)
    # the last piece takes the rest without rounding ...
    assert np.array_equal(l, r2)
    # ... so the three pieces add back to x exactly (in f64, no rounding)
    assert np.array_equal(h.astype(np.float64) + m + l, x.astype(np.float64))
    # and each piece has at most 8 significant bits
    for p in (h, m, l):
        assert np.array_equal(bf16_val(bf16_rne(p)), p)


def test_six_piece_product_error_below_f32_rounding():
    rng = np.random.default_rng(5)
    x = rng.uniform(-1, 1, 100000).astype(np.float32)
    y = rng.uniform(-1, 1, 100000).astype(np.float32)
    hx, mx, lx, _ = split3(x)
    hy, my, ly, _ = split3(y)
    f64 = lambda a: a.astype(np.float64)
    six = (f64(hx) * f64(hy) + f64(hx) * f64(my) + f64(mx) * f64(hy) + f64(hx) * f64(ly)
           + f64(lx) * f64(hy) + f64(mx) * f64(my))
    exact = f64(x) * f64(y)
    rel = np.abs(six - exact) / np.maximum(np.abs(exact), 1e-300)
    assert rel.max() <= 2.0 ** -21          # the three dropped pieces
    assert np.median(rel) <= 2.0 ** -24     # typically far below f32's ulp
    # every piece product is exact in f32 (8 x 8 significant bits)
    for a, b in ((hx, hy), (hx, my), (mx, hy), (hx, ly), (lx, hy), (mx, my)):
        assert np.array_equal((a * b).astype(np.float64), f64(a) * f64(b))
