"""The exact 3-part bf16 cut behind the fp32 split products (csrc/kernels/common.h ``Mma<float>::split3`` /
``mma_psb``), emulated bit for bit in numpy: conv1's forward, the FC head at >= 32-row tiles and the fp32 weight
gradients run their products as three ``v_mfma_f32_16x16x32_bf16`` on these parts instead of
``v_mfma_f32_16x16x4_f32``.  The GPU side is covered by the fp32 tolerance tests of ``tests/test_native_gpu.py``
(training steps against the PyTorch fp32 reference of the reference's step, ``/root/reference/ddp_tutorial_multi_gpu.py:75``);
this pins the arithmetic those kernels rely on."""
import numpy as np

HI_MASK = np.uint32(0xFFFF0000)


def split3(x: np.ndarray):
    """hi = top 16 bits of x, mid = top 16 bits of the (exact) remainder, lo = what is left (as common.h)."""
    x = np.asarray(x, dtype=np.float32)
    hi = (x.view(np.uint32) & HI_MASK).view(np.float32)
    r1 = (x - hi).astype(np.float32)
    mid = (r1.view(np.uint32) & HI_MASK).view(np.float32)
    lo = (r1 - mid).astype(np.float32)
    return hi, mid, lo


def _values(rng, n):
    mant = rng.uniform(-1.0, 1.0, n)
    exp = rng.integers(-60, 60, n)
    return (mant * np.exp2(exp)).astype(np.float32)


def test_split_is_exact_and_bf16_representable():
    rng = np.random.default_rng(0)
    x = np.concatenate([_values(rng, 200_000),
                        np.array([0.0, -0.0, 1.0, -1.0, 3.0e38, -3.0e38, 1.17549435e-38, np.float32(1) / 3],
                                 dtype=np.float32)])
    hi, mid, lo = split3(x)
    for part in (hi, mid, lo):  # every part is a bf16 value: its low 16 bits are zero
        assert not np.any(part.view(np.uint32) & np.uint32(0xFFFF))
    # x == hi + mid + lo exactly (checked in float64, where the sum of the three parts cannot round)
    s = hi.astype(np.float64) + mid.astype(np.float64) + lo.astype(np.float64)
    assert np.array_equal(s, x.astype(np.float64))
    # magnitudes: mid below 2^-7 |x|, lo below 2^-15 |x| (8 significant bits per part)
    nz = x != 0
    ax = np.abs(x[nz]).astype(np.float64)
    assert np.all(np.abs(mid[nz]) <= ax * 2.0 ** -7)
    assert np.all(np.abs(lo[nz]) <= ax * 2.0 ** -15)


def _six_products(a, b):
    """The per-lane sum of the three MFMAs of mma_psb, in float64: [ah|al].[bl|bh] + [ah|am].[bm|bm] + [ah|am].[bh|bh]."""
    ah, am, al = (p.astype(np.float64) for p in split3(a))
    bh, bm, bl = (p.astype(np.float64) for p in split3(b))
    return (ah * bl + al * bh) + (ah * bm + am * bm) + (ah * bh + am * bh)


def test_six_products_error_bound():
    rng = np.random.default_rng(1)
    a = rng.standard_normal(100_000).astype(np.float32)
    b = rng.standard_normal(100_000).astype(np.float32)
    exact = a.astype(np.float64) * b.astype(np.float64)
    err = np.abs(_six_products(a, b) - exact) / np.abs(exact)
    # the dropped terms mid*lo + lo*mid + lo*lo are below 2^-21 of |a b| in the worst case ...
    assert err.max() <= 2.0 ** -21
    # ... and ~2^-24 typically (fp32's own rounding unit is 2^-24)
    assert np.median(err) <= 2.0 ** -24


def test_chunk_dot_matches_fp32():
    """A 16-k chunk (one lane group's k-slots of one MFMA tile): the split dot product is as close to the exact
    dot product as an fp32 dot product with fp32 accumulation is."""
    rng = np.random.default_rng(2)
    a = rng.standard_normal((4096, 16)).astype(np.float32)
    b = rng.standard_normal((4096, 16)).astype(np.float32)
    exact = np.sum(a.astype(np.float64) * b.astype(np.float64), axis=1)
    split = np.sum(_six_products(a, b), axis=1).astype(np.float32)
    acc32 = np.zeros(4096, dtype=np.float32)
    for k in range(16):
        acc32 = (acc32 + a[:, k] * b[:, k]).astype(np.float32)
    scale = np.sum(np.abs(a.astype(np.float64) * b), axis=1)
    assert np.max(np.abs(split - exact) / scale) <= np.max(np.abs(acc32 - exact) / scale) * 2 + 2.0 ** -24


def test_non_finite_operands_give_nan_products():
    """Documented divergence from fp32 MFMA (PARITY.md N1): an infinite operand is cut into hi = inf and an
    inf - inf = NaN remainder, so its split product is NaN where the exact fp32 product is +-inf.  Both are
    non-finite, and the run's non-finite-loss guard (engine/runner.py check_finite) fires either way; a finite
    overflow-free training step never produces an infinite operand (the tolerance tests only see finite values)."""
    x = np.array([np.inf, -np.inf, np.nan, 1.0], dtype=np.float32)
    with np.errstate(invalid="ignore"):
        hi, mid, lo = split3(x)
        prod = _six_products(x, np.full(4, 2.0, dtype=np.float32))
    assert np.isinf(hi[0]) and np.isnan(mid[0]) and np.isnan(mid[2])
    assert np.all(np.isnan(prod[:3])) and prod[3] == 2.0
    assert not np.any(np.isfinite(prod[:3]))  # non-finite either way: the guard sees it
