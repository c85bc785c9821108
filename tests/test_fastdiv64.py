"""fp64 t/N without a division (CF64::div in fedagg.hip): q0 = RN(t*r), r = RN(1/N) from the
host, then two Markstein corrections q <- RN(q + RN(t - q*N)*r) computed with FMAs.

The claim is that the result equals RN(t/N) for |t| in [2^-600, 2^600] and
|N| in [2^-60, 2^60]. f64 cannot be enumerated, so the tests aim at where it could fail:
quotients constructed to lie as close to a rounding midpoint as a quotient of two doubles
can (|t/N - mid| = |d| / (N * 2^s), i.e. ~2^-k ulp for a k-bit odd N), quotients next to
representable values, and random operands over the whole guarded exponent range.

* CPU (`not gpu`): the exact instruction sequence emulated with rationals (every FMA /
  product rounded once by Python's correctly rounded int/Fraction -> float conversion),
  against Python's correctly rounded t / N.
* GPU: the fused FedAvg kernel computing 0 + (1*(t - 0))/N with the shortcut vs numpy's
  t / N, and vs the kernel's own IEEE division on random operands (fa_tune fastdiv64=0 in libfedagg_probe.so).
"""
import math
from fractions import Fraction

import numpy as np
import pytest


def _rn(fr):
    """Round a rational to the nearest double (ties to even), as an FMA does."""
    return float(fr) if fr.denominator != 1 else float(int(fr))


def _fma(a, b, c):
    return _rn(Fraction(a) * Fraction(b) + Fraction(c))


def emulate(t, N):
    r = 1.0 / N
    q = _rn(Fraction(t) * Fraction(r))
    e = _fma(-q, N, t)
    q = _fma(e, r, q)
    e = _fma(-q, N, t)
    return _fma(e, r, q)


def hard_cases(rng, n_div, per_div, kmax=52):
    """{N: [t, ...]} whose quotients t/N sit within |d|/(N_odd*2^s) of a binary64 rounding
    midpoint M/2^s (M odd, 54 bits): the closest a quotient of two doubles can get."""
    out = {}
    while len(out) < n_div:
        k = int(rng.integers(1, kmax + 1))
        Nodd = int(rng.integers(1 << (k - 1), 1 << k)) | 1           # odd, k bits
        s = k + 1
        shN = int(rng.integers(0, 8))
        ts = []
        tries = 0
        while len(ts) < per_div and tries < 20 * per_div:
            tries += 1
            d = int(rng.choice([-3, -1, 1, 3]))
            base = (-d * pow(Nodd, -1, 1 << s)) % (1 << s)            # M = base (mod 2^s), odd
            M = (1 << 53) + int(rng.integers(0, 1 << 52)) * 2
            M = M - (M % (1 << s)) + base
            if M < (1 << 53) or M >= (1 << 54):
                continue
            T = (M * Nodd + d) >> s                                   # exact: M*N + d = 0 (mod 2^s)
            if T >= (1 << 53) or T <= 0:
                continue
            sh = int(rng.integers(-40, 41))                           # scale t and N independently
            ts.append(math.ldexp(float(T), sh) * (1 if rng.random() < 0.5 else -1))
        out[float(Nodd << shN)] = ts
    return out


def near_exact_cases(rng, n_div, per_div):
    """{N: [t, ...]} with t = RN(q*N) moved by -2..2 ulps: quotients next to representable values."""
    out = {}
    for _ in range(n_div):
        N = float(int(rng.integers(1, 1 << int(rng.integers(1, 53)))))
        ts = []
        for _ in range(per_div):
            t = float(rng.standard_normal()) * 2.0 ** int(rng.integers(-30, 30)) * N
            k = int(rng.integers(-2, 3))
            for _ in range(abs(k)):
                t = float(np.nextafter(t, np.inf if k > 0 else -np.inf))
            ts.append(t)
        out[N] = ts
    return out


def _flat(*dicts):
    return [(t, N) for d in dicts for N, ts in d.items() for t in ts]


def test_emulated_fastdiv64_hard_cases():
    rng = np.random.default_rng(64)
    cases = _flat(hard_cases(rng, 300, 20), near_exact_cases(rng, 100, 20))
    bad = [(t, N) for t, N in cases if emulate(t, N) != t / N]
    assert not bad, f"{len(bad)} mismatches, e.g. {bad[:3]}"


def test_hard_case_construction_is_hard():
    """The constructed quotients really are within 2^-k ulp of a midpoint (the generator is sound)."""
    rng = np.random.default_rng(5)
    for t, N in _flat(hard_cases(rng, 50, 4)):
        Nodd = int(N)
        while not Nodd & 1:
            Nodd >>= 1
        z = Fraction(t) / Fraction(N)
        q = t / N
        ulp = Fraction(math.ulp(q))
        dist = abs(abs(z - Fraction(q)) - ulp / 2)
        assert 0 < dist <= 3 * ulp / (2 * Nodd)


@pytest.mark.gpu
def test_gpu_fastdiv64_vs_numpy():
    import torch

    from fedn_amd import ops
    rng = np.random.default_rng(6464)
    dev = "cuda:0"
    nbad = ntot = 0          # the product library: its fp64 division is the corrected reciprocal
    # one launch per divisor (N is per client step), 400 + 100 divisors x 256 quotients
    for N, tl in {**hard_cases(rng, 400, 256), **near_exact_cases(rng, 100, 256)}.items():
        tt = torch.tensor(tl, dtype=torch.float64, device=dev)
        z = torch.zeros_like(tt)
        a = torch.empty_like(tt)
        ops.fedavg_fold(a, [z, tt], [0, 1], [1, N], init=True)
        want = np.array(tl) / N + 0.0
        nbad += int((a.cpu().numpy().view(np.uint64) != want.view(np.uint64)).sum())
        ntot += len(tl)
    assert ntot > 100_000 and nbad == 0, f"{nbad} of {ntot} differ from numpy's t / N"


@pytest.mark.gpu
def test_gpu_fastdiv64_random_vs_ieee():
    import torch

    from fedn_amd import _abi, ops
    dev = "cuda:0"
    n = 1 << 24
    g = torch.Generator(device=dev).manual_seed(99)
    # random bit patterns over every exponent (guards: tiny / huge / inf / NaN take IEEE division)
    bits = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, device=dev, dtype=torch.int64)
    t_all = bits.view(torch.float64)
    # and dense in the guarded range
    mant = torch.rand(n, generator=g, device=dev, dtype=torch.float64) + 1.0
    ex = torch.randint(-650, 651, (n,), generator=g, device=dev)
    t_rng = torch.ldexp(mant, ex) * torch.where(torch.rand(n, generator=g, device=dev) < 0.5, -1.0, 1.0)
    z = torch.zeros(n, dtype=torch.float64, device=dev)
    a = torch.empty(n, dtype=torch.float64, device=dev)
    b = torch.empty(n, dtype=torch.float64, device=dev)
    divisors = [1, 2, 3, 7, 10, 4999, 5000, 65537, 1_000_003, (1 << 24) + 1, 123_456_789, (1 << 40) + 15,
                (1 << 52) - 1, (1 << 53) - 1, 2.0 ** 60, 2.0 ** 61, 0.5, 3.0 * 2 ** -61, 1e-300, -7, 0]
    divisors += [int(v) for v in np.random.default_rng(7).integers(1, 1 << 53, 8)]
    bad = {}
    try:
        for t in (t_all, t_rng):
            for N in divisors:
                ops.fedavg_fold(a, [z, t], [0, 1], [1, N], init=True)        # product libfedagg.so
                with _abi.use_probe():                                      # IEEE division, probe build
                    ops.tune(fastdiv64=0)
                    ops.fedavg_fold(b, [z, t], [0, 1], [1, N], init=True)
                diff = (a.view(torch.int64) != b.view(torch.int64)) & ~(torch.isnan(a) & torch.isnan(b))
                nd = int(diff.sum())
                if nd:
                    bad[N] = bad.get(N, 0) + nd
    finally:
        with _abi.use_probe():
            ops.tune(fastdiv64=1)
    assert not bad, f"fp64 fast division differs from IEEE division: {bad}"
