"""Exhaustive check of the fp32 division shortcut (CF32::fold_strip in fedagg.hip).

For every binary32 bit pattern t (all 2^32, NaNs and infinities included) and a set of
divisors N, the fused FedAvg kernel computes x + (1*(t - x))/N with x = 0, i.e. RN(t/N)
(then 0 + q). We run it once with the RN64(1/N)-product shortcut and once with IEEE
division (fa_tune fastdiv=0 in libfedagg_probe.so, itself pinned to numpy by the golden tests) and require
bit-identical outputs.
"""
import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

DIVISORS = [1, 2, 3, 5, 7, 10, 100, 127, 1000, 1023, 1025, 4096, 4999, 5000, 9973, 65535, 65537, 1_000_003,
            (1 << 24) - 1, 1 << 24, (1 << 24) + 2, 123_456_789, (1 << 27) + 12345, 3 << 25, (1 << 28) - 16,
            1 << 28, 0]
DIVISORS += [int(v) for v in np.random.default_rng(1234).integers(1, 1 << 24, 8)]


def test_fastdiv_exhaustive():
    from fedn_amd import _abi, ops
    dev = "cuda:0"
    chunk = 1 << 28
    zeros = torch.zeros(chunk, dtype=torch.float32, device=dev)
    a = torch.empty(chunk, dtype=torch.float32, device=dev)
    b = torch.empty(chunk, dtype=torch.float32, device=dev)
    bad = {}
    try:
        for c in range(1 << 32 >> 28):
            bits = torch.arange(c * chunk, (c + 1) * chunk, dtype=torch.int64, device=dev)
            t = (bits - (1 << 31)).to(torch.int32).view(torch.float32)   # every pattern once over all chunks
            del bits
            for N in DIVISORS:
                ops.fedavg_fold(a, [zeros, t], [0, 1], [1, N], init=True)    # product libfedagg.so
                with _abi.use_probe():                                      # IEEE division, probe build
                    ops.tune(fastdiv=0)
                    ops.fedavg_fold(b, [zeros, t], [0, 1], [1, N], init=True)
                ai, bi = a.view(torch.int32), b.view(torch.int32)
                diff = (ai != bi) & ~(torch.isnan(a) & torch.isnan(b))
                nd = int(diff.sum())
                if nd:
                    bad[N] = bad.get(N, 0) + nd
    finally:
        with _abi.use_probe():
            ops.tune(fastdiv=1)
    assert not bad, f"fast division differs from IEEE division: {bad}"
