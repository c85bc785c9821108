"""FedOpt sessions on float16 models at the ops level (fa_fedopt_step): numpy's half loops while the
pseudo-gradient is half (round 1: half updates over a half model), float64 after; ragged sizes,
misaligned buffers (the scalar path), K beyond one launch, and the pseudo-gradient carried through the
half workspace across non-final launches (waves) — all bit-exact against the oracle (numpy)."""
import numpy as np
import pytest
import torch

from golden_io import assert_lists_identical
from oracle import numpy_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _dev(a, offset):
    t = torch.from_numpy(np.ascontiguousarray(a))
    big = torch.empty(t.numel() + offset, dtype=t.dtype, device=DEV)
    d = big[offset:]
    d.copy_(t.to(DEV))
    return d


@pytest.mark.parametrize("opt", ["adam", "yogi", "adagrad"])
@pytest.mark.parametrize("K", [5, 70])
@pytest.mark.parametrize("offset", [0, 1])
@pytest.mark.parametrize("waves", [False, True])
def test_fedopt_f16_session(opt, K, offset, waves):
    from fedn_amd import ops
    rng = np.random.default_rng(K * 7 + offset + 3 * waves + len(opt))
    P = 100_003
    old = (1.0 + 0.1 * rng.standard_normal(P)).astype(np.float16)
    params = {"serveropt": opt, "learning_rate": 1e-2, "beta1": 0.9, "beta2": 0.99, "tau": 1e-3}
    st = ref.FedOptState()
    m_dev = v_dev = None
    for r in range(2):
        ups = [(old.astype(np.float64) + 0.01 * rng.standard_normal(P)).astype(np.float16) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 500, K)]
        Ns = [int(v) for v in np.cumsum(ns)]
        want, _ = ref.fedopt_combine(st, [([u], n) for u, n in zip(ups, ns)], [old], params)
        old_d = _dev(old, offset)
        pg_dt, m_dt = ops.fedopt_dtypes(torch.float16, old_d.dtype, None if m_dev is None else m_dev.dtype)
        pg = torch.empty(P, dtype=pg_dt, device=DEV)
        m_out = torch.empty(P, dtype=m_dt, device=DEV)
        v_out = torch.empty(P, dtype=torch.float64, device=DEV)
        out = torch.empty(P, dtype=torch.float64, device=DEV)
        ups_d = [_dev(u, offset) for u in ups]
        kw = dict(m_in=m_dev, m_out=m_out, v_in=v_dev, v_out=v_out, out=out, **params)
        if not waves:
            ops.fedopt_step(old_d, ups_d, ns, Ns, first=True, final=True, pg=pg, **kw)
        else:                                   # waves of 8 into the pg workspace, then a K = 0 server step
            for w in range(0, K, 8):
                ops.fedopt_step(old_d, ups_d[w:w + 8], ns[w:w + 8], Ns[w:w + 8], first=w == 0, final=False, pg=pg)
            ops.fedopt_step(old_d, [], [], [], first=False, final=True, pg=pg, upd_dtype=torch.float16, **kw)
        torch.cuda.synchronize()
        assert pg_dt == (torch.float16 if r == 0 else torch.float64)
        assert_lists_identical([out.cpu().numpy()], want, f"r{r} out")
        assert_lists_identical([m_out.cpu().numpy()], st.m, f"r{r} m")
        assert_lists_identical([v_out.cpu().numpy()], st.v, f"r{r} v")
        m_dev, v_dev, old = m_out, v_out, want[0]
