"""FEDN_AMD_POISON_REUSE (fedn_amd/reuse.py) catches the cross-stream reuse class it is for (VERDICT r5
item 3): a staged buffer written on a staging stream, read by a launch queued on a busy compute stream,
and dropped before that launch ran. With the knob on, the freed block is handed back on the staging
stream and filled with NaN before the read — the fold reads poison. The same buffer protected as the
pipelines protect theirs (held until the reader ran, or record_stream) folds the true bytes. The
pipelines' own multi-device, streaming and wave tests are then run with the knob on
(profiles/r06_poison_reuse.log)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(autouse=True)
def _knob():
    from fedn_amd import _abi, reuse
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    _abi.load()
    was = reuse.enabled()
    reuse.set_enabled(True)
    reuse.drain()                      # earlier tests' frees (a knob-on suite run) handled first
    if reuse.HOLD:
        # the holding mode leaves many same-size free blocks in the pool after a suite run: returned
        # first, so that none of them is offered before the dropped one (measured: needed there only)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    yield reuse
    reuse.drain()
    reuse.set_enabled(was)


def _busy(stream, ms_ish=40):
    """Queue ~tens of ms of folds on ``stream`` so a launch behind them waits."""
    from fedn_amd import ops
    P = 50_000_000
    ups = [torch.ones(P, device=DEV) for _ in range(8)]
    agg = torch.empty(P, device=DEV)
    for _ in range(ms_ish):
        ops.fedavg_fold(agg, ups, [1] * 8, list(range(1, 9)), init=True, stream=stream)
    return ups, agg


@pytest.mark.parametrize("protect", ["none", "hold", "record_stream"])
def test_knob_poisons_an_unprotected_drop_and_spares_a_protected_one(_knob, protect):
    from fedn_amd import ops
    reuse = _knob
    staging, compute = torch.cuda.Stream(DEV), torch.cuda.Stream(DEV)
    P = 1 << 20
    src = torch.full((P,), 3.0, device=DEV)
    out = torch.empty(P, device=DEV)
    keep = _busy(compute)                                  # the compute stream is busy for a while
    with torch.cuda.stream(staging):
        staged = reuse.watch(torch.empty(P, device=DEV), staging)
        staged.copy_(src)                                  # the "H2D" on the staging stream
    ready = torch.cuda.Event()
    ready.record(staging)
    compute.wait_event(ready)
    ops.fedavg_fold(out, [staged, staged], [0, 1], [1, 1], init=True, stream=compute)   # reads it later
    held = None
    if protect == "hold":
        held = staged
    elif protect == "record_stream":
        staged.record_stream(compute)
    del staged                                             # the last reference the caller had
    reuse.drain()
    compute.synchronize()
    got = out.cpu().numpy()
    if protect == "none":
        assert np.isnan(got).any(), "the knob did not catch an unprotected drop"
        assert reuse.stats()["poisoned"] >= 1
    else:
        assert (got == 3.0).all()
    del held, keep
    torch.cuda.synchronize()
