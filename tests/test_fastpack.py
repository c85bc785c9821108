"""CPU tests of the native small-update admission (fedn_amd/csrc/fastpack.c via
layout.fast_admission): it must admit exactly what staging._Pipeline.fast_host admits, pack the
same bytes as Layout.pack, and leave anything else to the general path (-1)."""
import numpy as np
import pytest

from fedn_amd import layout as L
from fedn_amd.layout import Layout, fast_admission, wait_pack_jobs

pytest.importorskip("fedn_amd._fastpack")

MNIST = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]


def _model(rng, shapes, dtypes):
    return [rng.standard_normal(s).astype(d) for s, d in zip(shapes, dtypes)]


def _packed(lay, arrays):
    out = np.zeros(lay.nbytes, np.uint8)
    lay.pack(arrays, out)
    return out


@pytest.mark.parametrize("shapes,dtypes", [
    (MNIST, ["f4"] * 6),
    ([(3, 5), (0,), (7,), (2, 0, 4), (1,)], ["f4", "f4", "f8", "f8", "f2"]),
    ([(1000,), (17,), (4, 4)], ["f8", "f4", "f8"]),
    ([(0,), (0, 3)], ["f4", "f4"]),
])
def test_admit_packs_like_layout(shapes, dtypes):
    rng = np.random.default_rng(0)
    first = _model(rng, shapes, dtypes)
    lay = Layout.of(first)
    admit = fast_admission(lay)
    assert admit is not None
    for _ in range(3):
        upd = _model(rng, shapes, dtypes)
        buf = np.full(lay.nbytes, 0xAB, np.uint8)
        t = admit(upd, buf.ctypes.data, (buf.ctypes.data, buf.nbytes))
        assert t >= 0
        if t:
            wait_pack_jobs(t)
        want = _packed(lay, upd)
        # bytes of the layout's padding are not written; every tensor's bytes are
        for i, off, nb in lay.pack_plan:
            assert np.array_equal(buf[off:off + nb], want[off:off + nb]), i
    assert fast_admission(lay) is admit                     # cached per layout


def test_admit_refuses_other_layouts():
    rng = np.random.default_rng(1)
    m = _model(rng, MNIST, ["f4"] * 6)
    lay = Layout.of(m)
    admit = fast_admission(lay)
    buf = np.zeros(lay.nbytes, np.uint8)
    before = buf.copy()

    class Sub(np.ndarray):
        pass

    bad = [
        m[:5],                                               # fewer tensors
        m + [m[0]],                                          # more tensors
        tuple(m),                                            # not a list
        [m[0].astype(np.float64)] + m[1:],                   # dtype
        [m[0].astype(">f4")] + m[1:],                        # byte order
        [m[0].T.copy()] + m[1:],                             # shape
        [m[0].reshape(-1)] + m[1:],                          # ndim
        [np.asfortranarray(m[0])] + m[1:],                   # not C-contiguous
        [m[0][::-1]] + m[1:],                                # negative strides
        [m[0].view(Sub)] + m[1:],                            # a subclass (fast_host refuses it too)
        [m[0].tolist()] + m[1:],                             # not an array
    ]
    for arrays in bad:
        assert admit(arrays, buf.ctypes.data, (buf.ctypes.data, buf.nbytes)) == -1
    assert np.array_equal(buf, before)                       # nothing queued, nothing written


def test_admission_missing_extension(monkeypatch):
    """Without the extension the pipelines keep the Python admission (same bytes, slower)."""
    monkeypatch.setattr(L, "_FAST", False)
    lay = Layout.of([np.ones(4, np.float32), np.ones(2, np.float32)])
    monkeypatch.delattr(lay, "_fast_admit", raising=False)
    assert fast_admission(lay) is None
    monkeypatch.delattr(lay, "_fast_admit")                # the next test sees the extension again


@pytest.mark.parametrize("piece", [64, 1000, 4096, 1 << 20])
def test_pack_range_pieces_equal_pack(piece):
    """Layout.pack_range (the piecewise stage of large host updates): the copies of every piece,
    run through the native gather, write exactly what Layout.pack writes; a non-contiguous source
    makes it refuse (None) so the stage packs whole."""
    from fedn_amd import codec
    rng = np.random.default_rng(piece)
    arrays = [rng.standard_normal((37, 41)).astype(np.float32), rng.standard_normal(1001),
              rng.standard_normal((5, 7)).astype(np.float16), np.zeros(0, np.float32),
              rng.standard_normal(3000).astype(np.float32)]
    lay = Layout.of(arrays)
    want = _packed(lay, arrays)
    got = np.zeros(lay.nbytes, np.uint8)
    ptr = got.ctypes.data
    for lo in range(0, lay.nbytes, piece):
        jobs = lay.pack_range(arrays, ptr, lo, min(lay.nbytes, lo + piece))
        assert jobs is not None
        codec.gather_raw(jobs, 4, (ptr, got.nbytes))
    for i, off, nb in lay.pack_plan:
        assert np.array_equal(got[off:off + nb], want[off:off + nb]), i
    bad = [np.asfortranarray(arrays[0])] + arrays[1:]
    assert lay.pack_range(bad, ptr, 0, lay.nbytes) is None


def test_threaded_cpu_baseline_matches_single_thread():
    """bench.py's threaded numpy line slices the same oracle over parameters: identical bits."""
    import bench
    from oracle import numpy_ref as ref
    rng = np.random.default_rng(3)
    sample = [rng.standard_normal(100_003).astype(np.float32) for _ in range(9)]
    ns = [int(v) for v in rng.integers(1, 5001, 9)]
    want = ref.fedavg_flat(sample, ns)
    out = bench.cpu_threaded(sample, ns, want)
    assert out["same_as_single_threaded"] and out["cores"] >= 1 and out["value"] > 0
    assert 1 <= bench.usable_cores() <= (__import__("os").cpu_count() or 1)


def test_admit_refuses_a_pack_past_its_buffer():
    """The fednpz ABI 4 window: an admission whose destination would run past the pinned buffer it
    packs into (the class of accounting slip that corrupted the heap in round 3: an arena put one
    update too far) raises CodecError and writes nothing — past the end, before the start, or one
    byte short."""
    from fedn_amd import codec
    rng = np.random.default_rng(5)
    m = _model(rng, MNIST, ["f4"] * 6)
    lay = Layout.of(m)
    admit = fast_admission(lay)
    arena = np.full(2 * lay.nbytes + 64, 0x5A, np.uint8)
    base = arena.ctypes.data
    window = (base, 2 * lay.nbytes)                            # an arena of two updates
    t = admit(m, base + lay.nbytes, window)                    # the second slot: fits exactly
    wait_pack_jobs(t)
    end = max(off + nb for _, off, nb in lay.pack_plan)       # the last byte a pack writes (+1)
    for dst, win in ((base + 2 * lay.nbytes, window),          # a third update into a 2-update arena
                     (base + 2 * lay.nbytes - end + 1, window),   # its last byte one past the arena
                     (base, (base + 8, 2 * lay.nbytes)),       # before the buffer
                     (base, (base, end - 1))):                 # one byte short
        before = arena.copy()
        with pytest.raises(codec.CodecError, match="outside"):
            admit(m, dst, win)
        wait_pack_jobs(codec.gather_start_raw([], [], [], 1, (0, 0)))   # nothing was queued
        assert np.array_equal(arena, before)


def test_gather_raw_and_start_refuse_past_the_window():
    from fedn_amd import codec
    src = np.arange(1000, dtype=np.uint8)
    dst = np.zeros(1000, np.uint8)
    p = dst.ctypes.data
    with pytest.raises(codec.CodecError, match="outside"):
        codec.gather_raw([(p + 1, src.ctypes.data, 1000)], 4, (p, 1000))
    with pytest.raises(codec.CodecError, match="outside"):
        codec.gather_start_raw([p - 1], [src.ctypes.data], [10], 4, (p, 1000))
    with pytest.raises(codec.CodecError, match="window"):
        codec.gather_raw([(p, src.ctypes.data, 10)], 4, (0, 1000))
    assert not dst.any()
    codec.gather_raw([(p, src.ctypes.data, 1000)], 4, (p, 1000))       # exactly the buffer: fine
    assert np.array_equal(dst, src)


def test_start_pack_into_refuses_past_the_window():
    """The Python-side pack (start_pack_into, the arena's non-fast path) checks the same window."""
    from fedn_amd import codec
    lay = Layout.of(_model(np.random.default_rng(6), MNIST, ["f4"] * 6))
    end = max(off + nb for _, off, nb in lay.pack_plan)
    buf = np.zeros(end + 3, np.uint8)                      # 4 bytes in, the last tensor's end is 1 byte past
    with pytest.raises((codec.CodecError, ValueError), match="outside|fit"):
        L.start_pack_into(lay, _model(np.random.default_rng(7), MNIST, ["f4"] * 6), buf.ctypes.data + 4,
                          (buf.ctypes.data, buf.nbytes))
    assert not buf.any()


def test_views_rebuild_the_model_from_its_packed_block():
    """_fastpack.views (the one-call round's result, smallround.py): every tensor a C-contiguous,
    writable view of the block at its packed offset, keeping the block alive."""
    import sys

    from fedn_amd import _fastpack
    rng = np.random.default_rng(3)
    arrays = _model(rng, [(3, 5), (0,), (7,), (2, 3, 4), (1,)], ["f4"] * 5)
    lay = Layout.of(arrays)
    offs = {i: off for i, off, _ in lay.pack_plan}
    plan = _fastpack.plan([(tuple(sh), np.dtype(dt), offs.get(i, 0)) for i, (sh, dt) in
                           enumerate(zip(lay.shapes, lay.dtypes))])
    block = _packed(lay, arrays)
    before = sys.getrefcount(block)
    views = _fastpack.views(plan, block)
    assert sys.getrefcount(block) == before + len(arrays)        # each view holds the block
    for v, a in zip(views, arrays):
        assert v.dtype == a.dtype and v.shape == a.shape and v.flags.c_contiguous and v.flags.writeable
        assert np.array_equal(v, a) and (v.size == 0 or v.base is block)
    del views, v                                 # (the loop variable held the last view)
    assert sys.getrefcount(block) == before
    with pytest.raises(ValueError):                              # a block smaller than the plan
        _fastpack.views(plan, block[:8].copy())


def test_native_round_calls_refuse_bad_arguments():
    """fold_host / fedopt_host check K and their addresses before any call (no GPU needed)."""
    from fedn_amd import _fastpack
    fp = _fastpack.fold_plan([(0, 0, 0, 16)])
    with pytest.raises(ValueError):
        _fastpack.fold_host(fp, 1, 0, 0, 4096, 64, 0, 4096, [], [], 0)          # K = 0
    with pytest.raises(ValueError):
        _fastpack.fold_host(fp, 1, 0, 0, 4096, 64, 65, 4096, [0.0] * 65, [1.0] * 65, 0)   # K > 64
    with pytest.raises(ValueError):
        _fastpack.fold_host(fp, 1, 0, 0, 4096, 64, 2, 4096, [0.0], [1.0, 2.0], 0)  # n / N lengths
    with pytest.raises(ValueError):
        _fastpack.fold_plan([(0, 0, -1, 16)])
    state = (0, -1, 4096, 1, 0, 1, 4096, 1)
    with pytest.raises(ValueError):
        _fastpack.fedopt_host(1, 0, 0, 0, 4096, 64, 1, 0, 0, 16, 4096, [1.0], [1.0], 0, state, 0, 1e-3, 0.9, 0.99,
                              1e-4)                                                    # old = NULL
    with pytest.raises(ValueError):
        _fastpack.fedopt_host(1, 0, 0, 4096, 4096, 64, 0, 0, 0, 16, 4096, [], [], 0, state, 0, 1e-3, 0.9, 0.99,
                              1e-4)                                                    # K = 0


def test_poison_knob_is_off_by_default_and_ignores_host_tensors():
    import torch

    from fedn_amd import reuse
    assert not reuse.enabled()
    t = torch.empty(16)
    assert reuse.watch(t) is t and reuse.stats()["watched"] == 0
    reuse.set_enabled(True)
    try:
        assert reuse.watch(t) is t and reuse.stats()["watched"] == 0   # host tensors are not watched
    finally:
        reuse.set_enabled(False)
