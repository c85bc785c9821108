"""Host-side pieces of the staging pipelines that need no GPU: the round-end chunking, the
global-model member table and the multi-device shard geometry (staging.py, layout.py)."""
import numpy as np
import pytest

from fedn_amd.layout import ALIGN, Layout
from fedn_amd.sharded import ALIGN_ELEMS
from fedn_amd.staging import MAX_CHUNKS, MIN_CHUNK_BYTES, chunks, old_groups, old_members


@pytest.mark.parametrize("n,isz", [(0, 4), (1, 4), (1023, 4), (100_000_000, 4), (350_000_000, 8), (2_000_003, 8),
                                   (24_000_077, 4)])
def test_chunks_cover_and_bounds(n, isz):
    cs = chunks(n, isz)
    if n == 0:
        assert cs == []
        return
    assert cs[0][0] == 0 and cs[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(cs, cs[1:]))
    assert len(cs) <= MAX_CHUNKS
    for lo, hi in cs[:-1]:
        assert lo % 1024 == 0 and (hi - lo) * isz >= MIN_CHUNK_BYTES


def test_old_members_matches_concatenation():
    rng = np.random.default_rng(3)
    ups = [rng.standard_normal((4, 5)).astype(np.float32), np.arange(3, dtype=np.int64),
           rng.standard_normal(7).astype(np.float32)]
    old = [rng.standard_normal((4, 5)), np.arange(3, dtype=np.int64) * 2, rng.standard_normal(7)]  # f64 old model
    lay = Layout.of(ups)
    mem = old_members(lay, old)
    cat = old_groups(lay, old)
    for dt in lay.groups:
        odt, parts = mem[dt]
        flat = np.empty(lay.group_elems[dt], odt)
        for a, off in parts:
            flat[off:off + a.size] = a
        assert flat.dtype == cat[dt].dtype
        np.testing.assert_array_equal(flat, cat[dt])


def test_old_members_rejects_like_old_groups():
    lay = Layout.of([np.zeros(3, np.float32), np.zeros(2, np.float32)])
    with pytest.raises(ValueError):
        old_members(lay, [np.zeros(3)])
    with pytest.raises(ValueError):
        old_members(lay, [np.zeros(4), np.zeros(2)])
    with pytest.raises(TypeError):
        old_members(lay, [np.zeros(3), np.zeros(2, np.float32)])


@pytest.mark.parametrize("ndev", [1, 2, 3, 8])
def test_shard_geometry(ndev):
    """Every group is covered by contiguous device slices (4 KiB-aligned starts), and each
    device buffer holds its slices at ALIGN-aligned offsets without overlap."""
    lay = Layout.of([np.zeros((300, 7), np.float32), np.zeros(5, np.int64), np.zeros(1029, np.float32),
                     np.zeros(3_000_017, np.float64)])
    bounds, dev_off, dev_bytes = lay.shard_geometry(ndev)
    for dt in lay.groups:
        b = bounds[dt]
        assert len(b) == ndev and b[0][0] == 0 and b[-1][1] == lay.group_elems[dt]
        assert all(x[1] == y[0] for x, y in zip(b, b[1:]))
        assert all(lo % ALIGN_ELEMS == 0 or lo == hi for lo, hi in b)
    for d in range(ndev):
        spans = sorted((dev_off[d][dt], dev_off[d][dt] + (bounds[dt][d][1] - bounds[dt][d][0]) * dt.itemsize)
                       for dt in lay.groups)
        assert all(a % ALIGN == 0 for a, _ in spans)
        assert all(x[1] <= y[0] for x, y in zip(spans, spans[1:]))
        assert spans[-1][1] <= dev_bytes[d]
