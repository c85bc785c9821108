"""Helper.save writes the reference's bytes: numpyhelper.Helper.save (numpyhelper.py:144-169) is
np.savez_compressed (:162), and tools/gen_golden.py recorded what the REAL reference wrote for
these models (kind "save" fixtures). codec.save_npz / Helper.save must reproduce those archives
byte for byte — zip headers, member order, .npy headers and the deflate stream — for mnist shapes,
mixed dtypes (f16 ... complex64, bool, unicode, big-endian), 0-d and empty arrays, Fortran order,
non-contiguous views, 70 members, and a member past numpy's 16 MiB write size."""
import io
import os
import json

import numpy as np
import pytest

from fedn_amd import codec
from fedn_amd.helper import Helper

import golden_io

SAVE_VIEWS = {
    "T": lambda b: b.T,
    "cols3": lambda b: b[:, ::3],
    "rev": lambda b: b[::-1],
    "perm201": lambda b: b.transpose(2, 0, 1),
    "bcast": lambda b: np.broadcast_to(b, (7,) + b.shape),
}

CASES = golden_io.case_names("save")


def _weights(z):
    views = json.loads(str(z["views"]))
    ws = [z[f"w_t{t}"] for t in range(int(z["w_len"]))]
    return [SAVE_VIEWS[v](w) if v else w for w, v in zip(ws, views)]


@pytest.mark.parametrize("name", CASES)
def test_fixture_big_members_through_the_parallel_deflate(name):
    """the same fixtures with the parallel threshold lowered to pdeflate.h's
    smallest input (two 256 KiB chunks), so every member it can take — the sparse fixture's 2.4 MB and
    20 MB members; the other fixtures' members are all under 512 KiB — is computed by it instead of
    libz, with no fallback: the archive is still the reference's."""
    import ctypes
    z = golden_io.load_case(name)["raw"]
    ws = _weights(z)
    lib = codec.load_lib()
    lib.fnpz_savez_config.restype = None
    lib.fnpz_savez_config.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                      ctypes.POINTER(ctypes.c_int64)]
    par0, par1, fb0, fb1 = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
    lib.fnpz_savez_config(0, 0, ctypes.byref(par0), ctypes.byref(fb0))
    lib.fnpz_savez_config(512 << 10, 256 << 10, None, None)
    try:
        got = codec.save_npz(ws, threads=4)
    finally:
        lib.fnpz_savez_config(32 << 20, 4 << 20, None, None)
    lib.fnpz_savez_config(0, 0, ctypes.byref(par1), ctypes.byref(fb1))
    assert got == z["npz"].tobytes()
    big = sum(1 for w in ws if np.asarray(w).nbytes >= 512 << 10)
    assert (par1.value - par0.value, fb1.value - fb0.value) == (big, 0)


def test_save_fixtures_present():
    assert len(CASES) >= 8


@pytest.mark.parametrize("name", CASES)
def test_helper_save_is_byte_identical_to_the_reference(name, tmp_path):
    z = golden_io.load_case(name)["raw"]
    ws = _weights(z)
    want = z["npz"].tobytes()
    path = Helper().save(ws, str(tmp_path / "m.npz"))
    with open(path, "rb") as f:
        assert f.read() == want
    bio = io.BytesIO()
    Helper().save(ws, bio)                      # a file-like target gets the same bytes
    assert bio.getvalue() == want
    assert codec.save_npz(ws, threads=3) == want
    back = Helper().load(path)                  # and the archive decodes to the weights
    assert len(back) == len(ws)
    for x, y in zip(ws, back):
        assert y.dtype == x.dtype and y.shape == x.shape
        assert np.asarray(x).tobytes() == y.tobytes()
    if "raw_binary" in z:
        p2 = Helper().save(ws, str(tmp_path / "m.bin"), file_type="raw_binary")
        with open(p2, "rb") as f:
            assert f.read() == z["raw_binary"].tobytes()


def test_blocks_writer_is_opt_in(tmp_path, monkeypatch):
    """FEDN_AMD_NPZ_WRITER=blocks selects the block-parallel archive (np.load reads it, its bytes are
    the codec's own); the default is numpy's; anything else is refused."""
    ws = [np.random.default_rng(0).standard_normal(100_000).astype(np.float32)]
    ref = io.BytesIO()
    np.savez_compressed(ref, **{"0": ws[0]})
    monkeypatch.setenv("FEDN_AMD_NPZ_WRITER", "blocks")
    p = Helper().save(ws, str(tmp_path / "b.npz"))
    data = open(p, "rb").read()
    assert data != ref.getvalue()
    assert np.load(io.BytesIO(data))["0"].tobytes() == ws[0].tobytes()
    monkeypatch.setenv("FEDN_AMD_NPZ_WRITER", "numpy")
    assert open(Helper().save(ws, str(tmp_path / "n.npz")), "rb").read() == ref.getvalue()
    monkeypatch.setenv("FEDN_AMD_NPZ_WRITER", "zstd")
    with pytest.raises(ValueError):
        Helper().save(ws, str(tmp_path / "x.npz"))


def _layouts(rng):
    base = rng.standard_normal((60, 50))
    yield "c", [base.astype(np.float32)]
    yield "f", [np.asfortranarray(base)]
    yield "slice", [base[3:50:2, ::-3]]
    yield "t3", [rng.standard_normal((3, 4, 5)).astype(np.float16).transpose(1, 2, 0)]
    yield "0d", [np.float64(2.5), np.array(-1, np.int16)]
    yield "struct", [np.zeros(6, dtype=[("a", "<i4"), ("b", "<f8", (2,))])]
    yield "ints", [np.arange(100_000, dtype=np.int64), np.arange(255, dtype=np.uint8)]
    yield "zeros", [np.zeros(300_000, np.float32)]
    yield "list", [[1.0, 2.0, 3.0], [[1, 2], [3, 4]]]        # numpy's asanyarray of python lists


@pytest.mark.parametrize("threads", [1, 4])
def test_matches_numpy_on_more_layouts(threads):
    """Beyond the fixtures: numpy itself (the library numpyhelper.save calls) on more layouts."""
    for tag, ws in _layouts(np.random.default_rng(7)):
        ref = io.BytesIO()
        np.savez_compressed(ref, **{str(i): w for i, w in enumerate(ws)})
        assert codec.save_npz(ws, threads=threads) == ref.getvalue(), tag


def test_object_arrays_fall_back_to_numpy():
    ws = [np.array([{"a": 1}, None], dtype=object)]
    ref = io.BytesIO()
    np.savez_compressed(ref, **{"0": ws[0]})
    assert codec.save_npz(ws) == ref.getvalue()


def test_file_handling_is_numpys(tmp_path):
    """numpy's own target handling around the bytes (np.savez_compressed, numpy/lib/_npyio_impl.py
    _savez): a path without ".npz" gets it appended (the reference then returns the path it was
    given), a path-like is accepted, a file object is written from its current offset (zipfile's
    header offsets count from the stream's start), and an unseekable stream gets zipfile's
    data-descriptor records — byte-equal to what numpy writes to the same kind of target."""
    import pathlib

    rng = np.random.default_rng(1)
    ws = [rng.standard_normal((30, 7)).astype(np.float32), np.arange(5)]
    ref = io.BytesIO()
    np.savez_compressed(ref, **{str(i): w for i, w in enumerate(ws)})
    want = ref.getvalue()

    p = str(tmp_path / "model")                      # no suffix: numpy writes model.npz
    assert Helper().save(ws, p) == p
    assert not os.path.exists(p) and open(p + ".npz", "rb").read() == want
    pl = tmp_path / "pl.npz"
    assert Helper().save(ws, pl) == pl and pl.read_bytes() == want

    def numpy_into(target):
        np.savez_compressed(target, **{str(i): w for i, w in enumerate(ws)})
        return target

    a, b = io.BytesIO(b"prefix-bytes"), io.BytesIO(b"prefix-bytes")
    a.seek(0, io.SEEK_END)
    b.seek(0, io.SEEK_END)
    Helper().save(ws, a)
    assert a.getvalue() == numpy_into(b).getvalue() and a.getvalue() != b"prefix-bytes" + want

    class Unseekable(io.RawIOBase):                 # a pipe: write only, no tell / seek
        def __init__(self):
            self.chunks = []

        def writable(self):
            return True

        def write(self, d):
            self.chunks.append(bytes(d))
            return len(d)
    u, v = Unseekable(), Unseekable()
    Helper().save(ws, u)
    got = b"".join(u.chunks)
    assert got == b"".join(numpy_into(v).chunks) and got != want
    assert [np.array_equal(x, y) for x, y in zip(np.load(io.BytesIO(got)).values(), ws)] == [True, True]

    class WriteOnly:                                # no read: numpy refuses it (os.fspath), so do we
        def write(self, d):
            return len(d)
    with pytest.raises(TypeError):
        np.savez_compressed(WriteOnly(), a=ws[0])
    with pytest.raises(TypeError):
        Helper().save(ws, WriteOnly())
