"""The exact writer's ZIP64 branches against numpy itself (numpyhelper.py:162, np.savez_compressed).

zipfile switches to ZIP64 sizes (version 45, 0xFFFFFFFF in the 32-bit fields), header offsets and end
records only past ZIP64_LIMIT (2 GiB - 1) and ZIP_FILECOUNT_LIMIT (65,535 members): a 1 B-parameter
fp32 model (configs[4]) crosses the first. Writing gigabytes twice per case is no unit test, so both
sides lower the limits to the same small values — CPython's zipfile by patching its module globals
(read at call time by FileHeader / _write_end_record), fnpz_savez through fnpz_savez_zip_limits —
and the archives must still be byte-equal: the same decisions at the same thresholds."""
import ctypes
import io
import zipfile

import numpy as np
import pytest

from fedn_amd import codec


@pytest.fixture
def limits(monkeypatch):
    lib = codec.load_lib()
    lib.fnpz_savez_zip_limits.argtypes = [ctypes.c_int64, ctypes.c_int64]
    lib.fnpz_savez_zip_limits.restype = None

    def set_limits(zip64, count):
        monkeypatch.setattr(zipfile, "ZIP64_LIMIT", zip64)
        monkeypatch.setattr(zipfile, "ZIP_FILECOUNT_LIMIT", count)
        lib.fnpz_savez_zip_limits(zip64, count)
    yield set_limits
    lib.fnpz_savez_zip_limits(0, 0)


def _numpy(ws):
    b = io.BytesIO()
    np.savez_compressed(b, **{str(i): w for i, w in enumerate(ws)})
    return b.getvalue()


def _models():
    rng = np.random.default_rng(64)
    return {
        "weights": [rng.standard_normal(s).astype(np.float32) for s in ((40, 30), (30,), (300, 12), (7,))],
        "incompressible": [rng.integers(0, 256, 5000, dtype=np.uint8), rng.integers(0, 256, 3, dtype=np.uint8)],
        "many": [np.full(3, i, np.int64) for i in range(9)],
        "empty_and_scalar": [np.zeros(0, np.float32), np.float64(2.5) * np.ones(()), np.arange(600, dtype=np.int16)],
    }


@pytest.mark.parametrize("name", list(_models()))
@pytest.mark.parametrize("zip64,count", [(1000, 65535), (4000, 65535), (1 << 20, 3), (300, 2)])
def test_zip64_branches_are_numpys(limits, name, zip64, count):
    ws = _models()[name]
    limits(zip64, count)
    want = _numpy(ws)
    assert codec.save_npz(ws, threads=3) == want
    # the lowered limits did take numpy down the ZIP64 paths being compared
    if zip64 < 4000 or count < len(ws):
        assert b"PK\x06\x06" in want or any(i.extract_version == 45 for i in zipfile.ZipFile(io.BytesIO(want)).infolist())


def test_only_the_compressed_size_past_the_limit(limits):
    """Incompressible bytes deflate to more than they are (a stored block's 5 bytes per 16,383
    literals outweigh what the .npy header saves): a limit between the two makes zipfile's
    `file_size > LIMIT or compress_size > LIMIT` true on the second test alone."""
    w = np.random.default_rng(3).integers(0, 256, 2_000_000, dtype=np.uint8)
    with zipfile.ZipFile(io.BytesIO(_numpy([w]))) as z:
        info = z.infolist()[0]
    assert info.compress_size > info.file_size
    limits(info.file_size, 65535)
    want = _numpy([w])
    assert zipfile.ZipFile(io.BytesIO(want)).infolist()[0].extract_version == 45
    assert codec.save_npz([w], threads=2) == want


def test_defaults_restored(limits):
    limits(500, 2)
    codec.load_lib().fnpz_savez_zip_limits(0, 0)
    ws = _models()["many"]
    ref = io.BytesIO()
    zipfile.ZIP64_LIMIT, zipfile.ZIP_FILECOUNT_LIMIT = (1 << 31) - 1, (1 << 16) - 1
    np.savez_compressed(ref, **{str(i): w for i, w in enumerate(ws)})
    assert codec.save_npz(ws) == ref.getvalue()
