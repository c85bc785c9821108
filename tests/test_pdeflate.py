"""The single-stream parallel deflate (fedn_amd/csrc/pdeflate.h) reproduces zlib 1.2.11's level-6
stream byte for byte — the stream numpyhelper.save's np.savez_compressed writes per member
(numpyhelper.py:162; zipfile feeds zlib.compressobj(-1, DEFLATED, -15) the .npy header, then the
payload in numpy's 16 MiB writes). zlib itself (CPython's zlib module, the same libz.so.1) is the
checker: every case compares fnpz_deflate_exact's bytes with zlib's for the same input pieces, and
asserts the parallel path produced them (FNPZ_EFALLBACK would mean zlib had to). Inputs cover what
moves a deflate parse: float weights (fp32 / fp16 / fp64, sparse), incompressible bytes (stored
blocks), zero and periodic runs (two parses out of phase across chunks: fix-ups, a parse that
never meets another and becomes the tail's source), long-distance repeats, text, and tails that
end inside matches — cut into many small chunks and odd deflate() pieces, so every chunk boundary,
sync, window slide and the faithful tail replay are exercised."""
import ctypes
import io
import zlib

import numpy as np
import pytest

from fedn_amd import codec

CHUNK = 1 << 18            # pdeflate's smallest chunk: many chunks per test input


def _lib():
    lib = codec.load_lib()
    lib.fnpz_deflate_exact.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                                       ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.POINTER(ctypes.c_int64)]
    lib.fnpz_savez_config.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                                      ctypes.POINTER(ctypes.c_int64)]
    lib.fnpz_savez_config.restype = None
    return lib


def _ends(n, hlen, seg):
    e, b = [hlen], hlen
    while b < n:
        b = min(n, b + seg)
        e.append(b)
    return e


def _zlib(buf, ends):
    c = zlib.compressobj(-1, zlib.DEFLATED, -15)
    out, p = [], 0
    for e in ends:
        out.append(c.compress(buf[p:e]))
        p = e
    out.append(c.flush())
    return b"".join(out)


def _exact(buf, ends, threads=4, chunk=CHUNK):
    lib = _lib()
    a = np.frombuffer(buf, np.uint8)
    cap = len(buf) + len(buf) // 8 + (1 << 16)
    out = np.empty(cap, np.uint8)
    n = ctypes.c_int64()
    e = (ctypes.c_int64 * len(ends))(*ends)
    rc = lib.fnpz_deflate_exact(a.ctypes.data, len(buf), e, len(ends), threads, chunk, out.ctypes.data, cap,
                                ctypes.byref(n))
    return rc, lib.fnpz_last_error().decode(), out[:n.value].tobytes()


def _inputs():
    rng = np.random.default_rng(2024)
    M = 1_000_000
    x = rng.standard_normal(M).astype(np.float32)
    sparse = x.copy()
    sparse[rng.random(M) < 0.9] = 0
    words = [bytes(rng.integers(97, 123, rng.integers(1, 9)).astype(np.uint8)) for _ in range(500)]
    yield "f32", x.tobytes()
    yield "f16", rng.standard_normal(2 * M).astype(np.float16).tobytes()
    yield "f64", rng.standard_normal(M // 2).tobytes()
    yield "sparse_f32", sparse.tobytes()
    yield "random_bytes", rng.integers(0, 256, 3 * M, dtype=np.uint8).tobytes()   # stored blocks
    yield "zeros", bytes(3 * M)                                                    # never in phase
    yield "period7", b"abcdefg" * (M // 2)
    yield "period40000", np.tile(rng.integers(0, 256, 40000, dtype=np.uint8), 80).tobytes()
    yield "text", b" ".join(words[i] for i in rng.integers(0, 500, 600_000))
    yield "ramp_i64", np.arange(M // 2, dtype=np.int64).tobytes()
    yield "regions", b"".join([x[:300_000].tobytes(), bytes(900_000), rng.integers(0, 256, 500_000, dtype=np.uint8)
                               .tobytes(), b"xy" * 300_000, x[300_000:600_000].tobytes()])
    yield "tail_zeros", x[:700_000].tobytes() + bytes(300_000)
    yield "tail_period3", x[:700_000].tobytes() + b"abc" * 70_000
    yield "small_alphabet", rng.integers(0, 3, 3 * M, dtype=np.uint8).tobytes()


CASES = list(_inputs())


@pytest.mark.parametrize("name,buf", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("seg", [16 << 20, 70_001])
def test_parallel_deflate_is_zlibs_stream(name, buf, seg):
    ends = _ends(len(buf), 128, seg)
    rc, info, got = _exact(buf, ends)
    assert rc == 0, info                       # the parallel path made it (no fallback)
    assert got == _zlib(buf, ends), (name, info)


def test_tiny_input_pieces_and_odd_header():
    """deflate() calls of a few KiB (the window is never full; tail replay from stale windows)."""
    rng = np.random.default_rng(5)
    buf = (rng.standard_normal(400_000).astype(np.float32).tobytes() + bytes(5000) +
           rng.integers(0, 4, 300_000, dtype=np.uint8).tobytes())
    for hlen, seg in ((1, 3001), (333, 65536 - 7), (200, 1 << 15)):
        ends = _ends(len(buf), hlen, seg)
        rc, info, got = _exact(buf, ends, threads=3)
        assert rc == 0, info
        assert got == _zlib(buf, ends), (hlen, seg)


def test_small_inputs_fall_back():
    rc, info, _ = _exact(b"x" * 1000, [1000])
    assert rc == codec.FNPZ_EFALLBACK and "too small" in info


@pytest.mark.parametrize("threads", [2, 5])
def test_save_npz_big_member_parallel_is_numpys(threads):
    """codec.save_npz with members over the parallel threshold: np.savez_compressed's archive."""
    lib = _lib()
    rng = np.random.default_rng(9)
    ws = [rng.standard_normal(1_200_000).astype(np.float32), np.arange(10, dtype=np.int64),
          np.where(rng.random(900_000) < 0.5, 0, rng.standard_normal(900_000))]
    before, fb0 = ctypes.c_int64(), ctypes.c_int64()
    lib.fnpz_savez_config(0, 0, ctypes.byref(before), ctypes.byref(fb0))
    lib.fnpz_savez_config(1 << 20, CHUNK, None, None)
    try:
        got = codec.save_npz(ws, threads=threads)
    finally:
        lib.fnpz_savez_config(32 << 20, 4 << 20, None, None)
    after, fb1 = ctypes.c_int64(), ctypes.c_int64()
    lib.fnpz_savez_config(0, 0, ctypes.byref(after), ctypes.byref(fb1))
    assert after.value - before.value == 2 and fb1.value == fb0.value   # both big members went parallel
    ref = io.BytesIO()
    np.savez_compressed(ref, **{str(i): w for i, w in enumerate(ws)})
    assert got == ref.getvalue()


def test_save_npz_member_over_its_thread_share_goes_parallel():
    """Below min_member, a member of >= 4 chunks holding more than 1/threads of the archive is
    deflated on every thread (member-parallel it would outlast the rest); smaller ones stay zlib's."""
    lib = _lib()
    rng = np.random.default_rng(11)
    ws = [rng.standard_normal(n).astype(np.float32) for n in (400_000, 300_000, 60_000, 1000)]
    before, fb0 = ctypes.c_int64(), ctypes.c_int64()
    lib.fnpz_savez_config(0, 0, ctypes.byref(before), ctypes.byref(fb0))
    lib.fnpz_savez_config(1 << 40, CHUNK, None, None)           # min_member out of reach
    try:
        got = codec.save_npz(ws, threads=4)                     # 1.6 MB and 1.2 MB of 3.0 MB: > 1/4 each
    finally:
        lib.fnpz_savez_config(32 << 20, 4 << 20, None, None)
    after, fb1 = ctypes.c_int64(), ctypes.c_int64()
    lib.fnpz_savez_config(0, 0, ctypes.byref(after), ctypes.byref(fb1))
    assert after.value - before.value == 2 and fb1.value == fb0.value
    ref = io.BytesIO()
    np.savez_compressed(ref, **{str(i): w for i, w in enumerate(ws)})
    assert got == ref.getvalue()


def _counts(lib):
    par, fb = ctypes.c_int64(), ctypes.c_int64()
    lib.fnpz_savez_config(0, 0, ctypes.byref(par), ctypes.byref(fb))
    return par.value, fb.value


def test_writer_checks_the_libz_it_stands_in_for():
    """The parallel path is allowed only on a libz it models, which is the one Python's zlib runs and
    which passes the self-test (fednpz.h ABI 7): true here (zlib 1.2.11, numpy's libz)."""
    on, why = codec.savez_zlib_status()
    assert zlib.ZLIB_RUNTIME_VERSION == "1.2.11"
    assert on, why
    assert "self-test passed" in why


def test_unmodelled_libz_sends_every_member_through_libz():
    """on a libz pdeflate.h does not model, a big member is NOT computed by pdeflate.h
    (its bytes would be 1.2.11's next to small members from the host's libz): every member goes through
    the process's libz, and the archive still equals np.savez_compressed on this host. The mismatch is
    forced through the test hook, with the parallel threshold lowered so the member would qualify."""
    lib = _lib()
    rng = np.random.default_rng(21)
    ws = [rng.standard_normal(1_200_000).astype(np.float32), np.arange(1000, dtype=np.int16)]
    ref = io.BytesIO()
    np.savez_compressed(ref, **{str(i): w for i, w in enumerate(ws)})
    codec.savez_force_zlib(True)
    lib.fnpz_savez_config(1 << 20, CHUNK, None, None)
    try:
        on, why = codec.savez_zlib_status()
        assert not on and "forced off" in why
        p0, f0 = _counts(lib)
        got = codec.save_npz(ws, threads=4)
        p1, f1 = _counts(lib)
    finally:
        lib.fnpz_savez_config(32 << 20, 4 << 20, None, None)
        codec.savez_force_zlib(False)
    assert (p1, f1) == (p0, f0)                  # no member went to pdeflate.h
    assert got == ref.getvalue()
    assert codec.savez_zlib_status()[0]           # the check is redone once the hook is cleared
    p2, _ = _counts(lib)
    lib.fnpz_savez_config(1 << 20, CHUNK, None, None)
    try:
        assert codec.save_npz(ws, threads=4) == ref.getvalue()
    finally:
        lib.fnpz_savez_config(32 << 20, 4 << 20, None, None)
    assert _counts(lib)[0] == p2 + 1             # and the same member goes parallel again


def test_python_running_another_libz_turns_the_parallel_path_off():
    """The version Python's zlib reports is the one numpy's archive comes from: a different one (as when
    CPython is linked against zlib-ng or a bundled zlib) turns the parallel path off."""
    lib = codec.load_lib()
    lib.fnpz_savez_zlib_expect(b"1.3.1", -1)
    try:
        on, why = codec.savez_zlib_status()
        assert not on and "1.3.1" in why
    finally:
        lib.fnpz_savez_zlib_expect(zlib.ZLIB_RUNTIME_VERSION.encode(), -1)
    assert codec.savez_zlib_status()[0]


def test_savez_stats_report_the_phases():
    lib = _lib()
    x = np.random.default_rng(3).standard_normal(600_000).astype(np.float32)
    lib.fnpz_savez_config(1 << 20, CHUNK, None, None)
    try:
        codec.save_npz([x], threads=3)
    finally:
        lib.fnpz_savez_config(32 << 20, 4 << 20, None, None)
    st = codec.savez_stats()
    assert list(st) == list(codec.SAVEZ_PHASES)
    assert all(v >= 0 for v in st.values()) and st["parse"] > 0 and st["total"] >= st["parse"]
