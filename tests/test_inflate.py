"""The codec's own raw-DEFLATE decoder and CRC-32 (fedn_amd/csrc/inflate.h, fnpz_inflate_raw /
fnpz_crc32) against zlib — the library numpy's np.savez_compressed / np.load go through
(numpyhelper.py:144-189). Every block type (stored, fixed, dynamic), every zlib level and strategy,
outputs resumed at arbitrary window sizes (the decoder stops at any output byte, inside a match
included), sync-flushed ranges (fnpz_write's independently inflatable blocks), and corrupted or
truncated streams: the decoder returns zlib's bytes for what zlib decodes, and rejects what zlib
rejects before the requested length. CPU only."""
import ctypes
import zlib

import numpy as np
import pytest

from fedn_amd import codec


def _inputs():
    rng = np.random.default_rng(5)
    out = {}
    for n in (0, 1, 7, 300, 4096, 70_000, 300_000):
        out[f"random{n}"] = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        out[f"float{n}"] = rng.standard_normal(n // 4).astype(np.float32).tobytes()
        out[f"text{n}"] = (b"abcabcabd hello world " * (n // 22 + 1))[:n]
        sparse = np.zeros(n, np.uint8)
        m = rng.random(n) < 0.05
        sparse[m] = rng.integers(1, 256, int(m.sum()), dtype=np.uint8)
        out[f"sparse{n}"] = sparse.tobytes()
        runs = np.repeat(rng.integers(0, 4, n // 1000 + 1, dtype=np.uint8), 1000)[:n]
        out[f"runs{n}"] = runs.tobytes()
    return out


INPUTS = _inputs()
STRATEGIES = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]


def _deflate(data, level, strategy, flush=zlib.Z_FINISH):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
    return c.compress(data) + c.flush(flush)


@pytest.mark.parametrize("level", [0, 1, 6, 9])
@pytest.mark.parametrize("strategy", STRATEGIES)
def test_every_level_and_strategy_against_zlib(level, strategy):
    for name, data in INPUTS.items():
        z = _deflate(data, level, strategy)
        out, end = codec.inflate_raw(z, len(data))
        assert out == data and end, (name, level, strategy)


@pytest.mark.parametrize("window", [1, 3, 258, 259, 4093, 65536])
def test_resumes_at_any_output_position(window):
    for name in ("float70000", "text70000", "sparse70000", "runs70000", "random4096"):
        data = INPUTS[name]
        for level, strategy in ((1, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_RLE), (9, zlib.Z_FIXED), (0, 0)):
            out, end = codec.inflate_raw(_deflate(data, level, strategy), len(data), window=window)
            assert out == data and end, (name, window, level, strategy)


def test_sync_flushed_range_decodes_without_a_final_block():
    """fnpz_write's blocks: each a deflate range ending in a sync flush (an empty stored block),
    read on its own: the output fills, no final block follows, and that is not an error."""
    for name in ("float300000", "text4096", "random70000"):
        data = INPUTS[name]
        z = _deflate(data, 6, zlib.Z_DEFAULT_STRATEGY, zlib.Z_SYNC_FLUSH)
        assert z.endswith(b"\x00\x00\xff\xff")
        out, end = codec.inflate_raw(z, len(data))
        assert out == data and not end


def test_short_and_long_outputs_are_errors():
    data = INPUTS["float4096"]
    z = _deflate(data, 6, zlib.Z_DEFAULT_STRATEGY)
    with pytest.raises(codec.CodecError, match="ended after"):
        codec.inflate_raw(z, len(data) + 1)          # the stream holds fewer bytes
    out, end = codec.inflate_raw(z, len(data) - 1)   # a prefix: fine, the final block not reached
    assert out == data[:-1] and not end


def test_crc32_matches_zlib():
    rng = np.random.default_rng(9)
    for n in (0, 1, 15, 16, 63, 64, 65, 127, 1000, 65536 + 13, 1_000_003):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for off in (0, 1, 7):
            chunk = data[off:]
            assert codec.crc32(chunk) == zlib.crc32(chunk)
            assert codec.crc32(chunk, 0x12345678) == zlib.crc32(chunk, 0x12345678)
    a, b = INPUTS["float300000"], INPUTS["text70000"]
    assert codec.crc32(b, codec.crc32(a)) == zlib.crc32(a + b)


def _zlib_prefix(z, n):
    """zlib's first n output bytes (None if it fails or runs short before them) and whether the
    stream also ends cleanly right there."""
    d = zlib.decompressobj(-15)
    try:
        out = d.decompress(z, n)
    except zlib.error:
        return None, False
    if len(out) != n:
        return None, False
    try:
        rest = d.decompress(d.unconsumed_tail, 1) if d.unconsumed_tail else b""
        rest += d.flush()
    except zlib.error:
        return out, False
    return out, d.eof and not rest


def test_corrupted_streams_rejected_like_zlib():
    """Bit flips, random bytes and truncations. A stream zlib decodes completely to the expected
    length (final block included) decodes identically; one where zlib fails or runs short before
    that length is rejected; otherwise (zlib reaches the length, the stream is bad after it) the
    decoder may stop at the full output or reject — but never returns other bytes."""
    rng = np.random.default_rng(17)
    names = [k for k, v in INPUTS.items() if 0 < len(v) <= 70_000]
    agree = rejected = 0
    for it in range(3000):
        data = INPUTS[names[rng.integers(len(names))]]
        z = bytearray(_deflate(data, int(rng.integers(0, 10)), STRATEGIES[rng.integers(len(STRATEGIES))]))
        mode = it % 3
        if mode == 0:
            for _ in range(int(rng.integers(1, 5))):
                z[rng.integers(len(z))] ^= 1 << int(rng.integers(8))
        elif mode == 1:
            del z[int(rng.integers(len(z))):]
        else:
            for _ in range(8):
                z[rng.integers(len(z))] = int(rng.integers(256))
        prefix, complete = _zlib_prefix(bytes(z), len(data))
        try:
            out, end = codec.inflate_raw(bytes(z), len(data))
        except codec.CodecError:
            out, end = None, False
        if complete:
            assert out == prefix and end, it
            agree += 1
        elif out is None:
            rejected += 1
        elif prefix is not None:
            assert out == prefix, it
        else:
            # zlib raised; the decoder stopped at the full output first (zlib decodes a length /
            # distance pair before it checks for room, this decoder checks first): the bytes zlib did
            # produce before its error must be the decoder's, and no clean end may be claimed
            assert not end, it
            part = _zlib_partial(bytes(z))
            assert out[:len(part)] == part[:len(out)], it
    assert agree > 100 and rejected > 1000


def _zlib_partial(z, piece=16):
    d = zlib.decompressobj(-15)
    out = b""
    for i in range(0, len(z), piece):
        try:
            out += d.decompress(z[i:i + piece])
        except zlib.error:
            break
    return out


def _npy(x):
    import io
    bio = io.BytesIO()
    np.lib.format.write_array(bio, x, allow_pickle=False)
    return bio.getvalue()


def _npz_one(x, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
    """A one-member npz like np.savez_compressed's (its container; any deflate level / strategy)."""
    npy = _npy(x)
    return _npz_member(npy, _deflate(npy, level, strategy))   # zipfile has no strategy knob


def _npz_member(npy, comp):
    """The zip records around one deflated .npy member, by hand."""
    import struct
    name = b"0.npy"
    crc = zlib.crc32(npy)
    local = struct.pack("<IHHHHHIIIHH", 0x04034B50, 20, 0, 8, 0, 0x21, crc, len(comp), len(npy), len(name), 0) + name
    central = struct.pack("<IHHHHHHIIIHHHHHII", 0x02014B50, 20, 20, 0, 8, 0, 0x21, crc, len(comp), len(npy),
                          len(name), 0, 0, 0, 0, 0, 0) + name
    eocd = struct.pack("<IHHHHIIH", 0x06054B50, 0, 0, 1, 1, len(central), len(local) + len(comp), 0)
    return local + comp + central + eocd


@pytest.fixture
def _small_parallel():
    codec.parallel_config(64 << 10, 16 << 10)
    yield
    codec.parallel_config(16 << 20, 4 << 20)


def test_parallel_decode_of_one_stream_matches_numpy(_small_parallel):
    """One large deflate stream split over threads: chunk starts found as block headers,
    back-references across chunk boundaries (a noisy 30,011-byte period: matches reach ~30 KB back)
    carried as markers, sparse runs, fp32 weights, text; levels 1 / 6 / 9 and the zlib strategies.
    Every decode equals np.load; streams without findable dynamic blocks (stored, fixed codes) fall
    back to the sequential decode, with the same result."""
    rng = np.random.default_rng(21)
    period = np.tile(rng.integers(0, 255, 30_011, dtype=np.uint8), 80)
    hit = rng.random(period.size) < 0.15                 # 15 % noise: still matched ~30 KB back
    period[hit] = rng.integers(0, 255, int(hit.sum()), dtype=np.uint8)
    xs = {"weights": rng.standard_normal(600_000).astype(np.float32),
          "period": period,
          "sparse": np.where(rng.random(2_000_000) < 0.97, 0, rng.integers(1, 255, 2_000_000)).astype(np.uint8),
          "text": np.frombuffer((b"federated averaging of model updates " * 60_000), dtype=np.uint8).copy()}
    before = codec.parallel_config()
    for name, x in xs.items():
        for level, strategy in ((1, zlib.Z_DEFAULT_STRATEGY), (6, zlib.Z_DEFAULT_STRATEGY), (9, zlib.Z_FILTERED),
                                (6, zlib.Z_RLE), (6, zlib.Z_HUFFMAN_ONLY), (6, zlib.Z_FIXED), (0, 0)):
            raw = _npz_one(x, level, strategy)
            got = codec.load_npz(raw, threads=8)[0]
            assert got.dtype == x.dtype and np.array_equal(got, x), (name, level, strategy)
    after = codec.parallel_config()
    assert after[0] - before[0] >= 10                   # most of them went parallel


def test_parallel_decode_rejects_corruption(_small_parallel):
    """A corrupted large stream fails loudly (CRC-32 or an invalid code), parallel or not."""
    rng = np.random.default_rng(22)
    x = rng.standard_normal(600_000).astype(np.float32)
    raw = bytearray(_npz_one(x))
    for k in range(20):
        bad = bytearray(raw)
        pos = 60 + int(rng.integers(len(raw) // 3, len(raw) - 200))
        bad[pos] ^= 1 << int(rng.integers(8))
        with pytest.raises(codec.CodecError):
            codec.load_npz(bytes(bad), threads=8)


def _spliced(npy, rng):
    """One deflate stream over `npy` made of runs of segments: each run from its own compressor
    (random level and strategy, stored included), segments within a run separated by sync / full
    flushes (so back-references cross some segment boundaries and not others), every run but the
    last ending on a sync flush — byte-aligned, non-final, so the runs concatenate into one valid
    stream of mixed block types."""
    cuts = np.sort(rng.choice(np.arange(1, len(npy)), size=int(rng.integers(3, 12)), replace=False))
    segs = np.split(np.frombuffer(npy, np.uint8), cuts)
    out, c = [], None
    for i, seg in enumerate(segs):
        if c is None or rng.random() < 0.4:
            level = int(rng.choice([0, 1, 6, 9]))
            c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, int(rng.choice(STRATEGIES)))
        last = i == len(segs) - 1
        flush = zlib.Z_FINISH if last else (zlib.Z_FULL_FLUSH if rng.random() < 0.3 else zlib.Z_SYNC_FLUSH)
        out.append(c.compress(seg.tobytes()) + c.flush(flush))
        if not last and rng.random() < 0.4:
            c = None                           # the next segment from a fresh compressor
    return b"".join(out)


def test_parallel_decode_of_spliced_streams(_small_parallel):
    """Streams whose blocks change type and table mid-stream (stored / fixed / dynamic runs,
    empty sync-flush blocks, back-references across some flush points): the parallel decode, with
    chunk starts found wherever a dynamic block happens to begin, equals np.load's bytes; streams
    that open with a stored or fixed block decode in order."""
    before = codec.parallel_config()
    for seed in range(16):
        rng = np.random.default_rng(700 + seed)
        parts = [rng.standard_normal(int(rng.integers(20_000, 120_000))).astype(np.float32).view(np.uint8),
                 np.where(rng.random(int(rng.integers(50_000, 300_000))) < 0.95, 0, 7).astype(np.uint8),
                 np.tile(rng.integers(0, 255, int(rng.integers(500, 40_000)), dtype=np.uint8), 6),
                 np.frombuffer(b"model update " * int(rng.integers(2_000, 20_000)), np.uint8)]
        rng.shuffle(parts)
        x = np.concatenate(parts)
        npy = _npy(x)
        comp = _spliced(npy, rng)
        assert zlib.decompress(comp, -15) == npy
        got = codec.load_npz(_npz_member(npy, comp), threads=int(rng.integers(2, 9)))[0]
        assert got.dtype == x.dtype and np.array_equal(got, x), seed
    after = codec.parallel_config()
    assert after[0] - before[0] >= 6                    # (10 of the 16 on these seeds)


def test_concurrent_parallel_decodes_share_the_pool(_small_parallel):
    """Several large streams decoded at once from Python threads (the staging workers on a burst
    of ModelUpdates): their chunks share one decode pool; every result equals np.load's, and more
    decodes at once than threads take the in-order decode for the surplus."""
    from concurrent.futures import ThreadPoolExecutor
    rng = np.random.default_rng(23)
    xs = [rng.standard_normal(int(rng.integers(150_000, 400_000))).astype(np.float32) for _ in range(12)]
    raws = [_npz_one(x, level=int(rng.choice([1, 6]))) for x in xs]
    before = codec.parallel_config()
    with ThreadPoolExecutor(12) as ex:
        for _ in range(3):
            got = list(ex.map(lambda r: codec.load_npz(r, threads=4)[0], raws))
            for g, x in zip(got, xs):
                assert g.dtype == x.dtype and np.array_equal(g, x)
    after = codec.parallel_config()
    assert after[0] - before[0] >= 6


def _header_bits(lengths, lead):
    """A dynamic block header (BFINAL 0, BTYPE 2, HLIT 0, HDIST 0, HCLEN = len(lengths) - 4, then the
    precode lengths, 3 bits each) behind ``lead`` zero bits, LSB-first as DEFLATE packs them."""
    bits = [0] * lead + [0] + [0, 1] + [0] * 5 + [0] * 5
    hclen = len(lengths) - 4
    bits += [(hclen >> i) & 1 for i in range(4)]
    for v in lengths:
        bits += [(v >> i) & 1 for i in range(3)]
    bits += [0] * (8 * 16)
    out = bytearray((len(bits) + 7) // 8)
    for i, b in enumerate(bits):
        out[i // 8] |= b << (i % 8)
    return bytes(out)


@pytest.mark.parametrize("lead", range(8))
def test_header_finder_reads_all_57_precode_bits(lead):
    """with the header at bit offset 7 and HCLEN = 19, the 19th precode length's top bit
    is the 57th bit after the first load's shift. A complete precode whose 19th length is 4 (0b100):
    read right it is complete (accepted); that bit read as 0 would leave it incomplete (rejected)."""
    lib = codec.load_lib()
    lib.fnpz_probe_dynamic_header.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_int64]
    complete = [1, 2, 3, 4] + [0] * 14 + [4]          # 1/2 + 1/4 + 1/8 + 1/16 + 1/16
    incomplete = [1, 2, 3, 4] + [0] * 15
    good, bad = _header_bits(complete, lead), _header_bits(incomplete, lead)
    assert lib.fnpz_probe_dynamic_header(good, len(good), lead) == 1
    assert lib.fnpz_probe_dynamic_header(bad, len(bad), lead) == 0
