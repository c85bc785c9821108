"""Decode-while-uploading (fedn_amd/upload.py, SURVEY.md §8(f) rank 1, ModelService.Upload
modelservice.py:198-221): the incremental npz decoder against np.load on the same bytes, fed
in the chunkings a gRPC stream can deliver, and the Upload tee against the stand-in
ModelService. CPU-only (host code; pinned=False)."""
import io
import threading
import zipfile

import numpy as np
import pytest

from fedn_amd import codec
from fedn_amd.updatehandler import MemoryModelService, MemoryModelStore, upload_requests
from fedn_amd.upload import DecodedUpdate, DecodeError, NpzStreamDecoder, StreamingUpload

ARRAYS = [np.arange(12, dtype=np.float32).reshape(3, 4), np.float64(2.5) * np.ones(()), np.zeros((0, 7), np.float32),
          np.arange(-5, 5, dtype=np.int64), np.linspace(0, 1, 33, dtype=np.float16), np.array([True, False, True]),
          np.random.default_rng(0).standard_normal((257, 129)).astype(np.float32), np.arange(10, dtype=np.uint8)]


def _savez(arrays, compressed=True):
    b = io.BytesIO()
    (np.savez_compressed if compressed else np.savez)(b, **{str(i): a for i, a in enumerate(arrays)})
    return b.getvalue()


def _decode(data, chunk):
    dec = NpzStreamDecoder()
    for o in range(0, len(data), chunk):
        dec.feed(data[o:o + chunk])
    return DecodedUpdate(dec.finish(), None).arrays


def _same_as_npload(data, got):
    z = np.load(io.BytesIO(data), allow_pickle=False)
    want = [z[str(i)] for i in range(len(z.files))]      # numpyhelper.load (numpyhelper.py:180-182)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        assert g.dtype == w.dtype and g.shape == w.shape and g.tobytes() == w.tobytes()


@pytest.mark.parametrize("compressed", [True, False])
@pytest.mark.parametrize("chunk", [1, 7, 4096, 1 << 20])
def test_decoder_matches_npload(compressed, chunk):
    data = _savez(ARRAYS, compressed)
    _same_as_npload(data, _decode(data, chunk))


def test_decoder_random_chunking():
    rng = np.random.default_rng(5)
    data = _savez([rng.standard_normal(70_000).astype(np.float32), rng.integers(0, 9, (40, 40))])
    dec = NpzStreamDecoder()
    o = 0
    while o < len(data):
        n = int(rng.integers(1, 50_000))
        dec.feed(data[o:o + n])
        o += n
    _same_as_npload(data, DecodedUpdate(dec.finish(), None).arrays)


def test_decoder_reads_native_codec_archives():
    """fedn_amd.codec.save_npz_blocks writes block-parallel deflate + a private extra field."""
    rng = np.random.default_rng(1)
    arrays = [rng.standard_normal(3_000_000).astype(np.float32), np.arange(5, dtype=np.int64)]
    data = bytes(codec.save_npz_blocks(arrays, block=1 << 20))
    _same_as_npload(data, _decode(data, 1 << 20))


class _NoSeek(io.RawIOBase):
    def __init__(self):
        self.b = bytearray()

    def writable(self):
        return True

    def write(self, x):
        self.b += x
        return len(x)


def _zip_members(members, stream=False, zip64=False, method=zipfile.ZIP_DEFLATED):
    """An npz written through zipfile: to an unseekable stream (data descriptors after every
    member) and/or with ZIP64 local headers."""
    out = _NoSeek() if stream else io.BytesIO()
    with zipfile.ZipFile(out, "w", compression=method) as zf:
        for name, arr in members:
            with zf.open(name + ".npy", "w", force_zip64=zip64) as f:
                np.lib.format.write_array(f, arr, allow_pickle=False)
    return bytes(out.b) if stream else out.getvalue()


@pytest.mark.parametrize("stream,zip64", [(True, False), (False, True), (True, True)])
def test_decoder_descriptors_and_zip64(stream, zip64):
    data = _zip_members([(str(i), a) for i, a in enumerate(ARRAYS)], stream, zip64)
    _same_as_npload(data, _decode(data, 333))


def test_decoder_key_order_is_numpyhelper_order():
    """Members named "1", "0" in archive order come back as [a["0"], a["1"]]."""
    a0, a1 = np.arange(3, dtype=np.float32), np.arange(4, dtype=np.int64)
    data = _zip_members([("1", a1), ("0", a0)])
    got = _decode(data, 100)
    assert got[0].tobytes() == a0.tobytes() and got[1].tobytes() == a1.tobytes()


def test_decoder_rejects_non_numpyhelper_keys():
    data = _savez([np.zeros(3)]).replace(b"0.npy", b"w.npy")
    with pytest.raises(DecodeError):
        _decode(data, 1000)


def test_decoder_rejects_corruption():
    data = bytearray(_savez([np.arange(1000, dtype=np.float32)], compressed=False))
    i = data.find(b"\x93NUMPY") + 200
    data[i] ^= 0xFF                                        # payload byte: CRC-32 must catch it
    with pytest.raises(DecodeError, match="CRC"):
        _decode(bytes(data), 64)


def test_decoder_rejects_truncation():
    data = _savez([np.arange(1000, dtype=np.float32)])
    with pytest.raises(DecodeError):
        _decode(data[:len(data) // 2], 64)


def test_decoder_rejects_object_and_fortran():
    b = io.BytesIO()
    np.savez(b, **{"0": np.array([1, "x"], dtype=object)})
    with pytest.raises(DecodeError):
        _decode(b.getvalue(), 100)
    data = _savez([np.asfortranarray(np.arange(6, dtype=np.float32).reshape(2, 3))])
    with pytest.raises(DecodeError):
        _decode(data, 100)


class _Handler:
    def __init__(self, wants=True):
        self.wants = wants
        self.adopted = {}

    def wants_upload(self):
        return self.wants

    def adopt(self, rid, fut):
        self.adopted[rid] = fut


def test_streaming_upload_tee():
    """Every request still reaches ModelService.Upload (the stored bytes are the upload); the
    decode is handed to the handler on the OK request and equals np.load of those bytes."""
    store = MemoryModelStore()
    h = _Handler()
    svc = StreamingUpload(MemoryModelService(store), h, workers=2, pinned=False)
    datas = {f"u{i}": _savez([np.random.default_rng(i).standard_normal(300_000).astype(np.float32), ARRAYS[3]])
             for i in range(3)}
    for rid, data in datas.items():
        resp = svc.Upload(upload_requests(data, rid, chunk=65536), None)
        assert resp.status == 0 and resp.id == rid
    for rid, data in datas.items():
        assert store.get(rid).data == data
        _same_as_npload(data, h.adopted[rid].result(timeout=30).arrays)
    svc.close()


def test_streaming_upload_opt_out_and_bad_bytes():
    store = MemoryModelStore()
    h = _Handler(wants=False)
    svc = StreamingUpload(MemoryModelService(store), h, workers=1, pinned=False)
    svc.Upload(upload_requests(_savez([np.zeros(5)]), "a"), None)
    assert h.adopted == {} and store.get("a") is not None
    h.wants = True
    svc.Upload(upload_requests(b"\x00" * 5000, "raw", chunk=1000), None)     # binaryhelper-like bytes
    with pytest.raises(DecodeError):
        h.adopted["raw"].result(timeout=30)
    assert store.get("raw").data == b"\x00" * 5000
    svc.close()


def test_streaming_upload_abandoned_stream_does_not_hang():
    """A stream that ends without its OK request releases the decoder thread."""
    h = _Handler()
    svc = StreamingUpload(MemoryModelService(MemoryModelStore()), h, workers=1, pinned=False)
    data = _savez([np.arange(10_000, dtype=np.float32)])
    reqs = list(upload_requests(data, "x", chunk=1000))[:-1]            # no OK
    assert svc.Upload(iter(reqs), None) is None
    assert "x" not in h.adopted
    t = threading.Thread(target=svc.close)
    t.start()
    t.join(30)
    assert not t.is_alive()


def test_streaming_upload_mixin():
    """StreamingUploadMixin on a ModelService class: the subclass is still the service (the
    gRPC server's isinstance check), uploads are teed once a handler is attached."""
    from fedn_amd.upload import StreamingUploadMixin

    class Service(StreamingUploadMixin, MemoryModelService):
        pass

    store = MemoryModelStore()
    svc = Service(store)
    assert isinstance(svc, MemoryModelService)
    data = _savez([np.arange(50_000, dtype=np.float32)])
    svc.Upload(upload_requests(data, "plain", chunk=4096), None)
    h = _Handler()
    svc.attach(h, workers=1, pinned=False)
    svc.Upload(upload_requests(data, "teed", chunk=4096), None)
    assert store.get("plain").data == data and store.get("teed").data == data
    assert list(h.adopted) == ["teed"]
    svc.Upload(upload_requests(data, "own-global", chunk=4096), svc)   # ModelService.set_model (context=self)
    assert store.get("own-global").data == data and "own-global" not in h.adopted
    _same_as_npload(data, h.adopted["teed"].result(timeout=30).arrays)
    svc.detach()


def test_staging_handler_upload_policy():
    """StagingUpdateHandler decodes uploads for npz helpers only."""
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler

    class binaryhelper:          # noqa: N801 — helper_kind keys on the plug-in module / name
        name = "binaryhelper"

    st = StagingUpdateHandler(MemoryUpdateHandler(), helper=None, device="cpu", workers=1)
    assert st.wants_upload()
    st.helper = binaryhelper()
    assert not st.wants_upload()
    st.close()


def test_streaming_upload_tee_is_bounded():
    """More concurrent uploads than the tee allows take the normal path, and an upload that
    outpaces its decoder by more than max_queued_chunks is abandoned (not adopted): the chunks
    held in host memory stay bounded; every upload is still stored untouched."""
    store = MemoryModelStore()
    h = _Handler()
    svc = StreamingUpload(MemoryModelService(store), h, workers=1, pinned=False, max_queued_chunks=4)
    blocker = threading.Event()
    svc._pool.submit(blocker.wait)                       # the only worker is busy: decoders must queue
    data = _savez([np.arange(40_000, dtype=np.float32)])
    svc.Upload(upload_requests(data, "late", chunk=1000), None)       # 160 chunks >> 4 queued
    blocker.set()
    assert store.get("late").data == data
    assert "late" not in h.adopted or h.adopted["late"].exception(timeout=30) is not None
    gens = [iter(upload_requests(data, f"c{i}", chunk=20_000)) for i in range(6)]
    outs = [threading.Thread(target=svc.Upload, args=(g, None)) for g in gens]
    for t in outs:
        t.start()
    for t in outs:
        t.join(60)
    assert all(store.get(f"c{i}").data == data for i in range(6))
    svc.close()
    assert svc._free._value == 4                        # every decoder slot released


def _zip_npz(arrays, level):
    """An npz written by zipfile at a given deflate level (np.savez_compressed's container, other levels)."""
    import zipfile
    b = io.BytesIO()
    with zipfile.ZipFile(b, "w", compression=zipfile.ZIP_DEFLATED, compresslevel=level) as z:
        for i, a in enumerate(arrays):
            with z.open(f"{i}.npy", "w", force_zip64=True) as f:
                np.lib.format.write_array(f, np.asarray(a), allow_pickle=False)
    return b.getvalue()


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_decoder_streams_across_its_history_window(level):
    """Members of several MiB (the streaming decoder's output goes through a 1 MiB buffer whose last
    32 KiB carry the back-references), periodic data with long matches that straddle those
    compactions, sparse data and fp32 weights, fed in random pieces from 1 byte to 200 KiB:
    byte-identical to np.load."""
    rng = np.random.default_rng(11 + level)
    arrays = [rng.standard_normal(1_500_000).astype(np.float32),
              np.tile(rng.integers(0, 255, 30_011, dtype=np.uint8), 100),            # matches ~30 KB back
              np.where(rng.random(800_000) < 0.95, 0, rng.standard_normal(800_000)).astype(np.float32),
              np.arange(300_000, dtype=np.int64)]
    data = _zip_npz(arrays, level)
    dec = NpzStreamDecoder()
    o = 0
    while o < len(data):
        n = int(rng.integers(1, 200_000)) if rng.random() < 0.7 else int(rng.integers(1, 64))
        dec.feed(data[o:o + n])
        o += n
    _same_as_npload(data, DecodedUpdate(dec.finish(), None).arrays)


def test_streaming_upload_tee_byte_budget():
    """The tee's byte budget over all streams (max_queued_bytes): an upload whose decoder cannot run
    is abandoned once its queued chunks would pass it, even with room in its own queue; every
    queued byte is accounted back once the streams end."""
    store = MemoryModelStore()
    h = _Handler()
    svc = StreamingUpload(MemoryModelService(store), h, workers=1, pinned=False, max_queued_chunks=10_000,
                          max_queued_bytes=20_000)
    blocker = threading.Event()
    svc._pool.submit(blocker.wait)
    data = _savez([np.arange(40_000, dtype=np.float32)])
    svc.Upload(upload_requests(data, "big", chunk=1000), None)          # 160 chunks, 160 KB > 20 KB
    blocker.set()
    assert store.get("big").data == data
    assert "big" not in h.adopted or h.adopted["big"].exception(timeout=30) is not None
    ok = _savez([np.arange(1000, dtype=np.float32)])                   # 4 KB: within the budget
    svc.Upload(upload_requests(ok, "small", chunk=1000), None)
    assert h.adopted["small"].result(timeout=30) is not None
    svc.close()
    assert svc._queued == 0
