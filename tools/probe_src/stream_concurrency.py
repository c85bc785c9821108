import io, sys, time, threading, numpy as np
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__)))))
from fedn_amd.upload import NpzStreamDecoder
from fedn_amd import codec
P = int(sys.argv[1]); T = int(sys.argv[2]); CH = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
x = np.random.default_rng(0).standard_normal(P).astype(np.float32)
b = io.BytesIO(); np.savez_compressed(b, **{"0": x, "1": np.arange(1000, dtype=np.float32)}); blob = b.getvalue()
chunks = [blob[i:i + CH] for i in range(0, len(blob), CH)]
def one():
    d = NpzStreamDecoder(alloc=lambda n: np.empty(n, np.uint8))
    for c in chunks: d.feed(c)
    return d.finish()
t = time.perf_counter(); codec.load_npz(blob, threads=1); t1 = time.perf_counter() - t
t = time.perf_counter(); m = one(); ts = time.perf_counter() - t
assert np.array_equal(m[0][3].view(np.float32), x)
ths = [threading.Thread(target=one) for _ in range(T)]
t = time.perf_counter()
for th in ths: th.start()
for th in ths: th.join()
tc = time.perf_counter() - t
MB = len(blob) / 1e6
print(f"blob {MB:.0f} MB; load_npz 1 thread {MB/t1:.0f} MB/s; stream 1 {MB/ts:.0f} MB/s; stream x{T} {T*MB/tc:.0f} MB/s total ({MB/tc:.0f} per stream)")
