"""K updates (np.savez_compressed, one stream each) decoded at once, as the staging handler's
workers do when a burst of ModelUpdates arrives: wall time until all are decoded, per thread
budget of each load_npz call. CPU only."""
import io, os, sys, time, json
from concurrent.futures import ThreadPoolExecutor
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from fedn_amd import codec
if os.environ.get("LIB"):
    codec.LIB_PATH = os.environ["LIB"]
P, K = int(sys.argv[1]), int(sys.argv[2])
x = np.random.default_rng(0).standard_normal(P).astype(np.float32)
b = io.BytesIO(); np.savez_compressed(b, **{"0": x}); raw = b.getvalue()
res = {"params": P, "K": K, "lib": os.path.basename(codec.LIB_PATH)}
with ThreadPoolExecutor(K) as ex:
    for t in [int(v) for v in sys.argv[3:]]:
        best = 1e9
        for rep in range(3):
            t0 = time.perf_counter()
            done = list(ex.map(lambda r: (codec.load_npz(r, threads=t), time.perf_counter() - t0)[1], [raw] * K))
            best = min(best, max(done))
        res[f"threads{t}_s"] = round(best, 4)
print(json.dumps(res), flush=True)
