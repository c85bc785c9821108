"""A/B of codec builds on one box: load_npz of a numpy-written single-tensor update through each
libfednpz variant given on the command line, alternating, best of rounds. Probe, not product."""
import io
import json
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from fedn_amd import codec  # noqa: E402

P = int(sys.argv[1])
libs = sys.argv[2:]
x = np.random.default_rng(0).standard_normal(P).astype(np.float32)
b = io.BytesIO()
np.savez_compressed(b, **{"0": x})
raw = b.getvalue()
best = {lib: 1e9 for lib in libs}
for _ in range(4):
    for lib in libs:
        codec.LIB_PATH, codec._lib = lib, None
        y = codec.load_npz(raw)[0]
        assert np.array_equal(y.view(np.uint32), x.view(np.uint32))
        t = time.perf_counter()
        codec.load_npz(raw)
        best[lib] = min(best[lib], time.perf_counter() - t)
print(json.dumps({lib.rsplit("/", 1)[-1]: round(v, 4) for lib, v in best.items()}))
