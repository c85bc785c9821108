"""Controller reduce (``Control.reduce`` control.py:648-693): C
combiner models held as npz bytes in a repository are fetched, decoded and averaged
unweighted (``increment_average(model, next, 1.0, i)``, control.py:682).

  reference-like  np.load per model (numpyhelper.load) + numpy increment_average on the host
                  (x + 1.0*(y - x)/i, fp32), the same loop as control.py
  fedn_amd        fedn_amd.reduce.reduce_models: decode with the native codec, fold on the GPU
                  (FedAvgPipeline, n = 1.0, N = i), result back to the host

Both decode the same bytes; the timings are split into load and aggregate as Control.reduce
reports them (meta keys), and the results are compared bit for bit.
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, codec  # noqa: E402


def reference_like(combiners, repo):
    """control.py:648-693 with numpyhelper (np.load; [np.add(x, n*(y-x)/N)], numpyhelper.py:32)."""
    meta = {"time_fetch_model": 0.0, "time_load_model": 0.0, "time_aggregate_model": 0.0}
    i, model = 1, None
    for c in combiners:
        data = repo[c["model_id"]]
        tic = time.time()
        z = np.load(io.BytesIO(data))
        model_next = [z[str(j)] for j in range(len(z.files))]
        meta["time_load_model"] += time.time() - tic
        tic = time.time()
        if model is None:
            model = model_next
        else:
            model = [np.add(x, 1.0 * (y - x) / i) for x, y in zip(model, model_next)]
        meta["time_aggregate_model"] += time.time() - tic
        i += 1
    return model, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--combiners", type=int, default=8)
    ap.add_argument("--params", type=int, default=100_000_000)
    a = ap.parse_args()
    _abi.load()
    torch.cuda.set_device(0)
    from fedn_amd.reduce import reduce_models
    C, P = a.combiners, a.params
    g = torch.Generator(device="cuda").manual_seed(0)
    base = torch.randn(P, device="cuda", generator=g)
    repo, combiners = {}, []
    for c in range(C):
        w = (base + 0.01 * torch.randn(P, device="cuda", generator=g)).cpu().numpy()
        b = io.BytesIO()
        np.savez_compressed(b, **{"0": w, "1": np.arange(1000, dtype=np.float32) * c})
        repo[f"m{c}"] = b.getvalue()
        combiners.append({"name": f"combiner{c}", "model_id": f"m{c}"})

    t0 = time.perf_counter()
    ref, ref_meta = reference_like(combiners, repo)
    t_ref = time.perf_counter() - t0
    res = {}
    for rep in range(2):                     # rep 0 warms pinned / device pools
        t0 = time.perf_counter()
        model, meta = reduce_models(combiners, fetch=repo.__getitem__, load=codec.load_npz)
        res = {"s": time.perf_counter() - t0, **meta}
    exact = all(np.array_equal(p.view(np.uint8), q.view(np.uint8)) for p, q in zip(model, ref))
    print(json.dumps({"what": "reduce", "combiners": C, "params": P,
                      "reference_like_s": round(t_ref, 4),
                      "reference_like": {k: round(v, 4) for k, v in ref_meta.items()},
                      "fedn_amd_s": round(res["s"], 4),
                      "fedn_amd": {k: round(v, 4) for k, v in res.items() if k != "s"},
                      "aggregate_speedup": round(ref_meta["time_aggregate_model"] / res["time_aggregate_model"], 1),
                      "bit_exact": exact, "host_cpus": os.cpu_count(), "codec_threads": codec.THREADS}), flush=True)


if __name__ == "__main__":
    main()
