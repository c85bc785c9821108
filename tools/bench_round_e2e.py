"""A combiner's round end, FEDn's way and the plug-in's, down to the global-model blob it stores.

After ``combine_models`` FEDn serialises the new model right away (roundhandler.py:465-470 ->
serialize_model_to_BytesIO, modelservice.py:128-146: ``helper.save(model)`` to a temp file, read
back, unlinked) and hands the bytes to the repository. Both steps sit between the last update and
the next round. This times them for K host-resident updates (numpy arrays, as ``helper.load``
returns them):

  reference  fedavg.py:45-83 restated around the oracle's numpyhelper arithmetic
             (tools/bench_small.py), then numpyhelper.save = np.savez_compressed
  plug-in    fedn_amd's FedAvg combine_models (GPU fold), then fedn_amd.helper.Helper.save
             (numpy's exact archive, fnpz_savez / pdeflate.h)

and checks that the two blobs are byte-identical. Run on the GPU box:
  python tools/bench_round_e2e.py [--params 100000000] [--clients 8]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi  # noqa: E402
from fedn_amd.aggregators import get_aggregator  # noqa: E402
from fedn_amd.helper import Helper  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_small  # noqa: E402  (the reference loop on the oracle's arithmetic: the CPU baseline)


def serialize(model, save):
    """serialize_model_to_BytesIO's steps (modelservice.py:128-146) with ``save(model) -> path``."""
    path = save(model)
    with open(path, "rb") as f:
        blob = f.read()
    os.unlink(path)
    return blob


def numpyhelper_save(weights):
    """numpyhelper.Helper.save (numpyhelper.py:144-169): np.savez_compressed of {str(i): w}."""
    fd, path = tempfile.mkstemp(suffix=".npz")
    os.close(fd)
    np.savez_compressed(path, **{str(i): w for i, w in enumerate(weights)})
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    _abi.load()
    P = a.params
    shapes = [(P // 2,), (P // 4,), (P - P // 2 - P // 4 - 10,), (10,)]
    rng = np.random.default_rng(7)
    base = [rng.standard_normal(s, dtype=np.float32) for s in shapes]
    ups = [[(b + np.float32(0.01) * rng.standard_normal(b.shape, dtype=np.float32)) for b in base]
           for _ in range(a.clients)]
    ns = [int(v) for v in rng.integers(1, 5001, a.clients)]
    helper = Helper()
    out = {"params": P, "clients": a.clients, "tensors": len(shapes)}
    for rep in range(a.reps):
        uh = MemoryUpdateHandler()
        agg = get_aggregator("fedavg", uh)
        for u, n in zip(ups, ns):
            uh.submit(u, n)
        t = time.perf_counter()
        model, _ = agg.combine_models(helper=helper)
        t1 = time.perf_counter()
        blob = serialize(model, helper.save)
        t2 = time.perf_counter()
        out["plugin_combine_s"], out["plugin_save_s"] = round(t1 - t, 3), round(t2 - t1, 3)
        out["plugin_round_end_s"] = round(t2 - t, 3)
        del model
    uh = MemoryUpdateHandler()
    for u, n in zip(ups, ns):
        uh.submit(u, n)
    t = time.perf_counter()
    ref_model, _ = bench_small.fedn_loop_fedavg(uh)
    t1 = time.perf_counter()
    ref_blob = serialize(ref_model, numpyhelper_save)
    t2 = time.perf_counter()
    out["reference_combine_s"], out["reference_save_s"] = round(t1 - t, 3), round(t2 - t1, 3)
    out["reference_round_end_s"] = round(t2 - t, 3)
    out["blob_MB"] = round(len(ref_blob) / 1e6, 1)
    out["blob_identical"] = blob == ref_blob
    out["speedup"] = round(out["reference_round_end_s"] / out["plugin_round_end_s"], 1)
    print(json.dumps(out), flush=True)
    if not out["blob_identical"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
