"""Round wall time with the wire format in the loop: client
updates arrive as npz bytes (as ModelService.Upload stores them), are decoded and folded,
and the aggregate is encoded again for storage (roundhandler.py:465-470).

  reference-like  per update np.load (numpy inflate) serially inside the round, then the
                  GPU fold; np.savez_compressed of the result (what FEDn does on the host)
  plain plug-in   the aggregator without the ingest wrapper: np.load of up to 8 queued
                  updates concurrently ahead of the fold (aggregatorbase.queued_updates)
  fedn_amd        StagingUpdateHandler: each update inflated by the native codec straight
                  into pinned memory by a worker pool as it arrives + H2D, the fold in
                  combine_models, codec.save_npz (parallel deflate) of the result
The K updates reuse one numpy-written archive (identical decode work per update).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--workers", type=int, default=16)
    a = ap.parse_args()
    _abi.load()
    torch.cuda.set_device(0)
    K, P = a.clients, a.params
    x = torch.randn(P, device="cuda").cpu().numpy()
    t0 = time.perf_counter()
    b = io.BytesIO()
    np.savez_compressed(b, **{"0": x})
    t_np_enc = time.perf_counter() - t0
    blob = b.getvalue()
    t0 = time.perf_counter()
    ref = np.load(io.BytesIO(blob))["0"]
    t_np_dec = time.perf_counter() - t0
    t0 = time.perf_counter()
    mine = codec.load_npz(blob)[0]
    t_nat_dec = time.perf_counter() - t0
    assert np.array_equal(ref.view(np.uint32), mine.view(np.uint32))
    t0 = time.perf_counter()
    enc = codec.save_npz([x])
    t_nat_enc = time.perf_counter() - t0
    t0 = time.perf_counter()
    back = codec.load_npz(enc)[0]
    t_nat_dec_idx = time.perf_counter() - t0
    assert np.array_equal(back.view(np.uint32), x.view(np.uint32))
    print(json.dumps({"what": "codec", "params": P, "archive_MB": len(blob) / 1e6, "numpy_encode_s": t_np_enc,
                      "native_encode_s": t_nat_enc, "numpy_decode_s": t_np_dec, "native_decode_s": t_nat_dec,
                      "native_decode_own_archive_s": t_nat_dec_idx, "threads": codec.THREADS,
                      "host_cpus": os.cpu_count()}), flush=True)

    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryUpdateHandler
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]

    # reference-like: decode inside the round (serial), fold, numpy encode
    t0 = time.perf_counter()
    uh = MemoryUpdateHandler()
    for k in range(K):
        uh.submit_bytes(blob, ns[k])

    class NumpyHelper:                       # numpyhelper.load semantics (np.load of the npz)
        def load(self, f):
            z = np.load(f)
            return [z[str(i)] for i in range(len(z.files))]
    from fedn_amd.aggregators import aggregatorbase
    aggregatorbase.LOAD_AHEAD = 1            # FEDn's loop: each update decoded in turn
    model, data = get_aggregator("fedavg", uh).combine_models(helper=NumpyHelper())
    aggregatorbase.LOAD_AHEAD = 8
    b = io.BytesIO()
    np.savez_compressed(b, **{str(i): w for i, w in enumerate(model)})
    t_ref = time.perf_counter() - t0
    ref_model = model

    # the plain plug-in (no ingest wrapper): updates decoded 8 ahead of the fold (np.load)
    t0 = time.perf_counter()
    uh = MemoryUpdateHandler()
    for k in range(K):
        uh.submit_bytes(blob, ns[k])
    model_pf, data_pf = get_aggregator("fedavg", uh).combine_models(helper=NumpyHelper())
    t_plain = time.perf_counter() - t0
    exact_pf = all(np.array_equal(p.view(np.uint32), q.view(np.uint32)) for p, q in zip(model_pf, ref_model))

    # fedn_amd: staged on arrival, native codec both ways
    for _ in range(2):                       # first pass warms pinned / device pools
        t0 = time.perf_counter()
        uh = MemoryUpdateHandler()
        st = StagingUpdateHandler(uh, helper=Helper(), workers=a.workers)
        for k in range(K):
            uh.submit_bytes(blob, ns[k], via=st)
        model, data2 = get_aggregator("fedavg", st).combine_models(helper=Helper())
        out = codec.save_npz(model)
        t_ours = time.perf_counter() - t0
        st.close()
    exact = all(np.array_equal(p.view(np.uint32), q.view(np.uint32)) for p, q in zip(model, ref_model))
    print(json.dumps({"what": "round", "clients": K, "params": P, "reference_like_s": t_ref,
                      "reference_time_model_load": data["time_model_load"],
                      "plain_plugin_load_ahead8_s": t_plain, "plain_plugin_bit_exact": exact_pf,
                      "plain_plugin_time_model_load": data_pf["time_model_load"], "fedn_amd_s": t_ours,
                      "speedup": t_ref / t_ours, "bit_exact": exact, "workers": a.workers,
                      "fedn_amd_data": {k: round(v, 4) for k, v in data2.items() if isinstance(v, float)},
                      "encoded_MB": len(out) / 1e6}), flush=True)


if __name__ == "__main__":
    main()
