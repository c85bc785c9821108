"""Round tail with uploads in the loop (ModelService.Upload
modelservice.py:198-221 → SendModelUpdate combiner.py:783-797 → combine_models).

K clients upload the same numpy-written npz (np.savez_compressed, one deflate stream per
tensor, as FEDn clients write it) concurrently in 1 MiB chunks, each paced at
``--client-MBps``, then send their ModelUpdate; the round aggregates once all have arrived.

  after-arrival  StagingUpdateHandler alone: each update is inflated by the native codec
                 when its ModelUpdate arrives (after its last chunk), then H2D
  streaming-host StreamingUpload in front of the ModelService: the update is inflated while
                 its chunks arrive into pinned host blocks; the ModelUpdate triggers the H2D
  streaming      the same, inflated through DeviceSink's pinned ring straight to HBM while
                 the chunks arrive; the ModelUpdate only triggers a D2D into the layout

Reported: ``tail_s`` = last ModelUpdate → combine_models returned (what a round waits for
after its last byte landed), the round wall time, and bit-equality of the two modes with a
fold of the same updates handed over as host arrays.
"""
import argparse
import io
import json
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi  # noqa: E402


def run(mode, blob, ns, rate, workers, store="memory", delete_workers=None):
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.helper import Helper
    from fedn_amd.ingest import StagingUpdateHandler
    from fedn_amd.updatehandler import MemoryModelService, MemoryUpdateHandler, upload_requests
    from fedn_amd.upload import StreamingUpload

    from fedn_amd.updatehandler import MemoryModelStore, TempFileModelStore
    K = len(ns)
    uh = MemoryUpdateHandler(TempFileModelStore() if store == "file" else MemoryModelStore())
    st = StagingUpdateHandler(uh, helper=Helper(), workers=workers, delete_workers=delete_workers)
    svc = MemoryModelService(uh.store)
    if mode.startswith("streaming"):
        svc = StreamingUpload(svc, st, workers=K, device_decode=mode == "streaming")
    order, lock, last = [], threading.Lock(), [0.0]
    decoded_at = []
    adopt = st.adopt

    def adopt_timed(rid, fut):                        # when each streamed decode completed
        fut.add_done_callback(lambda f: decoded_at.append(time.perf_counter()))
        adopt(rid, fut)
    st.adopt = adopt_timed

    def client(k):
        def paced():
            t0, sent = time.perf_counter(), 0
            for req in upload_requests(blob, f"u{k}"):
                yield req
                sent += len(req.data)
                dt = sent / rate - (time.perf_counter() - t0)
                if dt > 0:
                    time.sleep(dt)
        svc.Upload(paced(), None)
        with lock:                                    # SendModelUpdate, in arrival order
            uh.submit_uploaded(f"u{k}", ns[k], via=st)
            order.append(k)
            last[0] = time.perf_counter()

    t0 = time.perf_counter()
    ths = [threading.Thread(target=client, args=(k,)) for k in range(K)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    t_agg = time.perf_counter()
    agg = get_aggregator("fedavg", st)
    t_init = time.perf_counter() - t_agg
    t_del = [0.0]
    delete = st.delete_model

    def delete_timed(mu):
        t = time.perf_counter()
        delete(mu)
        t_del[0] += time.perf_counter() - t
    st.delete_model = delete_timed
    model, data = agg.combine_models(helper=Helper())
    t1 = time.perf_counter()
    st.close()
    if mode.startswith("streaming"):
        svc.close()
    t_comb = t1 - t_agg
    return model, order, {"round_s": t1 - t0, "tail_s": t1 - last[0], "upload_s": last[0] - t0,
                          "decode_lag_s": (max(decoded_at) - last[0]) if decoded_at else None,
                          "combine_s": t_comb, "aggregator_init_s": t_init, "delete_s": t_del[0],
                          "delete_plugin_s": st.delete_times["plugin_s"], "delete_store_s": st.delete_times["store_s"],
                          "delete_wait_s": st.delete_times["wait_s"], "delete_workers": st.delete_workers,
                          "store": store, **{k: v for k, v in data.items() if isinstance(v, float)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--params", type=int, default=25_000_000)
    ap.add_argument("--client-MBps", type=float, default=250.0)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--delete-workers", type=int, default=None,
                    help="store deletes side by side on this many threads (0: inline, one after another)")
    ap.add_argument("--store", choices=("memory", "file"), default="memory",
                    help="the update store: in-memory bytes, or files + os.remove as FEDn's TempModelStorage")
    a = ap.parse_args()
    _abi.load()
    torch.cuda.set_device(0)
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    K, P = a.clients, a.params
    x = torch.randn(P, device="cuda").cpu().numpy()
    tensors = [x, np.arange(1000, dtype=np.float32)]
    b = io.BytesIO()
    np.savez_compressed(b, **{str(i): w for i, w in enumerate(tensors)})
    blob = b.getvalue()
    ns = [int(v) for v in np.random.default_rng(0).integers(1, 5001, K)]
    res = {}
    for rep in range(a.reps):                         # rep 0 warms pinned / device pools
        for mode in ("after-arrival", "streaming-host", "streaming"):
            model, order, t = run(mode, blob, ns, a.client_MBps * 1e6, a.workers, a.store, a.delete_workers)
            uh = MemoryUpdateHandler()                # the same fold from host arrays
            for k in order:
                uh.submit([w.copy() for w in tensors], ns[k])
            want, _ = get_aggregator("fedavg", uh).combine_models(helper=None)
            t["bit_exact"] = all(np.array_equal(p.view(np.uint8), q.view(np.uint8)) for p, q in zip(model, want))
            res[mode] = t
            print(json.dumps({"rep": rep, "mode": mode, **{k: (round(v, 4) if isinstance(v, float) else v)
                                                           for k, v in t.items()}}), flush=True)
    print(json.dumps({"what": "upload", "store": a.store, "clients": K, "params": P,
                      "archive_MB": round(len(blob) / 1e6, 1),
                      "delete_plugin_s": round(res["streaming"]["delete_plugin_s"], 4),
                      "delete_store_s": round(res["streaming"]["delete_store_s"], 4),
                      "delete_wait_s": round(res["streaming"]["delete_wait_s"], 4),
                      "delete_workers": res["streaming"]["delete_workers"],
                      "client_MBps": a.client_MBps, "tail_after_arrival_s": round(res["after-arrival"]["tail_s"], 4),
                      "tail_streaming_host_s": round(res["streaming-host"]["tail_s"], 4),
                      "tail_streaming_s": round(res["streaming"]["tail_s"], 4),
                      "round_after_arrival_s": round(res["after-arrival"]["round_s"], 4),
                      "round_streaming_s": round(res["streaming"]["round_s"], 4),
                      "bit_exact": all(r["bit_exact"] for r in res.values())}), flush=True)


if __name__ == "__main__":
    main()
