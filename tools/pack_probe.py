"""Host copy rates into the kinds of host memory a small-update pack can target (the arena's pinned
bytes), to find what bounds the pack of many small updates: torch pinned (hipHostMalloc),
pageable numpy, and pageable memory page-locked with hipHostRegister (fa_host_register); each with
1 and 8 native threads (fnpz_gather), plus the H2D rate from each."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, codec, ops  # noqa: E402


def main():
    _abi.load()
    K, n = 64, 52650
    srcs = [np.random.default_rng(k).standard_normal(n).astype(np.float32) for k in range(K)]
    nbytes = K * n * 4
    pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    pageable = np.empty(nbytes, np.uint8)
    registered = np.empty(nbytes + 4096, np.uint8)
    off = (-registered.ctypes.data) % 4096
    registered = registered[off:off + nbytes]
    reg_t = torch.from_numpy(registered)
    ops.host_register(reg_t)
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda:0")
    out = {}
    for name, buf in (("torch_pinned", pinned.numpy()), ("pageable", pageable), ("host_registered", registered)):
        for threads in (1, 8):
            pairs = [(buf[k * n * 4:(k + 1) * n * 4].view(np.float32), s) for k, s in enumerate(srcs)]
            for _ in range(3):
                codec.gather(pairs, threads)
            t0 = time.perf_counter()
            for _ in range(20):
                codec.gather(pairs, threads)
            dt = (time.perf_counter() - t0) / 20
            out[f"{name}_t{threads}_GBps"] = nbytes / dt / 1e9
        src = torch.from_numpy(buf)
        for _ in range(3):
            dev.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            dev.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        out[f"{name}_h2d_GBps"] = nbytes / ((time.perf_counter() - t0) / 20) / 1e9
    ops.host_unregister(reg_t)
    print(json.dumps({"bytes": nbytes, **{k: round(v, 2) for k, v in out.items()}}), flush=True)
    large()


def large(P=100_000_000, reps=5):
    """The pack of ONE large update (a 100 M-param fp32 model, 400 MB) into a pinned slot with 4..64
    native threads: what bounds the multi-device plug-in, whose GPUs each take only a slice of every
    packed update over their own links (multidev.py)."""
    src = np.random.default_rng(0).standard_normal(P).astype(np.float32)
    dst = torch.empty(P * 4, dtype=torch.uint8, pin_memory=True).numpy().view(np.float32)
    res = {}
    for threads in (4, 8, 16, 24, 32, 48, 64):
        codec.gather([(dst, src)], threads)
        t0 = time.perf_counter()
        for _ in range(reps):
            codec.gather([(dst, src)], threads)
        res[f"t{threads}_GBps"] = round(P * 4 / ((time.perf_counter() - t0) / reps) / 1e9, 1)
    print(json.dumps({"large_update_bytes": P * 4, **res}), flush=True)


def inplace(P=100_000_000, updates=6, threads=24):
    """the multi-device host-resident round packs every update once into pinned
    memory (each GPU then takes its slice over its own link) at ~80-112 GB/s, about two links' worth.
    The alternative page-locks each decoded update IN PLACE (hipHostRegister of the numpy array) and
    H2D's straight from it — no copy, but a pinning cost per update (every round's updates are fresh
    memory). Per 100 M-param fp32 update (400 MB, fresh numpy arrays, first-touched): register,
    H2D (whole update to one GPU), unregister — against the native pack + H2D from a pinned slot."""
    rng = np.random.default_rng(1)
    dev = torch.empty(P * 4, dtype=torch.uint8, device="cuda:0")
    slot = torch.empty(P * 4, dtype=torch.uint8, pin_memory=True)
    st = torch.cuda.current_stream()
    rows = {"register_ms": [], "unregister_ms": [], "h2d_registered_ms": [], "pack_ms": [], "h2d_pinned_ms": [],
            "h2d_pageable_ms": []}
    for _ in range(updates):
        arr = rng.standard_normal(P, dtype=np.float32)           # a fresh decoded update
        t = torch.from_numpy(arr)
        t0 = time.perf_counter()
        try:
            ops.host_register(t)                                 # malloc'd: not page-aligned
        except Exception as e:  # noqa: BLE001 — reported, then the probe stops
            print(json.dumps({"inplace_register_error": str(e), "addr_mod_4096": arr.ctypes.data % 4096}), flush=True)
            return
        rows["register_ms"].append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        ops.copy_ptr_async(dev.data_ptr(), arr.ctypes.data, P * 4, st, torch.device("cuda", 0))
        st.synchronize()
        rows["h2d_registered_ms"].append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        ops.host_unregister(t)
        rows["unregister_ms"].append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        codec.gather([(slot.numpy().view(np.float32), arr)], threads)
        rows["pack_ms"].append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        dev.copy_(slot, non_blocking=True)
        st.synchronize()
        rows["h2d_pinned_ms"].append((time.perf_counter() - t0) * 1e3)
        t0 = time.perf_counter()
        dev.copy_(t.view(torch.uint8), non_blocking=True)
        st.synchronize()
        rows["h2d_pageable_ms"].append((time.perf_counter() - t0) * 1e3)
        del arr, t
    res = {k: round(float(np.median(v[1:])), 3) for k, v in rows.items()}       # the first update warms up
    res["register_GBps"] = round(P * 4 / res["register_ms"] / 1e6, 1)
    res["pack_GBps"] = round(P * 4 / res["pack_ms"] / 1e6, 1)
    res["h2d_registered_GBps"] = round(P * 4 / res["h2d_registered_ms"] / 1e6, 1)
    res["h2d_pinned_GBps"] = round(P * 4 / res["h2d_pinned_ms"] / 1e6, 1)
    res["h2d_pageable_GBps"] = round(P * 4 / res["h2d_pageable_ms"] / 1e6, 1)
    print(json.dumps({"inplace_update_bytes": P * 4, "pack_threads": threads, **res}), flush=True)


def busy(P=100_000_000, reps=4):
    """hipHostRegister / hipHostUnregister of one 400 MB update while the copy engines are busy with
    another update's H2D (what a pipelined round does): whether either call waits for the DMA."""
    rng = np.random.default_rng(2)
    dev = torch.empty(P * 4, dtype=torch.uint8, device="cuda:0")
    side = torch.empty(P * 4, dtype=torch.uint8, pin_memory=True)
    cs = torch.cuda.Stream()
    arrs = [rng.standard_normal(P, dtype=np.float32) for _ in range(2)]
    res = {"register_idle_ms": [], "register_busy_ms": [], "unregister_idle_ms": [], "unregister_busy_ms": [],
           "h2d_ms": []}
    for _ in range(reps):
        for busy_ in (False, True):
            a = arrs[0]
            if busy_:
                with torch.cuda.stream(cs):
                    dev.copy_(side, non_blocking=True)          # ~7 ms of DMA in flight
            t0 = time.perf_counter()
            ops.host_register_ptr(a.ctypes.data, a.nbytes)
            res["register_busy_ms" if busy_ else "register_idle_ms"].append((time.perf_counter() - t0) * 1e3)
            cs.synchronize()
            if busy_:
                with torch.cuda.stream(cs):
                    dev.copy_(side, non_blocking=True)
            t0 = time.perf_counter()
            ops.host_unregister_ptr(a.ctypes.data)
            res["unregister_busy_ms" if busy_ else "unregister_idle_ms"].append((time.perf_counter() - t0) * 1e3)
            cs.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(cs):
            dev.copy_(side, non_blocking=True)
        cs.synchronize()
        res["h2d_ms"].append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"busy_probe_bytes": P * 4, **{k: round(float(np.median(v)), 3) for k, v in res.items()}}),
          flush=True)


if __name__ == "__main__":
    if "--busy" in sys.argv:
        _abi.load()
        busy()
    elif "--inplace" in sys.argv:
        _abi.load()
        inplace()
    else:
        main()
