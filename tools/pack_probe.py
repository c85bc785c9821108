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


if __name__ == "__main__":
    main()
