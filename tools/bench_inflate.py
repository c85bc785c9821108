"""Decode of FEDn-written updates (np.savez_compressed: ONE deflate stream per member,
numpyhelper.py:144-169) on the host: numpy's own np.load (what numpyhelper.load does), and the
plug-in's native codec (codec.load_npz: fedn_amd/csrc/inflate.h's decoder + folded CRC-32). One
update alone (one core per member), and ``--clients`` updates decoded concurrently (the read-ahead's
shape, one member per core). Every decode compared bit-for-bit with the source arrays. CPU only.

    python tools/bench_inflate.py [--params 25000000 100000000] [--clients 16] [--threads 16]
"""
import argparse
import io
import json
import os
import sys
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import codec  # noqa: E402


def best(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, nargs="+", default=[25_000_000, 100_000_000])
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    for P in a.params:
        x = rng.standard_normal(P).astype(np.float32)
        b = io.BytesIO()
        np.savez_compressed(b, **{"0": x})
        raw = b.getvalue()
        out = {"params": P, "MB": x.nbytes / 1e6, "archive_MB": len(raw) / 1e6}

        def np_load():
            with np.load(io.BytesIO(raw)) as z:
                return z["0"]
        got = np_load()
        assert np.array_equal(got.view(np.uint32), x.view(np.uint32))
        out["numpy_load_s"] = best(np_load, a.reps)
        got = codec.load_npz(raw)[0]
        assert np.array_equal(got.view(np.uint32), x.view(np.uint32))
        out["native_load_s"] = best(lambda: codec.load_npz(raw), a.reps)
        out["numpy_MBps"] = x.nbytes / out["numpy_load_s"] / 1e6
        out["native_MBps"] = x.nbytes / out["native_load_s"] / 1e6
        out["speedup"] = out["numpy_load_s"] / out["native_load_s"]
        out["crc32_native_GBps"] = x.nbytes / best(lambda: codec.crc32(x), a.reps) / 1e9
        out["crc32_zlib_GBps"] = x.nbytes / best(lambda: zlib.crc32(x), a.reps) / 1e9
        # the other direction: the combiner's model serialisation (helper.save)
        t_np = best(lambda: np.savez_compressed(io.BytesIO(), **{"0": x}), 1)
        out["encode"] = {"numpy_s": t_np, "numpy_MB": len(raw) / 1e6}
        # helper.save's default: numpy's exact bytes (fnpz_savez; one big member -> pdeflate.h)
        exact = codec.save_npz([x], threads=a.threads)
        out["encode"]["exact_identical_to_numpy"] = exact == raw
        out["encode"]["exact_s"] = best(lambda: codec.save_npz([x], threads=a.threads), a.reps)
        out["encode"]["exact_speedup"] = t_np / out["encode"]["exact_s"]
        # a helper-written archive is numpy's: the decoder's single-stream split applies to it
        out["native_load_helper_written_s"] = best(lambda: codec.load_npz(exact), a.reps)
        for strat in ("default", "auto"):
            enc = codec.save_npz_blocks([x], threads=a.threads, strategy=strat)   # FEDN_AMD_NPZ_WRITER=blocks
            got = np.load(io.BytesIO(enc))["0"]
            assert np.array_equal(got.view(np.uint32), x.view(np.uint32))
            out["encode"][f"native_{strat}_s"] = best(lambda: codec.save_npz_blocks([x], threads=a.threads, strategy=strat), a.reps)
            out["encode"][f"native_{strat}_MB"] = len(enc) / 1e6
        if a.clients > 1 and P <= 25_000_000:
            archives = [raw] * a.clients
            with ThreadPoolExecutor(a.threads) as ex:
                def many(fn):
                    return list(ex.map(fn, archives))
                many(lambda r: codec.load_npz(r, threads=1))
                out["concurrent"] = {
                    "clients": a.clients, "threads": a.threads,
                    "native_GBps": a.clients * x.nbytes / best(lambda: many(lambda r: codec.load_npz(r, threads=1)),
                                                               a.reps) / 1e9,
                    "numpy_GBps": a.clients * x.nbytes / best(lambda: many(lambda r: np.load(io.BytesIO(r))["0"]),
                                                              a.reps) / 1e9}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
