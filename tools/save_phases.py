"""Where the exact npz writer's time goes: Helper.save of one 100 M-param fp32
model (numpyhelper.save's archive, byte for byte) timed end to end and by phase on the box's threads.

fnpz_savez_stats (include/fednpz.h, ABI 7) reports the last big member's phases: the input copy
(header + payload into one buffer), pdeflate.h's parallel LZ77 parse, the sync of neighbouring
chunks' parses, the window schedule + tail replay (serial), the block plan (trees, parallel), the
encode (parallel, then the serial first-byte merge), the CRC (parallel pieces, serial combine), and
the archive assembly (headers, member streams copied into place). "other" = the call's total minus
those: Python's argument set-up and the output buffer. Each row is the best of --reps runs; every
archive is checked against the first (and, with --numpy, against np.savez_compressed once).

  python tools/save_phases.py [--threads 8,16] [--params 100000000] [--numpy]
"""
import argparse
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import codec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", default="8,16")
    ap.add_argument("--params", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--numpy", action="store_true", help="also time np.savez_compressed once and compare bytes")
    a = ap.parse_args()
    x = np.random.default_rng(0).standard_normal(a.params).astype(np.float32)
    print(json.dumps({"zlib": codec.savez_zlib_status(), "params": a.params, "MB": x.nbytes / 1e6}), flush=True)
    first = None
    for th in (int(t) for t in a.threads.split(",")):
        best = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = codec.savez_into([x], threads=th)
            dt = time.perf_counter() - t0
            st = codec.savez_stats()
            if first is None:
                first = out.tobytes()
            same = out.tobytes() == first
            del out
            if best is None or dt < best[0]:
                best = (dt, st, same)
        dt, st, same = best
        known = sum(v for k, v in st.items() if k != "total")
        row = {"threads": th, "save_s": round(dt, 4), "identical": same,
               **{k: round(v, 4) for k, v in st.items()}, "other": round(dt - known, 4),
               "serial_s": round(st["sched"] + (dt - st["total"]), 4)}
        print(json.dumps(row), flush=True)
    if a.numpy:
        b = io.BytesIO()
        t0 = time.perf_counter()
        np.savez_compressed(b, **{"0": x})
        print(json.dumps({"numpy_s": round(time.perf_counter() - t0, 3), "identical_to_numpy": b.getvalue() == first}),
              flush=True)


if __name__ == "__main__":
    main()
