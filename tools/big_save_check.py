"""A member past zipfile's real ZIP64_LIMIT (2 GiB - 1): Helper.save's exact writer against
np.savez_compressed (numpyhelper.py:162) at full size — the sha256 of both archives, their times,
and the decoder's read-back. tests/test_savez_zip64.py covers the same branches at lowered limits.

  python tools/big_save_check.py [--params 600000000] [--threads N]
"""
import argparse
import hashlib
import io
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import codec  # noqa: E402


def _rss():
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")


def _maxrss():
    import resource
    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=600_000_000)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    ws = [rng.standard_normal(a.params, dtype=np.float32), rng.standard_normal((512, 10)).astype(np.float32)]
    out = {"params": a.params, "member_bytes": ws[0].nbytes, "zip64_limit": (1 << 31) - 1, "threads": a.threads}
    rss0 = _rss()
    t = time.perf_counter()
    mine = codec.save_npz(ws, threads=a.threads)
    out["exact_s"] = round(time.perf_counter() - t, 2)
    # the writer's peak host memory above what the process held before (the archive it returns
    # included): ru_maxrss is the process's high-water mark
    out["exact_peak_extra_gb"] = round((_maxrss() - rss0) / 1e9, 2)
    out["exact_peak_extra_x_member"] = round((_maxrss() - rss0) / ws[0].nbytes, 2)
    h_mine = hashlib.sha256(mine).hexdigest()
    out["archive_bytes"] = len(mine)
    t = time.perf_counter()
    back = codec.load_npz(mine)
    out["native_load_s"] = round(time.perf_counter() - t, 2)
    out["read_back_equal"] = all(np.array_equal(x, y) for x, y in zip(back, ws))
    del mine, back
    b = io.BytesIO()
    t = time.perf_counter()
    np.savez_compressed(b, **{str(i): w for i, w in enumerate(ws)})
    out["numpy_s"] = round(time.perf_counter() - t, 2)
    out["zlib"] = codec.savez_zlib_status()
    ref = b.getbuffer()
    out["identical"] = hashlib.sha256(ref).hexdigest() == h_mine
    out["sha256"] = h_mine[:16]
    print(json.dumps(out), flush=True)
    if not out["identical"] or not out["read_back_equal"]:
        sys.exit(1)


if __name__ == "__main__":
    main()
