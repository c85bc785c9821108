"""Regenerate every golden fixture from the REAL reference into a scratch directory and diff it
against tests/golden/ (build container only: tools/gen_golden.py needs /root/reference).

Checks that ``manifest.json`` lists exactly the generator's cases in the generator's order, and
that every fixture is byte-identical (if the bytes of an archive differ, its arrays are compared
key by key — values bit for bit, NaN positions only — to say what differs). Exit status 0 when
``tests/golden/`` is exactly what ``python tools/gen_golden.py`` writes.

Usage: python tools/verify_golden.py [--keep DIR]
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "..", "tests", "golden")


def _same_array(a, b):
    if a.dtype != b.dtype or a.shape != b.shape:
        return False
    if a.dtype.kind == "f":
        na, nb = np.isnan(a), np.isnan(b)
        return bool(np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint8), b[~nb].view(np.uint8)))
    return a.tobytes() == b.tobytes()


def diff(regen_dir, golden_dir=GOLDEN):
    """Returns a list of human-readable differences (empty: identical)."""
    problems = []
    with open(os.path.join(regen_dir, "manifest.json")) as f:
        want = json.load(f)["cases"]
    with open(os.path.join(golden_dir, "manifest.json")) as f:
        have = json.load(f)["cases"]
    if want != have:
        missing, extra = sorted(set(want) - set(have)), sorted(set(have) - set(want))
        problems.append(f"manifest differs: missing {missing}, extra {extra}, order "
                        f"{'same' if not missing and not extra and want == have else 'differs'}")
    for name in want:
        g, r = os.path.join(golden_dir, name + ".npz"), os.path.join(regen_dir, name + ".npz")
        if not os.path.exists(g):
            problems.append(f"{name}: not in tests/golden")
            continue
        with open(g, "rb") as fg, open(r, "rb") as fr:
            if fg.read() == fr.read():
                continue
        zg, zr = np.load(g, allow_pickle=False), np.load(r, allow_pickle=False)
        keys = sorted(set(zg.files) | set(zr.files))
        bad = [k for k in keys if k not in zg.files or k not in zr.files or not _same_array(zg[k], zr[k])]
        problems.append(f"{name}: archive bytes differ" + (f"; arrays differ: {bad}" if bad else
                                                          " (arrays identical, NaN payloads aside)"))
    return problems


def main():
    keep = sys.argv[sys.argv.index("--keep") + 1] if "--keep" in sys.argv else None
    with tempfile.TemporaryDirectory() as tmp:
        out = keep or tmp
        subprocess.run([sys.executable, os.path.join(HERE, "gen_golden.py"), "--out", out], check=True,
                       stdout=subprocess.DEVNULL)
        problems = diff(out)
    for p in problems:
        print(p)
    print(f"verify_golden: {'OK, tests/golden is what gen_golden.py writes' if not problems else 'DIFFERS'}")
    return 1 if problems else 0


if __name__ == "__main__":
    raise SystemExit(main())
