"""Turn rocprofv3 PMC runs of bench.py into per-launch HBM traffic for bench.py's roofline.

Usage: python tools/pmc_traffic.py <dir with pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/> <workload key> [kernel substring]
       [algorithmic bytes per launch]

gfx950 corrections (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE reports exactly 1/2 of the bytes of a wide (16 B/lane)
coalesced streaming read, so read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is exact for
16-B-per-lane streaming stores. Each counter comes from its own pass (--pmc X --kernel-trace).
"""
import csv
import datetime
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_sha():
    """sha256 (16 hex) of fedn_amd/csrc/fedagg.hip: bench.py reports an entry's traffic only while
    the kernel source is the one it was measured on."""
    with open(os.path.join(ROOT, "fedn_amd", "csrc", "fedagg.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def per_launch(path, kernel):
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    if not rows:
        raise SystemExit(f"no dispatch of {kernel!r} in {path}")
    vals = [float(r["Counter_Value"]) for r in rows]
    return sum(vals) / len(vals), len(vals)


def main():
    d, key = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_fedavg"
    alg = float(sys.argv[4]) if len(sys.argv) > 4 else None
    fetch, nf = per_launch(os.path.join(d, "pmc_FETCH_SIZE", "run_counter_collection.csv"), kernel)
    write, nw = per_launch(os.path.join(d, "pmc_WRITE_SIZE", "run_counter_collection.csv"), kernel)
    read_b = 2 * fetch * 1024
    write_b = write * 1024
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json")
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = {"bytes": read_b + write_b, "read_bytes": read_b, "write_bytes": write_b,
               "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write, "launches": [nf, nw], "kernel": kernel,
               "kernel_src_sha": kernel_sha(), "collected": datetime.date.today().isoformat(),
               "alg_bytes": alg, "traffic_over_alg": None if not alg else (read_b + write_b) / alg,
               "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count on 16-B streaming loads); "
                             "write = WRITE_SIZE x 1024"}
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps(db[key]))


if __name__ == "__main__":
    main()
