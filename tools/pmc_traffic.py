"""Turn rocprofv3 PMC runs of bench.py into per-launch HBM traffic for bench.py's roofline.

Usage: python tools/pmc_traffic.py <dir with pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/> <workload key> [kernel substring]
       [algorithmic bytes per launch]
       python tools/pmc_traffic.py --session gpurun_out/<tag>      (every workload of gpu_session.sh "pmc")

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
sys.path.insert(0, ROOT)


def file_sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def kernel_sha():
    """sha256 (16 hex) of fedn_amd/csrc/fedagg.hip (informational)."""
    return file_sha(os.path.join(ROOT, "fedn_amd", "csrc", "fedagg.hip"))


def lib_sha(session=None):
    """sha256 (16 hex) of the libfedagg.so the PMC runs loaded (written by gpu_session.sh into the
    session directory; else the in-tree file): bench.py reports an entry's traffic only while it
    loads that same library."""
    if session and os.path.exists(os.path.join(session, "lib_sha.txt")):
        return open(os.path.join(session, "lib_sha.txt")).read().split()[0][:16]
    return file_sha(os.path.join(ROOT, "fedn_amd", "libfedagg.so"))


def code_key(kernel, lib=None):
    """(mangled symbols, sha) of the measured kernels' gfx950 machine code in ``lib`` (default: the
    in-tree libfedagg.so, built from the source the PMC runs used): bench.py keeps an entry's traffic
    while the library it loads has the same bytes for those kernels (fedn_amd/codeobj.py)."""
    from fedn_amd import codeobj
    lib = lib or os.path.join(ROOT, "fedn_amd", "libfedagg.so")
    names = codeobj.kernels_matching(lib, kernel)
    if not names:
        raise SystemExit(f"no kernel matching {kernel!r} in {lib}")
    return names, codeobj.kernel_sha(lib, names)


def per_launch(path, kernel, take=None):
    """Average counter value per dispatch of the kernels whose name contains ``kernel`` (a string, or
    a tuple of strings that must all appear); ``take`` = (first, stop): only those dispatches of
    them, in dispatch order (two phases of one run that share a kernel instantiation)."""
    parts = (kernel,) if isinstance(kernel, str) else tuple(kernel)
    rows = [r for r in csv.DictReader(open(path)) if all(p in r["Kernel_Name"] for p in parts)]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    if take is not None:
        rows = rows[take[0]:take[1]]
    if not rows:
        raise SystemExit(f"no dispatch of {kernel!r} in {path}")
    vals = [float(r["Counter_Value"]) for r in rows]
    return sum(vals) / len(vals), len(vals)


def record(d, key, kernel, alg=None, session=None, take=None):
    fetch, nf = per_launch(os.path.join(d, "pmc_FETCH_SIZE", "run_counter_collection.csv"), kernel, take)
    write, nw = per_launch(os.path.join(d, "pmc_WRITE_SIZE", "run_counter_collection.csv"), kernel, take)
    read_b = 2 * fetch * 1024
    write_b = write * 1024
    out = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = {"bytes": read_b + write_b, "read_bytes": read_b, "write_bytes": write_b,
               "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write, "launches": [nf, nw], "kernel": kernel,
               "lib_sha": lib_sha(session), "kernel_src_sha": kernel_sha(), "collected": datetime.date.today().isoformat(),
               "alg_bytes": alg, "traffic_over_alg": None if not alg else (read_b + write_b) / alg,
               "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count on 16-B streaming loads); "
                             "write = WRITE_SIZE x 1024"}
    db[key]["symbols"], db[key]["code_sha"] = code_key(kernel)
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps({key: db[key]}))


# the workloads bench.py reports (tools/gpu_session.sh step "pmc" runs the passes into pmc1..3)
P, Q = 100_000_000, 350_000_000
SESSION = [
    # the fp32 fold's first launch stores inside the chip-wide clock window (k_fedavg_pipe_win)
    ("pmc1", f"fedavg_k64_p{P}_f32", "k_fedavg_pipe_win<float, float", 64 * P * 4 + P * 4),
    # bench.py's fedopt field: every phase is one windowed launch per round (k_fedopt_cw, K = 32); round 1
    # (12 launches) and the fp32-state phase (12 more) are both k_fedopt_cw<float, float, CF32>: round 1
    # is the first 12 dispatches
    ("pmc1", f"fedopt_adam_round1_k32_p{Q}", "k_fedopt_cw<float, float", 32 * Q * 4 + Q * 24, (0, 12)),
    ("pmc1", f"fedopt_adam_steady_k32_p{Q}", "k_fedopt_cw<float, double", Q * (4 * 32 + 48)),
    ("pmc2", f"fedavg_k8_p{P}_f32", "k_fedavg_pipe_win<float, float", 8 * P * 4 + P * 4),
    ("pmc3", f"fedavg_k64_p{P}_bf16", "k_fedavg_pipe_win<(anonymous namespace)::bf16, float", 64 * P * 2 + P * 4),
]


# tools/pmc_workloads.py runs (tools/gpu_session.sh step "pmcx"): (subdir, key, kernel, algorithmic bytes)
WAVE_BF16 = "k_fedopt_c<(anonymous namespace)::bf16, double, (anonymous namespace)::CF64, "
X_SESSION = [
    ("pmcx_f32state", f"fedopt_adam_steady_f32state_k32_p{Q}", "k_fedopt_cw<float, float", Q * (4 * 32 + 24)),
    ("pmcx_waves", "fedyogi_wave_first_p1000000000_w8_bf16", (WAVE_BF16 + "true, false,",), 1_000_000_000 * (2 * 8 + 16)),
    ("pmcx_waves", "fedyogi_wave_mid_p1000000000_w8_bf16", (WAVE_BF16 + "false, false,",), 1_000_000_000 * (2 * 8 + 24)),
    ("pmcx_waves", "fedyogi_wave_final_p1000000000_w8_bf16", (WAVE_BF16 + "false, true,",), 1_000_000_000 * 40, (0, 3)),
    # the fused last wave (8 bf16 updates, f64 old + pg read; f64 m / v / out written): dispatches 3..5
    ("pmcx_waves", "fedyogi_wave_mid_final_p1000000000_w8_bf16", (WAVE_BF16 + "false, true,",),
     1_000_000_000 * (2 * 8 + 40), (3, 6)),
]


def record_rank(session, world, R=8, sub=None):
    """bench.py's N > 1 roofline entry: one rank's fold per step = ``rounds`` launches of the replayed
    chunk fold (tools/pmc_rank_fold.py, --ag-rounds R); bytes per step = per-launch bytes x rounds."""
    from tools.pmc_rank_fold import rank_geometry
    C, rounds, L = rank_geometry(100_000_000, world, R)
    d = os.path.join(session, sub or f"pmcrank{world}")
    # the product's geometry rule (fedagg.hip kPipeMinClientBytes, bench.fold_kernel_label)
    kernel = "k_fedavg_pipe<float, float" if C * 4 >= 160 << 20 else "k_fedavg<float, float"
    fetch, nf = per_launch(os.path.join(d, "pmc_FETCH_SIZE", "run_counter_collection.csv"), kernel)
    write, nw = per_launch(os.path.join(d, "pmc_WRITE_SIZE", "run_counter_collection.csv"), kernel)
    read_b, write_b = 2 * fetch * 1024 * rounds, write * 1024 * rounds
    alg = rounds * (64 * C * 4 + C * 4)
    key = f"fedavg_k64_p{L}_r{rounds}_f32_rank_of_{world}"
    out = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[key] = {"bytes": read_b + write_b, "read_bytes": read_b, "write_bytes": write_b,
               "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write, "launches": [nf, nw], "kernel": kernel,
               "per": f"one rank's step: {rounds} launches of 64 x {C} fp32 (replayed on one GPU)",
               "lib_sha": lib_sha(session), "kernel_src_sha": kernel_sha(), "collected": datetime.date.today().isoformat(),
               "alg_bytes": alg, "traffic_over_alg": (read_b + write_b) / alg,
               "correction": "read = 2 x FETCH_SIZE x 1024 (gfx950 half-count on 16-B streaming loads); "
                             "write = WRITE_SIZE x 1024"}
    db[key]["symbols"], db[key]["code_sha"] = code_key(kernel)
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps({key: db[key]}))


def annotate(lib):
    """Key every existing entry on its kernels' machine code in ``lib`` — a build of the fedagg.hip the
    entries were collected on (their kernel_src_sha), at any path."""
    out = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    db = json.load(open(out))
    for key, ent in db.items():
        ent["symbols"], ent["code_sha"] = code_key(ent["kernel"], lib)
        print(key, ent["code_sha"], len(ent["symbols"]))
    json.dump(db, open(out, "w"), indent=1)


def main():
    if sys.argv[1] == "--annotate":
        return annotate(sys.argv[2])
    if sys.argv[1] == "--rank-session":
        for world in (2, 4, 8):
            for R in (1, 2, 4, 8, 16):   # bench.py AG_ROUNDS
                sub = f"pmcrank{world}_r{R}"
                if os.path.isdir(os.path.join(sys.argv[2], sub)):
                    record_rank(sys.argv[2], world, R, sub)
            if os.path.isdir(os.path.join(sys.argv[2], f"pmcrank{world}")):   # round-2 sessions: R = 8 only
                record_rank(sys.argv[2], world)
        return
    if sys.argv[1] == "--x-session":
        for sub, key, kernel, alg, *take in X_SESSION:
            record(os.path.join(sys.argv[2], sub), key, kernel, alg, session=sys.argv[2], take=take[0] if take else None)
        return
    if sys.argv[1] == "--session":
        for sub, key, kernel, alg, *take in SESSION:
            record(os.path.join(sys.argv[2], sub), key, kernel, alg, session=sys.argv[2], take=take[0] if take else None)
        return
    d, key = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_fedavg"
    alg = float(sys.argv[4]) if len(sys.argv) > 4 else None
    record(d, key, kernel, alg)


if __name__ == "__main__":
    main()
