"""Host native code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only, build container).

Builds ``libfednpz.so`` (csrc/npz_codec.cpp: the npz codec and the native pack / gather;
csrc/savez.cpp + pdeflate.h: the numpy-identical writer and its parallel deflate) and the
``_fastpack`` extension (csrc/fastpack.c: admission + pack of small updates) with
``-fsanitize=address,undefined`` into a scratch copy of the package, then runs the CPU tests that
drive them — the codec, decoder, upload, writer (golden bytes, ZIP64, zlib-exact parallel
deflate), pack and staging-host tests —
inside that copy with the sanitizer runtimes preloaded into the (uninstrumented) Python. Any
sanitizer report aborts the run (``halt_on_error``); the summary goes to stdout.

    python tools/asan_host.py [--out profiles/r05_asan_host.log]

GPU code is not sanitized here (no GPU sanitizer on this pool); libfedagg.so is copied as built.
"""
import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# (not tests/test_codec_nomem.py: it caps the address space, which ASan's shadow memory cannot live in)
TESTS = ["tests/test_codec.py", "tests/test_inflate.py", "tests/test_upload.py", "tests/test_fastpack.py",
         "tests/test_staging_host.py", "tests/test_savez_golden.py", "tests/test_savez_zip64.py", "tests/test_pdeflate.py"]
SAN = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", "-g", "-O1"]


def runtime(name):
    out = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True, check=True).stdout.strip()
    if not os.path.isabs(out) or not os.path.exists(out):
        raise SystemExit(f"sanitizer runtime {name} not found")
    return os.path.realpath(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None, help="also write the log here")
    a = ap.parse_args()
    import numpy
    log = []

    def say(msg):
        print(msg, flush=True)
        log.append(msg)

    with tempfile.TemporaryDirectory(prefix="fedn_asan_") as tmp:
        for d in ("fedn_amd", "tests", "oracle", "include"):
            shutil.copytree(os.path.join(ROOT, d), os.path.join(tmp, d),
                            ignore=shutil.ignore_patterns("__pycache__", "*.pyc", "_fastpack.so", "libfednpz.so"))
        shutil.copy(os.path.join(ROOT, "bench.py"), tmp)
        pkg = os.path.join(tmp, "fedn_amd")
        cmds = [["g++", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", *SAN, "-I", os.path.join(tmp, "include"),
                 "-o", os.path.join(pkg, "libfednpz.so"), os.path.join(pkg, "csrc", "npz_codec.cpp"),
                 os.path.join(pkg, "csrc", "savez.cpp"), "-lz"],
                ["gcc", "-fPIC", "-shared", "-Wall", *SAN, "-I", sysconfig.get_paths()["include"], "-I",
                 numpy.get_include(), "-o", os.path.join(pkg, "_fastpack.so"), os.path.join(pkg, "csrc", "fastpack.c")]]
        for c in cmds:
            say("$ " + " ".join(c))
            subprocess.run(c, check=True)
        env = dict(os.environ,
                   LD_PRELOAD=":".join([runtime("libasan.so"), runtime("libubsan.so")]),
                   ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1:alloc_dealloc_mismatch=0:"
                                "new_delete_type_mismatch=0:detect_odr_violation=0",
                   UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
                   PYTHONDONTWRITEBYTECODE="1")
        # -s: a report printed inside a test reaches the log even when the sanitizer ends the process
        cmd = [sys.executable, "-m", "pytest", "-q", "-s", "-p", "no:cacheprovider", "-m", "not gpu", *TESTS]
        say(f"$ LD_PRELOAD={env['LD_PRELOAD']} ASAN_OPTIONS={env['ASAN_OPTIONS']} "
            f"UBSAN_OPTIONS={env['UBSAN_OPTIONS']} " + " ".join(cmd))
        t0 = time.time()
        p = subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True)
        out = p.stdout + p.stderr
        reports = [ln for ln in out.splitlines() if "ERROR: AddressSanitizer" in ln or "runtime error:" in ln]
        tail = "\n".join(out.strip().splitlines()[-15:])
        say(tail)
        say(f"exit status {p.returncode}; {len(reports)} sanitizer report(s); {time.time() - t0:.1f} s")
        for r in reports[:20]:
            say("REPORT: " + r)
        # the instrumentation is live: a gather that READS past a 10-byte source (the destination
        # window only bounds writes) must be caught by ASan in the same build and environment
        probe = ("import numpy as np; from fedn_amd import codec; s = np.zeros(10, np.uint8); d = np.zeros(4096, np.uint8);"
                 " codec.gather_raw([(d.ctypes.data, s.ctypes.data, 4096)], 1, (d.ctypes.data, 4096))")
        q = subprocess.run([sys.executable, "-c", probe], cwd=tmp, env=env, capture_output=True, text=True)
        caught = "ERROR: AddressSanitizer" in q.stderr
        say(f"self-check (an over-read planted on purpose): {'caught by ASan' if caught else 'NOT caught'}; "
            + next((ln.strip() for ln in q.stderr.splitlines() if "ERROR: AddressSanitizer" in ln), ""))
        if not caught:
            reports.append("self-check not caught: the sanitizer is not active")
    if a.out:
        with open(a.out, "w") as f:
            f.write("\n".join(log) + "\n")
    raise SystemExit(p.returncode or (1 if reports else 0))


if __name__ == "__main__":
    main()
