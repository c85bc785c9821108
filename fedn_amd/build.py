"""Build libfedagg.so (gfx950) in-tree with hipcc. ``python -m fedn_amd.build [--force]``."""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "fedagg.hip")
HDR = os.path.join(ROOT, "include", "fedagg.h")
OUT = os.path.join(HERE, "libfedagg.so")
PROBE_HDR = os.path.join(ROOT, "include", "fedagg_probe.h")
PROBE_OUT = os.path.join(HERE, "libfedagg_probe.so")   # + measurement knobs / probe kernels (tools/)
ARCH = os.environ.get("FEDN_AMD_ARCH", "gfx950")

# -ffp-contract=off: numpy never fuses a*b+c, so neither may we (bit-exact parity).
# hipcc's defaults keep f32 denormals and correctly rounded f32/f64 division and sqrt.
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", "-Wall", f"--offload-arch={ARCH}"]


def hipcc():
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found")


NPZ_SRC = os.path.join(HERE, "csrc", "npz_codec.cpp")
NPZ_HDR = os.path.join(ROOT, "include", "fednpz.h")
NPZ_INFLATE = os.path.join(HERE, "csrc", "inflate.h")      # the codec's DEFLATE decoder + CRC-32
NPZ_SAVEZ = os.path.join(HERE, "csrc", "savez.cpp")        # numpy-identical writer (fnpz_savez)
NPZ_PDEFLATE = os.path.join(HERE, "csrc", "pdeflate.h")    # its single-stream parallel deflate
NPZ_GUARD = os.path.join(HERE, "csrc", "fnpz_guard.h")      # no exception across the C ABI
NPZ_OUT = os.path.join(HERE, "libfednpz.so")


def _stale(out, *deps):
    return not os.path.exists(out) or any(os.path.getmtime(out) < os.path.getmtime(d) for d in deps)


def build_codec(force=False, verbose=True):
    """Host-side npz codec (C++17 + zlib, no GPU code)."""
    deps = [d for d in (NPZ_SRC, NPZ_HDR, NPZ_INFLATE, NPZ_SAVEZ, NPZ_PDEFLATE, NPZ_GUARD) if os.path.exists(d)]
    if not force and not _stale(NPZ_OUT, *deps):
        return NPZ_OUT
    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    tmp = NPZ_OUT + ".tmp"
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", "-I", os.path.join(ROOT, "include"),
           "-o", tmp, NPZ_SRC, NPZ_SAVEZ, "-lz"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, NPZ_OUT)
    return NPZ_OUT


FASTPACK_SRC = os.path.join(HERE, "csrc", "fastpack.c")
FASTPACK_OUT = os.path.join(HERE, "_fastpack.so")       # CPython extension: ``fedn_amd._fastpack``


def build_fastpack(force=False, verbose=True):
    """The small-update admission + pack extension (C, CPython and numpy C API; no GPU code)."""
    if not force and not _stale(FASTPACK_OUT, FASTPACK_SRC):
        return FASTPACK_OUT
    import sysconfig

    import numpy
    cc = os.environ.get("CC") or shutil.which("gcc") or "gcc"
    tmp = FASTPACK_OUT + ".tmp"
    cmd = [cc, "-O2", "-fPIC", "-shared", "-Wall", "-I", sysconfig.get_paths()["include"], "-I", numpy.get_include(),
           "-o", tmp, FASTPACK_SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, FASTPACK_OUT)
    return FASTPACK_OUT


def build(force=False, verbose=True):
    """Product library, probe library, codec and the pack extension; the two hipcc builds run
    concurrently."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(4) as ex:
        futs = [ex.submit(build_codec, force, verbose), ex.submit(build_hip, force, verbose),
                ex.submit(build_hip, force, verbose, True), ex.submit(build_fastpack, force, verbose)]
        for f in futs:
            f.result()
    return OUT


def build_hip(force=False, verbose=True, probe=False):
    out = PROBE_OUT if probe else OUT
    deps = (SRC, HDR, PROBE_HDR)
    if not force and not _stale(out, *deps):
        return out
    tmp = out + ".tmp"
    cmd = [hipcc()] + FLAGS + (["-DFEDAGG_PROBES"] if probe else []) + ["-I", os.path.join(ROOT, "include"),
                                                                          "-o", tmp, SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv), NPZ_OUT)
