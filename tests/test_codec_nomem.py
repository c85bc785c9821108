"""No C++ exception crosses libfednpz's C ABI (fedn_amd/csrc/fnpz_guard.h): when memory or threads
run out inside a call, the call returns FNPZ_ENOMEM (raised as MemoryError) instead of
std::terminate aborting the process — for a combiner, the difference between one failed save or
load and a dead round. Each case runs in a child process whose address space is capped
(RLIMIT_AS) just above what it already maps, then checks that the library still works once the
cap is lifted."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import io, resource, sys
    import numpy as np
    sys.path.insert(0, {root!r})
    from fedn_amd import codec
    codec.load_lib()
    x = np.random.default_rng(0).standard_normal(12_000_000).astype(np.float32)   # 48 MB
    blob = codec.save_npz([x[:1_000_000]], threads=2)                               # warm: pools exist
    big = io.BytesIO(); np.savez_compressed(big, **{{"0": x}}); big = big.getvalue()
    out = np.empty_like(x)
    def vm():
        for line in open("/proc/self/status"):
            if line.startswith("VmSize:"):
                return int(line.split()[1]) * 1024
    soft, hard = resource.getrlimit(resource.RLIMIT_AS)
    resource.setrlimit(resource.RLIMIT_AS, (vm() + {room}, hard))
    try:
        {call}
        print("NO-ERROR")
    except MemoryError as e:
        print("MEMORYERROR", e)
    resource.setrlimit(resource.RLIMIT_AS, (soft, hard))
    back = codec.load_npz(codec.save_npz([x], threads=4))                           # still usable
    print("USABLE", bool(np.array_equal(back[0], x)))
""")

# (the call, room above the current mapping): room enough for the Python-side output buffer the
# call allocates first (numpy would raise its own MemoryError there), not for the native work
CALLS = {
    # the exact writer: the member copy / symbol buffers of the parallel deflate, its worker threads
    "save": ("codec.save_npz([x], threads=8)", 64 << 20),
    # the decoder: the parallel split's chunk buffers on the decode pool's workers
    "load": ("codec.load_npz(big)", 64 << 20),
}


@pytest.mark.parametrize("what", list(CALLS))
def test_out_of_memory_is_an_error_not_an_abort(what):
    call, room = CALLS[what]
    code = CHILD.format(root=ROOT, room=room, call=call)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "OMP_NUM_THREADS": "1"})
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])   # -6 would be std::terminate's abort
    assert "MEMORYERROR" in r.stdout and "fednpz status 6" in r.stdout, r.stdout
    assert "USABLE True" in r.stdout, r.stdout
