"""The C ABI headers are plain C: a C99 program includes both, links both libraries and
calls the version / error / validation entry points (no GPU work)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

C_PROG = r"""
#include <stdio.h>
#include "fedagg.h"
#include "fednpz.h"
int main(void) {
    fnpz_entry e;
    int n = 0;
    const unsigned char junk[32] = {0};
    if (fa_abi_version() != FA_ABI_VERSION) return 1;
    if (fnpz_abi_version() != FNPZ_ABI_VERSION) return 2;
    if (fa_promote(FA_F32, FA_F64) != FA_F64) return 3;
    if (fa_fedavg_fold(0, FA_F32, 0, FA_F32, 0, 0, 2, 10, 1, 0) != FA_EINVAL) return 4;
    if (fa_last_error()[0] == 0) return 5;
    if (fnpz_open(junk, sizeof junk, &e, 1, &n) != FNPZ_EFORMAT) return 6;
    {
        unsigned char dst[32] = {0};
        void* d = dst;
        const void* s = junk;
        int64_t nb = sizeof junk;
        if (fnpz_gather(1, &d, &s, &nb, 4, dst, sizeof dst) != FNPZ_OK || dst[0] != junk[0]) return 7;
        if (fnpz_gather(1, &d, &s, &nb, 0, dst, sizeof dst) != FNPZ_EINVAL) return 8;
        if (fnpz_gather(1, &d, &s, &nb, 4, dst, sizeof dst - 1) != FNPZ_ENOSPC) return 9;
        if (fnpz_gather_start(1, &d, &s, &nb, 4, dst + 1, sizeof dst) != -FNPZ_ENOSPC) return 10;
    }
    printf("ok %s\n", fnpz_last_error());
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_headers_are_c99_and_link(tmp_path):
    src = tmp_path / "abi.c"
    src.write_text(C_PROG)
    exe = tmp_path / "abi"
    lib = os.path.join(ROOT, "fedn_amd")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe),
                    "-L", lib, "-lfedagg", "-lfednpz", f"-Wl,-rpath,{lib}"], check=True)
    env = dict(os.environ, LD_LIBRARY_PATH=lib + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    assert r.stdout.startswith("ok")
