"""The C ABI library loads and exports every entry point include/fedagg.h declares (CPU-only:
no compute call is made; only argument-validation paths that return before touching a device)."""
import ctypes
import os
import re

import pytest

from fedn_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "fedagg.h")
PROBE_HEADER = os.path.join(ROOT, "include", "fedagg_probe.h")


def header_functions(path=HEADER):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fa_[a-z0-9_]+)\s*\(", src)))


def test_library_present_and_loads():
    assert os.path.exists(_abi.lib_path()), "build libfedagg.so first (__graft_entry__.build())"
    lib = _abi.load()
    assert lib.fa_abi_version() == _abi.ABI_VERSION


def test_exports_every_declared_symbol():
    names = header_functions()
    assert "fa_fedavg_fold" in names and "fa_fedopt_step" in names
    raw = ctypes.CDLL(_abi.lib_path())
    for n in names:
        assert hasattr(raw, n), f"libfedagg.so does not export {n}"
    assert set(names) == set(_abi.EXPORTS), "ctypes signature table out of sync with the header"
    for n in header_functions(PROBE_HEADER):
        assert not hasattr(raw, n), f"the product library exports the measurement entry point {n}"


def test_probe_library_exports_both_headers():
    """libfedagg_probe.so (tools/, A/B tests) = the product entry points + fedagg_probe.h."""
    raw = ctypes.CDLL(_abi.PROBE_PATH)
    probe = header_functions(PROBE_HEADER)
    assert "fa_tune" in probe and set(probe) == set(_abi.PROBE_EXPORTS)
    for n in header_functions() + probe:
        assert hasattr(raw, n), f"libfedagg_probe.so does not export {n}"
    assert _abi.load_probe().fa_abi_version() == _abi.ABI_VERSION


def test_promote_table():
    lib = _abi.load()
    P = lib.fa_promote
    assert P(_abi.FA_F32, _abi.FA_F32) == _abi.FA_F32
    assert P(_abi.FA_F32, _abi.FA_F64) == _abi.FA_F64
    assert P(_abi.FA_BF16, _abi.FA_F32) == _abi.FA_F32
    assert P(_abi.FA_NONE, _abi.FA_BF16) == _abi.FA_F32
    assert P(_abi.FA_F16, _abi.FA_F32) == _abi.FA_F32
    assert P(_abi.FA_I64, _abi.FA_F32) == _abi.FA_NONE


@pytest.mark.parametrize("call,code", [
    ("null_agg", _abi.FA_EINVAL),
    ("neg_P", _abi.FA_EINVAL),
    ("init_K0", _abi.FA_EINVAL),
])
def test_fedavg_argument_errors(call, code):
    lib = _abi.load()
    ptrs = _abi.ptr_array([16, 32])
    n = _abi.double_array([1, 2])
    N = _abi.double_array([1, 3])
    if call == "null_agg":
        rc = lib.fa_fedavg_fold(None, 0, ptrs, 0, n, N, 2, 10, 1, None)
    elif call == "neg_P":
        rc = lib.fa_fedavg_fold(16, 0, ptrs, 0, n, N, 2, -1, 1, None)
    else:
        rc = lib.fa_fedavg_fold(16, 0, ptrs, 0, n, N, 0, 10, 1, None)
    assert rc == code
    assert lib.fa_last_error().decode()
    with pytest.raises(_abi.FedAggError):
        _abi.check(rc)


def test_noop_calls_return_ok():
    lib = _abi.load()
    ptrs = _abi.ptr_array([16])
    n = _abi.double_array([1])
    assert lib.fa_fedavg_fold(16, 0, ptrs, 0, n, n, 0, 10, 0, None) == _abi.FA_OK   # K = 0, continue
    assert lib.fa_fedavg_fold(16, 0, ptrs, 0, n, n, 1, 0, 0, None) == _abi.FA_OK    # P = 0


def test_fedopt_argument_errors():
    lib = _abi.load()
    ptrs = _abi.ptr_array([16])
    n = _abi.double_array([1])
    args = dict(old=16, od=0, ups=ptrs, ud=0, n=n, N=n, K=1, pg=0, flags=3, m=0, md=-1, mo=32, vi=0, vo=48, out=64,
                opt=0, P=10)

    def call(**kw):
        a = {**args, **kw}
        return lib.fa_fedopt_step(a["old"], a["od"], a["ups"], a["ud"], a["n"], a["N"], a["K"], a["pg"], a["flags"],
                                  a["m"], a["md"], a["mo"], a["vi"], a["vo"], a["out"], a["opt"], 1e-3, 0.9, 0.99,
                                  1e-4, a["P"], None)
    assert call(old=0) == _abi.FA_EINVAL
    assert call(opt=7) == _abi.FA_EINVAL
    assert call(od=_abi.FA_I64) == _abi.FA_EDTYPE
    assert call(flags=2, K=0) == _abi.FA_EINVAL        # continue without a pg workspace
    assert call(flags=1, K=0) == _abi.FA_EINVAL        # FIRST needs an update
    assert call(P=0) == _abi.FA_OK
