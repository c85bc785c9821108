"""FEDN_AMD_POISON_REUSE=1: make a cross-stream reuse bug corrupt the round instead of hiding.

The hazard (the multi-device race fixed in round 5): a device buffer written on one
stream (a staging stream's H2D) is read by a launch enqueued on another (a pipeline's compute stream);
if its last Python reference is dropped while that launch has not run yet, torch's caching allocator
hands the block to the next allocation on the WRITER's stream at once, and a new H2D can overwrite it
before the read. Whether that corrupts a round is a matter of timing, so a test can pass by luck.

With the knob on, every buffer registered with :func:`watch` (the staging allocations of ingest.py,
upload.py, staging.py, multidev.py, mixed.py) is watched: the moment its storage is freed (the tensor
and every view of it dropped), a poison
thread allocates blocks of the same size on the same stream until the allocator hands it that very
block (or 0.3 ms pass) and fills it with 0xFF bytes — a NaN in every float dtype — on that stream. A
buffer still read by an enqueued launch and not protected (held until the reader ran, or
``record_stream``'d) is then overwritten right away, and the round's result is wrong; a protected one
is either not handed out until its reader finished (the poison lands after the read: harmless) or not
at all. ``stats()`` counts buffers watched, poisoned and never handed back. Off: ``watch`` is a no-op.
"""
import os
import queue
import threading
import time
import weakref

import torch

ENABLED = os.environ.get("FEDN_AMD_POISON_REUSE", "") == "1"
RETRY_S = 300e-6   # an unprotected block comes back at once; a protected one is safe whenever it does
# FEDN_AMD_POISON_HOLD=1: keep every same-size block the allocator offers first until the freed one comes
# back (more of them are reached; the default returns them every 8 tries), at most HOLD_BYTES
HOLD = os.environ.get("FEDN_AMD_POISON_HOLD", "") == "1"
HOLD_BYTES = 8 << 30

_q = queue.Queue()
_stats = {"watched": 0, "poisoned": 0, "not_reissued": 0, "poisoned_bytes": 0, "freed_bytes": 0}
_lock = threading.Lock()
_thread = None


def enabled():
    return ENABLED


def set_enabled(on):
    """Turn the knob on or off in this process (tests; the environment variable sets it at import)."""
    global ENABLED
    ENABLED = bool(on)


def watch(t, stream=None):
    """Register device tensor ``t``, allocated on ``stream`` (None: the device's current stream), for
    poisoning once it is freed; returns ``t``."""
    if not ENABLED or t is None or not t.is_cuda or t.numel() == 0:
        return t
    global _thread
    stream = stream if stream is not None else torch.cuda.current_stream(t.device)
    st = t.untyped_storage()           # its PyObject lives as long as the storage: views keep it too
    weakref.finalize(st, _q.put, (st.data_ptr(), st.nbytes(), t.device, stream))
    with _lock:
        _stats["watched"] += 1
        if _thread is None:
            _thread = threading.Thread(target=_poisoner, name="fedn_amd_poison", daemon=True)
            _thread.start()
    return t


def _poisoner():
    while True:
        ptr, nbytes, device, stream = _q.get()
        try:
            _poison(ptr, nbytes, device, stream)
        finally:
            _q.task_done()


def _poison(ptr, nbytes, device, stream):
    held = []                            # same-size blocks the allocator offered first (kept until done)
    deadline = time.perf_counter() + RETRY_S
    with torch.cuda.device(device), torch.cuda.stream(stream):
        while True:
            b = torch.empty(nbytes, dtype=torch.uint8, device=device)
            # the allocator may hand the block back merged with a free neighbour (a block split at
            # another offset): whatever part of the freed range it returns is poisoned
            lo, hi = max(ptr, b.data_ptr()), min(ptr + nbytes, b.data_ptr() + nbytes)
            if lo < hi:
                b[lo - b.data_ptr():hi - b.data_ptr()].fill_(0xFF)   # on the writer's stream, as its next H2D
                with _lock:
                    _stats["poisoned"] += 1
                    _stats["poisoned_bytes"] += hi - lo
                    _stats["freed_bytes"] += nbytes
                return
            held.append(b)
            if len(held) >= 64 or (HOLD and len(held) * nbytes > HOLD_BYTES) or time.perf_counter() > deadline:
                with _lock:
                    _stats["not_reissued"] += 1
                    _stats["freed_bytes"] += nbytes
                return
            if len(held) % 8 == 0:
                if not HOLD:
                    held.clear()         # give the block time to come back (its free may still run)
                time.sleep(20e-6)


def drain():
    """Wait until every freed watched buffer has been handled (tests call it before reading stats)."""
    if ENABLED:
        _q.join()


def stats():
    with _lock:
        return dict(_stats)
