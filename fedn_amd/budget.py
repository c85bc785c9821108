"""HBM admission control for updates staged on arrival (ingest.StagingUpdateHandler).

FEDn folds any number of host-resident updates one at a time (fedavg.py:47-68, fedopt.py:74-98):
its memory use is one update plus the model. Staging every update into HBM on arrival is faster
but bounded by HBM (288 GB per MI355X: a 1 B-param fp32 model with 64 clients is 256 GB). So each
staging reserves its bytes from a per-device budget first; an update the budget cannot hold is
NOT staged — it stays host-side (its raw bytes in FEDn's model storage) and the aggregator loads
and folds it through the host path at its place in the FIFO, exactly as FEDn would. A round never
runs out of HBM and never drops a client. A staged update returns its bytes to the budget when
the last reference to it goes (the pipeline folded it, or the round ended).

Budget per device: ``FEDN_AMD_HBM_BUDGET`` (bytes; suffixes K / M / G / T, powers of 1024) or
``FEDN_AMD_HBM_FRACTION`` (default 0.75) of the device memory free when the budget first sees the
device — the rest is left for the pipelines' own buffers (the running model, FedOpt's state,
staging slots).
"""
import os
import threading
import weakref

import torch

DEFAULT_FRACTION = 0.75
_UNITS = {"": 1, "K": 1 << 10, "M": 1 << 20, "G": 1 << 30, "T": 1 << 40}


def parse_bytes(text):
    """'12G' -> 12 * 2**30; plain integers are bytes."""
    t = str(text).strip().upper().rstrip("B").rstrip("I")
    unit = t[-1] if t and t[-1] in _UNITS else ""
    num = t[:-1] if unit else t
    try:
        val = float(num) * _UNITS[unit]
    except ValueError:
        raise ValueError(f"cannot read a byte count from {text!r}") from None
    if val < 0:
        raise ValueError(f"negative byte budget {text!r}")
    return int(val)


class HbmBudget:
    """Bytes of staged updates allowed per device; thread-safe (staging workers reserve, the
    round thread's garbage collection releases)."""

    def __init__(self, limit=None, fraction=None):
        env = os.environ.get("FEDN_AMD_HBM_BUDGET")
        self.limit = limit if limit is not None else (parse_bytes(env) if env else None)
        self.fraction = fraction if fraction is not None else float(
            os.environ.get("FEDN_AMD_HBM_FRACTION", DEFAULT_FRACTION))
        self._cap = {}
        self._used = {}
        # re-entrant: a staged update's finalizer (``hold``) may run — and release — while this thread
        # is inside reserve() (garbage collection runs at any allocation)
        self._lock = threading.RLock()
        self.refused = 0              # stagings turned away (reported by the ingest)

    def _capacity(self, key, device):
        cap = self._cap.get(key)
        if cap is None:
            if self.limit is not None:
                cap = self.limit
            else:
                free, _ = torch.cuda.mem_get_info(device)
                cap = int(free * self.fraction)
            self._cap[key] = cap
        return cap

    def reserve(self, parts):
        """``parts`` = [(device, nbytes)]: reserve all or nothing; True if granted."""
        with self._lock:
            keys = [(str(torch.device(d)), d, n) for d, n in parts]
            for key, dev, n in keys:
                if self._used.get(key, 0) + n > self._capacity(key, dev):
                    self.refused += 1
                    return False
            for key, _, n in keys:
                self._used[key] = self._used.get(key, 0) + n
            return True

    def release(self, parts):
        with self._lock:
            for d, n in parts:
                key = str(torch.device(d))
                self._used[key] = max(0, self._used.get(key, 0) - n)

    def hold(self, obj, parts):
        """Return the reservation ``parts`` when ``obj`` (a staged update) is garbage collected."""
        fin = weakref.finalize(obj, self.release, list(parts))
        try:
            obj.budget_fin = fin      # so that take() can move the reservation to what replaces obj
        except AttributeError:
            pass
        return obj

    def take(self, obj):
        """Move the reservation ``hold`` attached to ``obj`` to the caller (who must ``release`` or
        ``hold`` it): the parts, or [] if there is none. An update decoded into HBM during its upload
        hands its reservation to its staged copy this way, instead of both counting against the
        budget."""
        fin = getattr(obj, "budget_fin", None)
        if fin is None:
            return []
        det = fin.detach()
        obj.budget_fin = None
        return list(det[2][0]) if det is not None else []

    def used(self, device):
        with self._lock:
            return self._used.get(str(torch.device(device)), 0)
