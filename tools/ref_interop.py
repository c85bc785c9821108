"""The plug-ins' read-ahead drain (``aggregatorbase.queued_updates``) against FEDn's REAL
UpdateHandler, ModelService and TempModelStorage — build container only (it imports
/root/reference the way tools/gen_golden.py does; nothing here runs on the GPU box, and the
fold itself is not involved: this checks the host-side queue semantics).

For each case two identical sessions receive the same uploads through the reference's
``ModelService.set_model`` + ``UpdateHandler.on_model_update``: one is drained by FEDn's own
sequential loop (fedavg.py:47-78: ``next_model_update`` then ``load_model_update``), the other by
``queued_updates`` with up to 8 concurrent ``load_model_update`` calls. Checked:
  * same updates, same FIFO order, bit-identical decoded arrays and metadata;
  * a byte cap that limits the window to 2 decoded updates;
  * an early stop (generator closed after j updates) leaves the queue exactly as FEDn's loop
    would have left it after j updates (same qsize, same update ids in the same order);
  * a BaseException out of one load leaves the queue as FEDn's loop does when that load raises.

Run:  python tools/ref_interop.py   (prints one JSON line per case; exit 1 on any mismatch)
"""
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd.aggregators.aggregatorbase import queued_updates  # noqa: E402
from tools.gen_golden import MNIST_SHAPES, Harness, _import_reference, _perturb, _rng_model  # noqa: E402


class Stop(BaseException):
    pass


def session(ref, K, seed):
    rng = np.random.default_rng(seed)
    h = Harness(ref, "fedavg")
    base = _rng_model(rng, MNIST_SHAPES, np.float32)
    h.put_model(base, "global-0")
    for _ in range(K):
        h.push_update(_perturb(rng, base, np.float32), int(rng.integers(1, 5001)), "global-0")
    return h


def sequential(h, upto=None, raise_at=None):
    """FEDn's loop (fedavg.py:47-78) up to ``upto`` updates; a BaseException at ``raise_at``."""
    out = []
    uh = h.uh
    while not uh.model_updates.empty():
        if upto is not None and len(out) == upto:
            break
        mu = uh.next_model_update()
        if raise_at is not None and len(out) == raise_at:
            break                                   # the load raised: mu is consumed, the rest stays
        arrays, meta = uh.load_model_update(mu, h.helper)
        out.append((mu.model_update_id, arrays, meta))
    return out


def read_ahead(h, upto=None, raise_at=None, **kw):
    out = []
    uh = h.uh
    real0 = uh.load_model_update
    live = [0, 0]                                   # loads in flight now, most at once
    lock = threading.Lock()

    def counted(mu, helper):
        with lock:
            live[0] += 1
            live[1] = max(live[1], live[0])
        try:
            time.sleep(0.01)                        # a decode that takes a while, as a 100 M-param one does
            return real0(mu, helper)
        finally:
            with lock:
                live[0] -= 1
    uh.load_model_update = counted
    if raise_at is not None:
        real = uh.load_model_update
        ids = []

        def load(mu, helper):
            ids.append(mu.model_update_id)
            if len(ids) == raise_at + 1:
                raise Stop()
            return real(mu, helper)
        uh.load_model_update = load
    gen = queued_updates(uh, h.helper, **kw)
    try:
        for mu, load in gen:
            arrays, meta = load()
            out.append((mu.model_update_id, arrays, meta))
            if upto is not None and len(out) == upto:
                break                               # the caller stops before taking the next update
    except Stop:
        pass
    finally:
        gen.close()
    h.max_concurrent_loads = live[1]
    return out


def remaining_ids(h):
    return [mu.model_update_id for mu in list(h.uh.model_updates.queue)]


def same(a, b):
    if len(a) != len(b):
        return False
    for (ia, xa, ma), (ib, xb, mb) in zip(a, b):
        if ma != mb or len(xa) != len(xb):
            return False
        if not all(np.asarray(p).dtype == np.asarray(q).dtype and np.array_equal(np.asarray(p).view(np.uint8),
                                                                                  np.asarray(q).view(np.uint8))
                   for p, q in zip(xa, xb)):
            return False
    return True


def main():
    ref = _import_reference()
    ok = True
    K = 24
    cases = [("full_drain_ahead8", {}, dict(ahead=8)),
             ("full_drain_byte_cap_2", {}, dict(ahead=8, ahead_bytes=2 * 4 * sum(int(np.prod(s)) for s in MNIST_SHAPES))),
             ("stop_after_5", dict(upto=5), dict(ahead=8)),
             ("base_exception_at_7", dict(raise_at=7), dict(ahead=8))]
    for i, (name, stop, kw) in enumerate(cases):
        a, b = session(ref, K, 100 + i), session(ref, K, 100 + i)
        # the two sessions hold different uuids; compare by position in the upload order
        order_a = remaining_ids(a)
        order_b = remaining_ids(b)
        seq = sequential(a, **stop)
        ra = read_ahead(b, **{**stop, **kw})
        pos_a = {u: j for j, u in enumerate(order_a)}
        pos_b = {u: j for j, u in enumerate(order_b)}
        seq_n = [(pos_a[u], x, m) for u, x, m in seq]
        ra_n = [(pos_b[u], x, m) for u, x, m in ra]
        rest_a = [pos_a[u] for u in remaining_ids(a)]
        rest_b = [pos_b[u] for u in remaining_ids(b)]
        good = same(seq_n, ra_n) and rest_a == rest_b and a.uh.model_updates.qsize() == b.uh.model_updates.qsize()
        ok &= good
        print(json.dumps({"case": name, "uploads": K, "folded_in_order": [p for p, _, _ in ra_n],
                          "left_queued": rest_b, "fedn_left_queued": rest_a, "arrays_bit_identical": same(seq_n, ra_n),
                          "max_concurrent_load_model_update": b.max_concurrent_loads,
                          "ok": good}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
