"""Stress of the FedOpt one-call round's state hand-over (smallround.SmallFedOptRound): many short
sessions of the plug-in on small float32 / float64 models, each round's m and v read back at once
(``agg.m`` / ``agg.v``: torch D2H copies on the default stream of the HBM buffers the one-call step
wrote on the session's own stream) and compared bit for bit with the oracle; prints the count of
rounds whose model, m or v differ. Run on the GPU box: python tools/fedopt_small_stress.py
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd.aggregators import fedopt, fedopt_f32state  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402
from oracle import numpy_ref as ref  # noqa: E402  (the checker only)


def same(a, b):
    return len(a) == len(b) and all(x.dtype == y.dtype and x.shape == y.shape and
                                    np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(a, b))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sessions", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    rng = np.random.default_rng(7)
    bad = {"model": 0, "m": 0, "v": 0}
    rounds = 0
    t0 = time.time()
    for s in range(a.sessions):
        f32 = s % 2 == 0
        shapes = [(40, 30), (30,), (7,)] if s % 3 else [(64, 784), (64,), (10, 64), (10,)]
        opt = ("adam", "yogi", "adagrad")[s % 3]
        params = {"serveropt": opt, "learning_rate": 1e-2}
        uh = MemoryUpdateHandler()
        agg = (fedopt_f32state.Aggregator if f32 else fedopt.Aggregator)(uh, device="cuda:0")
        st = ref.FedOptState()
        old = [rng.standard_normal(sh).astype(np.float32) for sh in shapes]
        for r in range(a.rounds):
            K = int(rng.integers(1, 6))
            ups = [([(w + 0.01 * rng.standard_normal(w.shape)).astype(np.float32) for w in old], int(n))
                   for n in rng.integers(1, 5001, K)]
            gid = uh.put_global_model(old, f"g{r}")
            for arrays, n in ups:
                uh.submit(arrays, n, model_id=gid)
            model, _ = agg.combine_models(helper=None, parameters=params)
            m_now, v_now = agg.m, agg.v                 # read back at once
            combine = ref.fedopt_combine_f32state if f32 else ref.fedopt_combine
            want, _ = combine(st, ups, old, params)
            bad["model"] += not same(model, want)
            bad["m"] += not same(m_now, st.m)
            bad["v"] += not same(v_now, st.v)
            rounds += 1
            old = model
        if s % 50 == 0:
            print(json.dumps({"sessions": s + 1, "rounds": rounds, "bad": bad, "s": round(time.time() - t0, 1)}), flush=True)
    print(json.dumps({"sessions": a.sessions, "rounds": rounds, "bad": bad, "s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
