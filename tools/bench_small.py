"""Round latency of the plug-ins for SMALL models (BASELINE configs[0]'s mnist-pytorch shapes and a
mid-size CNN), host-resident numpy updates through the real combine_models call — the regime most
FEDn deployments run in, where FEDn's numpy loop is already fast and the GPU path must not add
latency. Beside it, two CPU columns on one host core: the numpy restatement's arithmetic alone
(oracle/, bit-equal to FEDn: ``round_ms_numpy_oracle_1core``), and the same arithmetic inside
FEDn's own combine_models loop restated (fedavg.py:45-83, fedopt.py:74-121: queue, load,
bookkeeping and per-update log calls) over the same in-memory update handler as the plug-in
(``round_ms_numpy_fedn_loop``) — what the reference aggregator itself takes for the round. Every GPU
round is checked bit-identical to the oracle.

Run on the GPU box:  python tools/bench_small.py
"""
import json
import logging
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi  # noqa: E402
from fedn_amd.aggregators import get_aggregator  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402
from oracle import numpy_ref as ref  # noqa: E402  (the checker and the CPU baseline only)

MNIST = [(64, 784), (64,), (32, 64), (32,), (10, 32), (10,)]          # examples/mnist-pytorch model.py:18-32
CNN = [(64, 3, 3, 3), (64,), (128, 64, 3, 3), (128,), (256, 128, 3, 3), (256,), (512, 256, 3, 3), (512,),
       (4096, 512), (4096,), (10, 4096), (10,)]                        # ~3.7 M params, 12 tensors
ref_logger = logging.getLogger("fedn")     # the plug-ins log to the same logger, at the same level
PARAMS = {"serveropt": "adam", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}


def models(rng, shapes, K):
    base = [rng.standard_normal(s).astype(np.float32) for s in shapes]
    ups = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    return base, ups, ns


def same(a, b):
    return len(a) == len(b) and all(x.dtype == y.dtype and np.array_equal(x.view(np.uint8), y.view(np.uint8))
                                    for x, y in zip(a, b))


def fedn_loop_fedavg(uh, helper=None, delete_models=True):
    """fedavg.py:45-83 restated with the oracle's arithmetic (the reference's per-update log calls
    included: their messages are formatted whatever the level)."""
    log = ref_logger
    name = "fedavg"
    data = {"time_model_load": 0.0, "time_model_aggregation": 0.0}
    model, nr, total = None, 0, 0
    log.info("AGGREGATOR({}): Aggregating model updates... ".format(name))
    while not uh.model_updates.empty():
        try:
            log.info("AGGREGATOR({}): Getting next model update from queue.".format(name))
            mu = uh.next_model_update()
            log.info("AGGREGATOR({}): Loading model metadata {}.".format(name, mu.model_update_id))
            tic = time.time()
            model_next, metadata = uh.load_model_update(mu, helper)
            data["time_model_load"] += time.time() - tic
            log.info("AGGREGATOR({}): Processing model update {}, metadata: {}  ".format(name, mu.model_update_id,
                                                                                         metadata))
            total += metadata["num_examples"]
            tic = time.time()
            model = model_next if nr == 0 else ref.increment_average(model, model_next, metadata["num_examples"], total)
            data["time_model_aggregation"] += time.time() - tic
            nr += 1
            if delete_models:
                uh.delete_model(mu)
        except Exception as e:  # noqa: BLE001
            log.error(f"AGGREGATOR({name}): Error encoutered while processing model update: {e}")
    data["nr_aggregated_models"] = nr
    return model, data


def fedn_loop_fedopt(uh, st, params, helper=None, delete_models=True):
    """fedopt.py:75-121 restated with the oracle's arithmetic (validation, loop, server step)."""
    log = ref_logger
    name = "fedopt"
    data = {"time_model_load": 0.0, "time_model_aggregation": 0.0, "nr_aggregated_models": 0}
    p = ref.validate_parameters(params)
    log.info(f"Aggregator {name} starting model aggregation.")
    pg, old, nr, total = None, None, 0, 0
    while not uh.model_updates.empty():
        try:
            log.info(f"Aggregator {name}: Fetching next model update.")
            mu = uh.next_model_update()
            tic = time.time()
            model_next, metadata = uh.load_model_update(mu, helper)
            data["time_model_load"] += time.time() - tic
            log.info(f"Processing model update {mu.model_update_id}")
            total += metadata["num_examples"]
            tic = time.time()
            if nr == 0:
                old = uh.load_model(helper, mu.model_id)
                pg = ref.subtract(model_next, old)
            else:
                pg = ref.increment_average(pg, ref.subtract(model_next, old), metadata["num_examples"], total)
            data["time_model_aggregation"] += time.time() - tic
            nr += 1
            if delete_models:
                uh.delete_model(mu)
                log.info(f"Deleted model update {mu.model_update_id} from storage.")
        except Exception as e:  # noqa: BLE001
            log.error(f"Error processing model update: {e}. Skipping this update.")
    data["nr_aggregated_models"] = nr
    model = ref._server_step(st, pg, old, p)
    log.info(f"Aggregator {name} completed. Aggregated {nr} models.")
    return model, data


def run(kind, shapes, K, rounds=20, warm=3):
    """Each path runs its warm + timed rounds back to back (the oracle's arithmetic, then the GPU
    plug-in, then FEDn's loop restated), so no path's rounds are interleaved with another path's
    work. Every round of the two other paths is checked against the oracle's model of the same round
    right after it (outside the timing), and a round's model is dropped once checked — as FEDn drops
    it after serialising it — so the plug-in's pinned result blocks are reused from round to round."""
    rng = np.random.default_rng(K)
    base, ups, ns = models(rng, shapes, K)
    params = PARAMS if kind == "fedopt" else None

    st, old = ref.FedOptState(), base
    cpu, want = [], []
    for r in range(warm + rounds):
        t1 = time.perf_counter()
        if kind == "fedavg":
            w, _ = ref.fedavg_combine(list(zip(ups, ns)))
        else:
            w, _ = ref.fedopt_combine(st, list(zip(ups, ns)), old, PARAMS)
            old = w
        cpu.append(time.perf_counter() - t1)
        want.append(w)

    uh = MemoryUpdateHandler()
    agg = get_aggregator(kind, uh)
    gid = uh.put_global_model(base, "g0")
    times, ok = [], True
    for r in range(warm + rounds):
        for a, n in zip(ups, ns):
            uh.submit(a, n, model_id=gid)
        t0 = time.perf_counter()
        model, _ = agg.combine_models(helper=None, delete_models=True, parameters=params)
        times.append(time.perf_counter() - t0)
        ok &= same(model, want[r])
        if kind == "fedopt":                     # the next round starts from the new global model
            gid = uh.put_global_model(model, f"g{r + 1}")
        del model

    uh_loop, st_loop = MemoryUpdateHandler(), ref.FedOptState()
    gid_loop = uh_loop.put_global_model(base, "g0")
    loop = []
    for r in range(warm + rounds):
        for a, n in zip(ups, ns):
            uh_loop.submit(a, n, model_id=gid_loop)
        t2 = time.perf_counter()
        if kind == "fedavg":
            got_loop, _ = fedn_loop_fedavg(uh_loop)
        else:
            got_loop, _ = fedn_loop_fedopt(uh_loop, st_loop, PARAMS)
            gid_loop = uh_loop.put_global_model(got_loop, f"g{r + 1}")
        loop.append(time.perf_counter() - t2)
        ok &= same(got_loop, want[r])

    P = sum(int(np.prod(s)) for s in shapes)
    med = lambda xs: float(np.median(xs[warm:])) * 1e3  # noqa: E731
    gpu_ms, cpu_ms, loop_ms = med(times), med(cpu), med(loop)
    return {"aggregator": kind, "params": P, "tensors": len(shapes), "clients": K,
            "round_ms_gpu_plugin": gpu_ms, "round_ms_numpy_oracle_1core": cpu_ms, "speedup": cpu_ms / gpu_ms,
            "round_ms_numpy_fedn_loop": loop_ms, "speedup_vs_fedn_loop": loop_ms / gpu_ms,
            "bit_exact_all_rounds": bool(ok), "rounds": rounds}


def main():
    _abi.load()
    for kind in ("fedavg", "fedopt"):
        for shapes, K in ((MNIST, 2), (MNIST, 10), (MNIST, 64), (CNN, 10), (CNN, 64)):
            print(json.dumps(run(kind, shapes, K)), flush=True)


if __name__ == "__main__":
    main()
