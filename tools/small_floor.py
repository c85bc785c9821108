"""configs[0]'s K = 2 round against its floor: the mnist-pytorch model (52,650
params, 6 tensors), two host numpy updates, FedAvg through the plug-in's combine_models — next to
what the round cannot go below on this box:

  sync_idle        hipStreamSynchronize on an idle stream
  launch_sync      one 1-element zero-copy fold launch + synchronize (the GPU round trip)
  fold_zero_copy   the round's own launch: the 3-client fold of 52,650 fp32 params reading the pinned
                   arena and writing the pinned result over PCIe, + synchronize
  pack_k2          the two updates' copies into the pinned arena (native gather) + wait
  plugin           the whole combine_models round (median)
  fedn_loop        FEDn's own loop restated around the numpy arithmetic (tools/bench_small.py)
  fedn_loop_no_arith  the same loop with increment_average made the identity: the queue / load /
                   log / delete share every aggregator pays; budget = fedn_loop - this is what a
                   plug-in has for its arithmetic, against gpu_floor = pack_k2 + the K = 2 fold

and a cProfile of the plug-in's host work. Run on the GPU box: python tools/small_floor.py
"""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedn_amd import _abi, ops  # noqa: E402
from fedn_amd.aggregators import get_aggregator  # noqa: E402
from fedn_amd.updatehandler import MemoryUpdateHandler  # noqa: E402
from oracle import numpy_ref as ref  # noqa: E402  (the checker only)

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench_small  # noqa: E402

MNIST = bench_small.MNIST


def med(f, n=400, warm=20):
    for _ in range(warm):
        f()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 2), round(ts[len(ts) // 10] * 1e6, 2)


def main():
    _abi.load()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.current_stream(dev)
    out = {}
    out["sync_idle_us"] = med(lambda: st.synchronize())
    one = torch.ones(64, dtype=torch.float32, pin_memory=True)
    res = torch.empty(64, dtype=torch.float32, pin_memory=True)
    p_one = ops.host_device_ptr(one.data_ptr(), dev)
    p_res = ops.host_device_ptr(res.data_ptr(), dev)

    def launch1():
        ops.fedavg_fold_raw(p_res, torch.float32, 1, [p_one, p_one], torch.float32, [0.0, 1.0], [1.0, 2.0], True, st, dev)
        st.synchronize()
    out["launch_sync_us"] = med(launch1)
    ev = torch.cuda.Event()

    def launch1_spin():
        ops.fedavg_fold_raw(p_res, torch.float32, 1, [p_one, p_one], torch.float32, [0.0, 1.0], [1.0, 2.0], True, st, dev)
        ev.record(st)
        while not ev.query():
            pass
    out["launch_spin_us"] = med(launch1_spin)
    rng = np.random.default_rng(0)
    P = sum(int(np.prod(s)) for s in MNIST)
    arena = torch.empty(3 * P, dtype=torch.float32, pin_memory=True)
    arena.copy_(torch.from_numpy(rng.standard_normal(3 * P).astype(np.float32)))
    out_h = torch.empty(P, dtype=torch.float32, pin_memory=True)
    pa = ops.host_device_ptr(arena.data_ptr(), dev)
    po = ops.host_device_ptr(out_h.data_ptr(), dev)

    def fold3():
        ops.fedavg_fold_raw(po, torch.float32, P, [pa, pa + 4 * P, pa + 8 * P], torch.float32, [0.0, 7.0, 9.0],
                            [1.0, 7.0, 16.0], True, st, dev)
        st.synchronize()
    out["fold_zero_copy_us"] = med(fold3)

    def fold3_spin():
        ops.fedavg_fold_raw(po, torch.float32, P, [pa, pa + 4 * P, pa + 8 * P], torch.float32, [0.0, 7.0, 9.0],
                            [1.0, 7.0, 16.0], True, st, dev)
        ev.record(st)
        while not ev.query():
            pass
    out["fold_zero_copy_spin_us"] = med(fold3_spin)

    def fold2_spin():          # K = 2 needs only the two updates: x1 + n2 (x2 - x1) / N
        ops.fedavg_fold_raw(po, torch.float32, P, [pa + 4 * P, pa + 8 * P], torch.float32, [7.0, 9.0],
                            [7.0, 16.0], True, st, dev)
        ev.record(st)
        while not ev.query():
            pass
    out["fold2_zero_copy_spin_us"] = med(fold2_spin)
    from fedn_amd import codec
    ups = [rng.standard_normal(P).astype(np.float32) for _ in range(2)]
    dst = arena.numpy()

    def pack2():
        t = None
        for k, u in enumerate(ups):
            t = codec.gather_start_raw([dst.ctypes.data + (k + 1) * 4 * P], [u.ctypes.data], [4 * P], 8,
                                       (dst.ctypes.data, dst.nbytes))
        codec.gather_wait(t)
    out["pack_k2_us"] = med(pack2)

    base = [rng.standard_normal(s).astype(np.float32) for s in MNIST]
    cl = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(2)]
    ns = [int(v) for v in rng.integers(1, 5001, 2)]
    uh = MemoryUpdateHandler()
    agg = get_aggregator("fedavg", uh)
    box = {}

    def plugin():
        for u, n in zip(cl, ns):
            uh.submit(u, n)
        box["m"], _ = agg.combine_models(helper=None)
    out["plugin_us"] = med(plugin, n=400)
    want, _ = ref.fedavg_combine(list(zip(cl, ns)))
    out["plugin_bit_exact"] = bench_small.same(box["m"], want)
    uh2 = MemoryUpdateHandler()

    def loop():
        for u, n in zip(cl, ns):
            uh2.submit(u, n)
        bench_small.fedn_loop_fedavg(uh2)
    out["fedn_loop_us"] = med(loop, n=400)
    # the loop's own share that any plug-in pays as well (queue, load, logging, delete): the same
    # loop with the arithmetic taken out; FEDn's arithmetic alone is the rest
    real = ref.increment_average
    ref.increment_average = lambda m, mn, n, N: m
    try:
        out["fedn_loop_no_arith_us"] = med(loop, n=400)
    finally:
        ref.increment_average = real
    out["fedn_arith_us"] = med(lambda: real(cl[0], cl[1], ns[1], ns[0] + ns[1]))
    # round 6: the one-call round's own floor (smallround.py): the native wait + fold_host + stream wait
    # over an arena already packed, into a pooled pinned block — no Python between launch and wait
    from fedn_amd import smallround
    from fedn_amd.layout import Layout
    sess = smallround.SmallSession(dev, Layout.of(cl[0]))
    for k, u in enumerate(cl):
        sess.wait(sess.admit(u, k))
    blk = sess.result_block()
    out["fold_host_k2_us"] = med(lambda: sess.fold(blk, 2, [0.0, float(ns[1])], [1.0, float(ns[0] + ns[1])], 0))
    out["admit_us"] = med(lambda: sess.wait(sess.admit(cl[1], 1)))
    # FedOpt K = 2 (adam) through the plug-in and FEDn's loop restated, the same updates
    uh3 = MemoryUpdateHandler()
    gid = uh3.put_global_model(base, "g0")
    opt = get_aggregator("fedopt", uh3)

    def plugin_opt():
        for u, n in zip(cl, ns):
            uh3.submit(u, n, model_id=gid)
        box["o"], _ = opt.combine_models(helper=None, parameters=bench_small.PARAMS)
    out["plugin_fedopt_us"] = med(plugin_opt, n=400)
    uh4 = MemoryUpdateHandler()
    gid4 = uh4.put_global_model(base, "g0")
    st4 = ref.FedOptState()

    def loop_opt():
        for u, n in zip(cl, ns):
            uh4.submit(u, n, model_id=gid4)
        bench_small.fedn_loop_fedopt(uh4, st4, bench_small.PARAMS)
    out["fedn_loop_fedopt_us"] = med(loop_opt, n=400)
    gpu_floor = out["pack_k2_us"][0] + min(out["fold2_zero_copy_spin_us"][0], out["fold_zero_copy_us"][0])
    out["budget_us"] = round(out["fedn_loop_us"][0] - out["fedn_loop_no_arith_us"][0], 2)
    out["gpu_floor_us"] = round(gpu_floor, 2)
    print(json.dumps(out), flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        plugin()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())
    # the FedOpt plug-in's host work, by own time and by cumulative time
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(300):
        plugin_opt()
    pr.disable()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(35)
        print(f"# FedOpt plug-in, by {key}")
        print(s.getvalue())


if __name__ == "__main__":
    main()
