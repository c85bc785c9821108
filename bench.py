"""bench.py — device-resident FedAvg reduce on MI355X (BASELINE.json metric).

One "step" = one complete FedAvg aggregation of K client updates (default 64 x 100 M
fp32, all resident in HBM) into a fresh aggregate: fedavg.py's fold loop
``x <- x + (n_k*(y_k - x))/N_k`` over k = 1..K-1 in queue order.
value = aggregated client-params/s = K * P / t_step for the WHOLE job.

N = 1 (the BASELINE metric's workload — 64 x 100 M fp32, the north star's one-GPU target — on
one GPU): one libfedagg launch per step. Beside it: ``fedopt`` (configs[3]) and, with --configs1,
``configs1`` (BASELINE configs[1]: the same model with 8 clients).

N > 1 (BASELINE configs[2]: the same 100 M-param model, param-sharded across N GPUs with an
RCCL all-gather): one process per GPU; the flat model is dealt block-cyclically over the
ranks in R rounds (sharded.CyclicShardedFedAvg); each rank folds its chunk of round i and an
RCCL ``all_gather_into_tensor`` of round i (on a communication stream) runs while round i+1
folds, so every GPU ends the step holding the whole aggregated model. The all-gather is
INSIDE the timed step; total work is fixed as N grows ("scaling": "strong").
Beside the line at N > 1: ``weak_scaling`` (every rank folds its own 100 M slice, no
collective), ``allgather`` (a plain all-gather of the model), ``gather_to_host`` (each rank
D2H's its slice, FEDn's real consumer, roundhandler.py:465-468), ``in_process`` (one
process driving all N GPUs, as a FEDn combiner with FEDN_AMD_DEVICES does: each device folds
its slice and copies it into one pinned host model) and ``fedopt_waves`` (BASELINE configs[4]:
1 B bf16 params x 128 FedYogi updates streamed from pinned host memory in waves, sliced over the
N GPUs of one process, each over its own PCIe link; fedn_amd/waves.py).

Also measured in the same run:
  roofline      algorithmic bytes of the fold (K*P*4 + P*4 per launch at N = 1; per rank and
                step at N > 1) / its kernel time (HIP events on the launch stream) vs the
                8.0 TB/s HBM3E peak; ``traffic`` = HBM bytes per launch from rocprofv3 PMC
                counters (profiles/pmc_traffic.json, collected by tools/gpu_session.sh pmc + tools/pmc_traffic.py --session) when
                that entry was measured on the libfedagg.so this run loads (its sha256), else
                null with the reason
  cpu_baseline  the numpy restatement of numpyhelper.increment_average (oracle/, bit-equal to
                FEDn) on a bounded sample (K clients x S params) on one host core; its result is
                also compared bit-for-bit with the GPU aggregate of the same elements
  achievable    (N = 1) the achievable-peak reference on the same box: a STREAM-style
                copy and a streaming read of one 4 GiB buffer (probe kernels of libfedagg_probe.so)
                and the headline kernel's fraction of the copy rate
  fedopt        (N = 1) BASELINE configs[3]: FedAdam over 32 device-resident 350 M fp32 updates,
                one fused pseudo-gradient + server-step launch; round 1 and steady state (fp64
                old / m / v, the dtype flow fedopt.py produces), each with its own roofline, a
                bit-exact check of a sample against the oracle and ``access_pattern``: the same
                loads and stores with the arithmetic cut to adds (probe kernel k_fedopt_mix), the
                HBM ceiling of the kernel's own traffic pattern
  configs0      (N = 1) BASELINE configs[0]: the mnist-pytorch model's K = 2 round through the
                plug-ins' combine_models (FedAvg and FedAdam, the one-call small rounds of
                fedn_amd/smallround.py), median µs per round, bit-exact, beside FEDn's own loop
                restated around the oracle's numpy arithmetic (its cpu_baseline)
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "aggregated params/sec (device-resident) — FedAvg 64-client reduce, 100M fp32"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
AG_ROUNDS = (1, 2, 4, 8, 16)   # N > 1 candidates for the fold + all-gather rounds (--ag-rounds 0)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--params", type=int, default=100_000_000, help="params of the (global) model")
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32")
    ap.add_argument("--cpu-sample", type=int, default=100_000_000,
                    help="params per client in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--ag-rounds", type=int, default=0,
                    help="N > 1: rounds of the overlapped fold + all-gather (0 = the fastest of AG_ROUNDS, chosen in "
                         "the untimed warm-up)")
    ap.add_argument("--fedopt-params", type=int, default=350_000_000, help="configs[3] side field (0 = skip)")
    ap.add_argument("--fedopt-clients", type=int, default=32)
    ap.add_argument("--no-side", action="store_true", help="N > 1: skip the beside-the-line measurements")
    ap.add_argument("--configs1", action="store_true",
                    help="N = 1: add the configs[1] field (K = 8, same kernel: off by default so that a rocprofv3 "
                         "--stats run of the default command averages the headline launches only)")
    ap.add_argument("--waves-params", type=int, default=1_000_000_000, help="configs[4] side field (0 = skip)")
    ap.add_argument("--waves-clients", type=int, default=128)
    ap.add_argument("--waves-pool", type=int, default=8, help="distinct pinned host updates (reused cyclically)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-achievable", dest="achievable", action="store_false",
                    help="N = 1: skip the achievable-peak copy / read reference")
    ap.add_argument("--transport", choices=["auto", "collective", "p2p", "p2p_kernel", "p2p_fused"], default="auto",
                    help="N > 1: how each folded round reaches every GPU — RCCL all-gather, direct peer DMA copies, "
                         "one push kernel per round, or the fold kernel storing into every peer itself (auto = the "
                         "fastest in the untimed warm-up)")
    ap.add_argument("--host-clients", type=int, default=16,
                    help="host_resident side field: host numpy updates through the plug-in (0 = skip)")
    ap.add_argument("--launch-check", action="store_true", help="rank set-up only (gloo, no GPU): the launcher's test")
    return ap.parse_args()


_T0 = time.perf_counter()


def progress(msg):
    """A progress line on stderr (rank 0; stdout carries only the JSON line): a long multi-rank run
    shows where it is."""
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def make_updates(K, P, dtype, device, seed):
    """Synthetic client updates: base ~ N(0,1), client k = base + 0.01 N(0,1)."""
    g = torch.Generator(device=device).manual_seed(seed)
    base = torch.randn(P, generator=g, device=device)
    ups = []
    for _ in range(K):
        u = torch.randn(P, generator=g, device=device).mul_(0.01).add_(base)
        ups.append(u.to(torch.bfloat16) if dtype == "bf16" else u)
    del base
    torch.cuda.synchronize(device)
    return ups


def file_sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def pmc_traffic(workload):
    """(HBM bytes per launch, provenance) from rocprofv3 PMC runs (tools/gpu_session.sh pmc) — only if
    the measured kernels' gfx950 code in the loaded libfedagg.so is the code the entry was collected
    on (``code_sha`` over ``symbols``, fedn_amd/codeobj.py; entries without it: the sha256 of the
    whole file); else (None, reason)."""
    from fedn_amd import _abi
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            ent = json.load(f).get(workload)
    except (OSError, ValueError):
        return None, {"note": "profiles/pmc_traffic.json unreadable"}
    if ent is None:
        return None, {"note": f"no PMC entry for workload {workload}"}
    src = {"file": "profiles/pmc_traffic.json", "workload": workload, "lib_sha": ent.get("lib_sha"),
           "kernel_src_sha": ent.get("kernel_src_sha"), "collected": ent.get("collected"),
           "read_bytes": ent.get("read_bytes"), "write_bytes": ent.get("write_bytes")}
    if ent.get("code_sha") and ent.get("symbols"):
        # keyed on the measured kernels' own gfx950 machine code + descriptors (fedn_amd/codeobj.py):
        # valid on any build of the library whose those bytes are unchanged (another build path, other
        # kernels edited), stale as soon as they change
        from fedn_amd import codeobj
        try:
            now = codeobj.kernel_sha(_abi.lib_path(), ent["symbols"])
        except (OSError, ValueError) as e:
            now = None
            src["note"] = f"code object unreadable: {e}"
        src["code_sha"] = ent["code_sha"]
        if now != ent["code_sha"]:
            src.setdefault("note", "stale: the measured kernels' machine code changed since the PMC run; re-run "
                                   "tools/gpu_session.sh pmc + tools/pmc_traffic.py --session")
            return None, src
        return ent["bytes"], src
    if ent.get("lib_sha") != file_sha(_abi.lib_path()):
        src["note"] = ("stale: collected on another build of libfedagg.so; re-run tools/gpu_session.sh pmc + "
                       "tools/pmc_traffic.py --session")
        return None, src
    return ent["bytes"], src


def cpu_baseline(ups, ns, agg, S):
    """Time the oracle (numpy, 1 core) on a K x S sample and check the GPU result on it."""
    from oracle import numpy_ref as ref  # test infrastructure: the baseline/checker only

    S = min(S, agg.numel())
    sample = [u[:S].float().cpu().numpy() for u in ups]
    t0 = time.perf_counter()
    want = ref.fedavg_flat(sample, ns)
    dt = time.perf_counter() - t0
    got = agg[:S].cpu().numpy()
    exact = bool(np.array_equal(got.view(np.uint32), want.view(np.uint32)))
    return {"value": len(ups) * S / dt, "unit": "params/s", "cores": 1, "kind": "port",
            "sample": f"{len(ups)} clients x {S} fp32 params (first {S} of each client buffer); "
                      f"numpy {np.__version__} oracle/numpy_ref.fedavg_flat, single-threaded, "
                      f"{os.cpu_count()} host cores present", "seconds": dt,
            "gpu_bit_exact_on_sample": exact, "threaded": cpu_threaded(sample, ns, want)}


def usable_cores():
    """The cores this process may keep busy: its CPU affinity, capped by a cgroup CPU quota (a GPU box
    shows every core of the machine but grants a share of them)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:                     # cgroup v2: "<quota> <period>"
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        try:                                                         # cgroup v1
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                quota = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                period = int(f.read())
            if quota > 0:
                n = min(n, max(1, -(-quota // period)))
        except (OSError, ValueError):
            pass
    return n


def cpu_threaded(sample, ns, want):
    """SURVEY §8(d)'s optional labelled line: the same oracle over the same sample sliced by
    parameters across every core this process may use (numpy ufuncs release the GIL; each element's
    recurrence is untouched, so the result is the single-threaded one, checked)."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import numpy_ref as ref  # test infrastructure: the baseline/checker only
    cores = usable_cores()
    S = want.size
    bounds = [(S * i // cores, S * (i + 1) // cores) for i in range(cores)]
    out = np.empty_like(want)

    def part(lo, hi):
        out[lo:hi] = ref.fedavg_flat([u[lo:hi] for u in sample], ns)

    with ThreadPoolExecutor(cores) as ex:
        t0 = time.perf_counter()
        for f in [ex.submit(part, lo, hi) for lo, hi in bounds]:
            f.result()
        dt = time.perf_counter() - t0
    return {"value": len(sample) * S / dt, "unit": "params/s", "cores": cores, "seconds": dt,
            "same_as_single_threaded": bool(np.array_equal(out.view(np.uint32), want.view(np.uint32))),
            "note": "numpy oracle sliced over parameters on a thread per core; reported beside the 1-core "
                    "baseline, not instead of it"}


def timed_steps(step, steps, stream, world, device, on_cpu):
    """Barrier + sync, ``steps`` calls of ``step`` bracketed by HIP events on ``stream``, sync +
    barrier; returns (wall seconds, mean event ms), each the max over ranks."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    ranks = dist.is_initialized()
    if ranks:
        dist.barrier()
    torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize(device)
    if ranks:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ev_ms = sum(s.elapsed_time(e) for s, e in ev) / steps
    t = torch.tensor([elapsed, ev_ms], dtype=torch.float64, device="cpu" if on_cpu else device)
    if ranks:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), float(t[1])


def fedopt_waves_side(a, devs, sample=1_000_000):
    """BASELINE configs[4]: K bf16 updates of P params streamed from pinned host memory in waves of 8,
    FedYogi, parameter-sliced over ``devs`` in one process (each GPU copies only its slice of every
    update over its own PCIe link; fedn_amd.waves). The first ``sample`` params of the result are
    checked bit-for-bit against the oracle on the exact f32 upcasts of the same bf16 updates."""
    import hashlib

    from fedn_amd.waves import WaveFedOpt
    from oracle import numpy_ref as ref  # the checker of the sample only
    P, K, pool = a.waves_params, a.waves_clients, a.waves_pool
    g = torch.Generator(device=devs[0]).manual_seed(5)
    base = torch.randn(P, generator=g, device=devs[0])
    host = []
    for _ in range(pool):
        h = torch.empty(P, dtype=torch.bfloat16, pin_memory=True)
        h.copy_((base + 0.01 * torch.randn(P, generator=g, device=devs[0])).to(torch.bfloat16))
        host.append(h)
    base = base.cpu()
    ups = [host[k % pool] for k in range(K)]
    ns = [int(v) for v in np.random.default_rng(5).integers(1, 5001, K)]
    params = {"serveropt": "yogi"}
    wf = WaveFedOpt(devs, P, wave=8)
    old = wf.slices(base.double())
    wf.round(ups[:8], ns[:8], old, params)                         # warm-up (allocations, kernels)
    wf = WaveFedOpt(devs, P, wave=8)
    t0 = time.perf_counter()
    outs = wf.round(ups, ns, old, params)
    t = time.perf_counter() - t0
    # per-kernel rooflines: the same round again with HIP events around every launch (round 1 of a
    # session: waves read 8 bf16 updates + f64 old and write the f64 pg workspace, later waves also
    # read it; the last wave reads it and writes m / v / out instead, the server step fused)
    spans = {}
    WaveFedOpt(devs, P, wave=8).round(ups, ns, old, params, kernel_times=spans)
    per_el = {"first": lambda k: 2 * k + 16, "mid": lambda k: 2 * k + 24, "final": lambda k: 40,
              "mid_final": lambda k: 2 * k + 40, "first_final": lambda k: 2 * k + 32}
    kern = {}
    for kind, rows in spans.items():
        ms = sum(r[3] for r in rows) / len(rows)
        b = sum(r[1] * per_el[kind](r[2]) for r in rows) / len(rows)
        traffic, tsrc = pmc_traffic(f"fedyogi_wave_{kind}_p{P // len(devs)}_w8_bf16")
        kern[kind] = {"launches": len(rows), "ms": ms, "alg_bytes_per_launch": b,
                      "roofline": {"bound": "hbm", "achieved": b / ms / 1e6, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": b / ms / 1e6 / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc},
                      "kernel": {"first": "k_fedopt_c<bf16, double, CF64, FIRST, !FINAL>",
                                 "mid": "k_fedopt_c<bf16, double, CF64, !FIRST, !FINAL>",
                                 "final": "k_fedopt_c<bf16, double, CF64, !FIRST, FINAL> (K = 0 server step)",
                                 "mid_final": "k_fedopt_c<bf16, double, CF64, !FIRST, FINAL> (last wave + server step)",
                                 "first_final": "k_fedopt_c<bf16, double, CF64, FIRST, FINAL> (one wave)"}[kind],
                      "bytes_per_element": {"first": "2W + 16 (W bf16 updates, f64 old, f64 pg written)",
                                            "mid": "2W + 24 (W bf16 updates, f64 old, f64 pg read + written)",
                                            "final": "40 (f64 old + pg read; f64 m / v / out written)",
                                            "mid_final": "2W + 40 (W bf16 updates, f64 old + pg read; f64 m / v / "
                                                         "out written)",
                                            "first_final": "2W + 32 (W bf16 updates, f64 old read; f64 m / v / out "
                                                           "written)"}[kind]}
    res = wf.gather(outs)
    S = min(sample, P)
    want, _ = ref.fedopt_combine(ref.FedOptState(), [([ups[k][:S].float().numpy()], n) for k, n in enumerate(ns)],
                                 [base[:S].double().numpy()], {**ref.DEFAULT_FEDOPT, **params})
    exact = bool(np.array_equal(res[:S].numpy().view(np.uint64), want[0].view(np.uint64)))
    checksum = hashlib.sha256(res.numpy().tobytes()).hexdigest()[:16]
    del host, ups, old, outs, wf, res
    torch.cuda.empty_cache()
    return {"s": t, "value": K * P / t, "unit": "params/s", "params": P, "clients": K, "wave": 8, "devices": len(devs),
            "h2d_GBps_total": K * P * 2 / t / 1e9, "h2d_GBps_per_link": K * P * 2 / t / 1e9 / len(devs),
            "checksum_sha256_16": checksum, "bit_exact_on_sample": exact, "kernels": kern,
            "sample": f"first {S} params vs oracle/numpy_ref.fedopt_combine on the f32 upcasts",
            "note": f"BASELINE configs[4]: {pool} distinct pinned bf16 updates reused cyclically (every one "
                    "crosses PCIe); PCIe-bound by design; not in value"}


def fedavg_pattern(ups, agg, stream, device, alg_bytes, kern_ms, a):
    """The headline fold's traversal with one add per element instead of the fold (fa_stream_sum,
    libfedagg_probe.so: the same pipelined 4-strip kernel, client table and non-temporal stores):
    the HBM ceiling of the fold's own access pattern on this box."""
    from fedn_amd import _abi, ops
    with _abi.use_probe():
        fn = lambda: ops.stream_sum(agg, ups, stream=stream)  # noqa: E731
        for _ in range(3):
            fn()
        _, ms = timed_steps(fn, a.steps, stream, 1, device, False)
    return {"ms": ms, "frac": alg_bytes / (ms / 1e3) / 1e9 / HBM_PEAK_GBS, "kernel_over_pattern": ms / kern_ms,
            "kernel": "k_fedavg_pipe<CADD> (fa_stream_sum, libfedagg_probe.so)",
            "note": "the fold's exact traversal with x + y instead of x + n(y - x)/N and no store window; "
                    "not in value (the windowed fold can beat it)"}


def achieved_of(alg_bytes, kern_ms):
    return alg_bytes / (kern_ms / 1e3) / 1e9


def achievable_side(device, headline_gbs, nbytes=4 << 30):
    """SURVEY.md §8(d)'s achievable-peak reference on this box: a STREAM-style copy (16 B per lane,
    read once + written once) and a streaming read of one ``nbytes`` buffer, by the probe kernels
    of libfedagg_probe.so (measurement only; the headline ran on libfedagg.so)."""
    from fedn_amd import _abi, ops
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(device)
    res = {}
    with _abi.use_probe():
        sink = ops.stream_read_sink(src)
        for name, fn, moved in (("copy", lambda: ops.stream_copy(dst, src, stream=stream), 2 * nbytes),
                                ("read", lambda: ops.stream_read(src, sink, stream=stream), nbytes)):
            for _ in range(3):
                fn()
            _, ms = timed_steps(fn, 10, stream, 1, device, False)
            res[f"{name}_GBps"] = moved / (ms / 1e3) / 1e9
    res["headline_frac_of_copy"] = headline_gbs / res["copy_GBps"]
    res["kernels"] = "k_stream_copy / k_stream_read<16> (libfedagg_probe.so)"
    res["note"] = f"achievable-peak reference on this box over one {nbytes >> 30} GiB buffer; not in value"
    del src, dst, sink
    torch.cuda.empty_cache()
    return res


def side(fn):
    """A beside-the-line measurement: an error is reported in its field, never instead of value."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001
        return {"error": f"{type(e).__name__}: {e}"}


def configs0_side(device, rounds=300, warm=30):
    """BASELINE configs[0]'s round (examples/mnist-pytorch: 52,650 fp32 params in 6 tensors, K = 2 host
    numpy updates) through the plug-ins' combine_models (the one-call small rounds, fedn_amd/smallround.py),
    FedAvg and FedAdam, median µs per round including the stand-in update handler's submit of both
    updates — beside FEDn's own loop restated around the oracle's numpy arithmetic over the same
    handler (tools/bench_small.py: fedavg.py:45-83, fedopt.py:74-121), the CPU baseline of this field.
    Every plug-in round is checked bit-exact against the oracle."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import bench_small
    from fedn_amd.aggregators import get_aggregator
    from fedn_amd.updatehandler import MemoryUpdateHandler
    from oracle import numpy_ref as ref  # the checker and the CPU baseline only

    rng = np.random.default_rng(0)
    base = [rng.standard_normal(s).astype(np.float32) for s in bench_small.MNIST]
    cl = [[(b + 0.01 * rng.standard_normal(b.shape)).astype(np.float32) for b in base] for _ in range(2)]
    ns = [int(v) for v in rng.integers(1, 5001, 2)]

    def med(fn):
        for _ in range(warm):
            fn()
        ts = []
        for _ in range(rounds):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2] * 1e6

    out, box = {}, {}
    with torch.cuda.device(device):
        uh = MemoryUpdateHandler()
        agg = get_aggregator("fedavg", uh)

        def avg():
            for u, n in zip(cl, ns):
                uh.submit(u, n)
            box["avg"], _ = agg.combine_models(helper=None)
        out["fedavg_us"] = med(avg)
        want, _ = ref.fedavg_combine(list(zip(cl, ns)))
        out["fedavg_bit_exact"] = bench_small.same(box["avg"], want)
        uh2 = MemoryUpdateHandler()
        gid = uh2.put_global_model(base, "g0")
        opt = get_aggregator("fedopt", uh2)
        st = ref.FedOptState()

        def fedadam():
            for u, n in zip(cl, ns):
                uh2.submit(u, n, model_id=gid)
            box["opt"], _ = opt.combine_models(helper=None, parameters=bench_small.PARAMS)
        fedadam()                           # round 1 (m / v None), then the steady state is timed
        ref.fedopt_combine(st, list(zip(cl, ns)), base, bench_small.PARAMS)
        out["fedadam_us"] = med(fedadam)
        for _ in range(warm + rounds):      # the oracle's session over the same rounds
            want_o, _ = ref.fedopt_combine(st, list(zip(cl, ns)), base, bench_small.PARAMS)
        ok = bench_small.same(box["opt"], want_o)
        out["fedadam_bit_exact"] = ok
    uh3 = MemoryUpdateHandler()

    def loop_avg():
        for u, n in zip(cl, ns):
            uh3.submit(u, n)
        bench_small.fedn_loop_fedavg(uh3)
    uh4 = MemoryUpdateHandler()
    gid4 = uh4.put_global_model(base, "g0")
    st4 = ref.FedOptState()

    def loop_opt():
        for u, n in zip(cl, ns):
            uh4.submit(u, n, model_id=gid4)
        bench_small.fedn_loop_fedopt(uh4, st4, bench_small.PARAMS)
    out["cpu_baseline"] = {"fedavg_us": med(loop_avg), "fedadam_us": med(loop_opt), "unit": "us per round",
                           "cores": 1, "kind": "port",
                           "sample": "FEDn's combine_models loop restated (tools/bench_small.py) around "
                                     "oracle/numpy_ref's numpyhelper arithmetic, the same handler and updates"}
    out["unit"] = "us per round (median, incl. the handler's submit of both updates)"
    out["config"] = "BASELINE configs[0]: mnist-pytorch (52,650 fp32 params, 6 tensors), 2 host numpy updates"
    return out


def fold_kernel_label(P, in_bytes, K, ran=None):
    """The fold kernel's description; ``ran`` = the family the library reports it launched last on this
    thread (ops.last_kernel(), fa_last_kernel) — what ran, not what the size rules suggest."""
    from fedn_amd import ops
    ran = ran or ops.last_kernel()
    strips = ("4 x 16-B strips per lane" if in_bytes == 4 else "8 strips of 4 elements per lane, bf16 -> f32")
    if ran == "k_fedavg_pipe_win":
        return (f"k_fedavg_pipe_win ({strips}, next client prefetched; every wave's stores inside a chip-wide "
                "window of the GPU's 100 MHz clock)")
    if ran == "k_fedavg_pipe":
        return f"k_fedavg_pipe ({strips}, next client prefetched; no store window)"
    if ran == "k_fedavg":
        return f"k_fedavg (1 x 16-B strip per lane, {8 if in_bytes < 4 or K <= 8 else 4} clients loaded ahead)"
    return ran or "unknown (no fold launched on this thread)"


OPT_KERNELS = {
    "k_fedopt_cw": ("k_fedopt_cw (pseudo-gradient fold + Adam step fused; 4 coalesced element pairs per lane; the "
                    "stores of all waves in a common window of the GPU's 100 MHz clock)"),
    "k_fedopt_c": ("k_fedopt_c (pseudo-gradient fold + Adam step fused; 4 coalesced element pairs per lane; no "
                   "store window)"),
    "k_fedopt": "k_fedopt (pseudo-gradient fold + Adam step fused; per-lane strips)",
}


def configs1_side(ups, ns, agg, stream, device, in_bytes, a):
    """BASELINE configs[1]: FedAvg of 8 device-resident updates of the same model (the first 8
    buffers of the main line's), one launch per step, its own roofline."""
    from fedn_amd import ops
    K, P = len(ups), agg.numel()
    Ns = [int(v) for v in np.cumsum(ns)]
    step = lambda: ops.fedavg_fold(agg, ups, ns, Ns, init=True, stream=stream)  # noqa: E731
    for _ in range(3):
        step()
    el, kms = timed_steps(step, a.steps, stream, 1, device, False)
    b = K * P * in_bytes + P * 4
    traffic, tsrc = pmc_traffic(f"fedavg_k{K}_p{P}_{a.dtype}")
    return {"value": K * P / (el / a.steps), "unit": "params/s", "ms_per_step": el / a.steps * 1e3,
            "roofline": {"bound": "hbm", "achieved": b / (kms / 1e3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                         "kernel": fold_kernel_label(P, in_bytes, K), "kernel_ms": kms, "alg_bytes_per_launch": b},
            "config": f"BASELINE configs[1]: FedAvg, {K} device-resident {a.dtype} updates x {P} params"}


def fedopt_side(P, K, device, steps=10, warm=2, sample=1_000_000, pattern_probe=True):
    """BASELINE configs[3]: FedAdam, K device-resident fp32 updates of P params, state in HBM;
    one fused fa_fedopt_step launch per round. Round 1 (old fp32, m / v None) and steady state
    (old / m / v fp64). Algorithmic bytes: K*P*4 + P*4 + P*(4+8+8) and P*(4K+48)."""
    from fedn_amd import ops
    from oracle import numpy_ref as ref  # the checker of the sample only

    g = torch.Generator(device=device).manual_seed(4)
    old32 = torch.randn(P, generator=g, device=device)
    ups = [torch.randn(P, generator=g, device=device).mul_(0.01).add_(old32) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(4).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    out = torch.empty(P, dtype=torch.float64, device=device)
    v = torch.empty(P, dtype=torch.float64, device=device)
    m32 = torch.empty(P, dtype=torch.float32, device=device)
    stream = torch.cuda.current_stream(device)
    params = {"serveropt": "adam", "learning_rate": 1e-3, "beta1": 0.9, "beta2": 0.99, "tau": 1e-4}
    kw = {k: params[k] for k in ("learning_rate", "beta1", "beta2", "tau")}

    def r1():
        ops.fedopt_step(old32, ups, ns, Ns, first=True, final=True, m_out=m32, v_out=v, out=out, serveropt="adam",
                        stream=stream, **kw)

    res = {}
    for _ in range(warm):
        r1()
    _, ms1 = timed_steps(r1, steps, stream, 1, device, False)
    ran = {"round1": ops.last_kernel()}
    # checker: round 1 on a sample, then the steady-state inputs of the sample
    S = min(sample, P)
    old_s = old32[:S].cpu().numpy()
    ups_s = [([u[:S].cpu().numpy()], n) for u, n in zip(ups, ns)]
    st = ref.FedOptState()
    t0 = time.perf_counter()
    want1, _ = ref.fedopt_combine(st, ups_s, [old_s], params)
    cpu1 = time.perf_counter() - t0
    ok1 = bool(np.array_equal(out[:S].cpu().numpy().view(np.uint64), want1[0].view(np.uint64)) and
               np.array_equal(m32[:S].cpu().numpy().view(np.uint32), st.m[0].view(np.uint32)) and
               np.array_equal(v[:S].cpu().numpy().view(np.uint64), st.v[0].view(np.uint64)))
    old64, m64, v64 = out.clone(), m32.double(), v.clone()
    m_out = torch.empty(P, dtype=torch.float64, device=device)
    v_out = torch.empty(P, dtype=torch.float64, device=device)
    out2 = torch.empty(P, dtype=torch.float64, device=device)

    def r2():
        ops.fedopt_step(old64, ups, ns, Ns, first=True, final=True, m_in=m64, m_out=m_out, v_in=v64, v_out=v_out,
                        out=out2, serveropt="adam", stream=stream, **kw)

    for _ in range(warm):
        r2()
    _, ms2 = timed_steps(r2, steps, stream, 1, device, False)
    ran["steady"] = ops.last_kernel()
    st.m = [st.m[0].astype(np.float64)]           # the GPU's steady state takes m in float64 (round >= 3)
    t0 = time.perf_counter()
    want2, _ = ref.fedopt_combine(st, ups_s, want1, params)
    cpu2 = time.perf_counter() - t0
    ok2 = bool(np.array_equal(out2[:S].cpu().numpy().view(np.uint64), want2[0].view(np.uint64)) and
               np.array_equal(m_out[:S].cpu().numpy().view(np.uint64), st.m[0].view(np.uint64)) and
               np.array_equal(v_out[:S].cpu().numpy().view(np.uint64), st.v[0].view(np.uint64)))
    # fp32-state mode (aggregators.fedopt_f32state, fa_fedopt_step_ex state F32): the steady state of a
    # float32 model with float32 m / v — round 1's results rounded to f32 as the mode stores them
    old_f, m_f, v_f = out.float(), m32.clone(), v.float()
    m_o32, v_o32, out32 = (torch.empty(P, dtype=torch.float32, device=device) for _ in range(3))

    def r3():
        ops.fedopt_step(old_f, ups, ns, Ns, first=True, final=True, m_in=m_f, m_out=m_o32, v_in=v_f, v_out=v_o32,
                        out=out32, serveropt="adam", stream=stream, **kw)

    for _ in range(warm):
        r3()
    _, ms3 = timed_steps(r3, steps, stream, 1, device, False)
    ran["steady_f32state"] = ops.last_kernel()
    st3 = ref.FedOptState()
    st3.m, st3.v = [m_f[:S].cpu().numpy()], [v_f[:S].cpu().numpy()]
    t0 = time.perf_counter()
    want3, _ = ref.fedopt_combine_f32state(st3, ups_s, [old_f[:S].cpu().numpy()], params)
    cpu3 = time.perf_counter() - t0
    ok3 = bool(np.array_equal(out32[:S].cpu().numpy().view(np.uint32), want3[0].view(np.uint32)) and
               np.array_equal(m_o32[:S].cpu().numpy().view(np.uint32), st3.m[0].view(np.uint32)) and
               np.array_equal(v_o32[:S].cpu().numpy().view(np.uint32), st3.v[0].view(np.uint32)))
    # the ceiling of the kernel's own access pattern: the same loads and stores with one add per value
    # (k_fedopt_mix, libfedagg_probe.so; its outputs are not used), timed after the product launches
    pattern = {}
    if pattern_probe:
        from fedn_amd import _abi
        try:
            with _abi.use_probe():
                ops.tune(opt_mix=1)
                for phase, fn in (("round1", r1), ("steady", r2)):
                    for _ in range(warm):
                        fn()
                    pattern[phase] = timed_steps(fn, steps, stream, 1, device, False)[1]
        finally:
            with _abi.use_probe():
                ops.tune(opt_mix=0)
    for phase, ms, b, ok, cpu_s in (("round1", ms1, K * P * 4 + P * 4 + P * 20, ok1, cpu1),
                                    ("steady", ms2, P * (4 * K + 48), ok2, cpu2),
                                    ("steady_f32state", ms3, P * (4 * K + 24), ok3, cpu3)):
        wl = f"fedopt_adam_{phase}_k{K}_p{P}"
        traffic, tsrc = pmc_traffic(wl)
        gbs = b / ms / 1e6
        res[phase] = {"ms": ms, "params_per_s": K * P / (ms / 1e3),
                      "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": gbs / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                                   "kernel": OPT_KERNELS.get(ran[phase], ran[phase]),
                                   "alg_bytes_per_launch": b},
                      "bit_exact_on_sample": ok,
                      "sample": f"first {S} params of every buffer vs oracle/numpy_ref" +
                                (".fedopt_combine_f32state (the mode's definition: the reference step on the "
                                 "stored f32 state, rounded once to f32)" if phase == "steady_f32state" else ""),
                      "cpu_baseline": {"value": K * S / cpu_s, "unit": "params/s", "cores": 1, "kind": "port",
                                       "sample": f"{K} clients x {S} params: oracle/numpy_ref.fedopt_combine (the "
                                                 "fedopt.py restatement, numpy, single-threaded)", "seconds": cpu_s}}
        if phase in pattern:
            res[phase]["access_pattern"] = {
                "ms": pattern[phase], "frac": b / pattern[phase] / 1e6 / HBM_PEAK_GBS,
                "kernel_over_pattern": pattern[phase] / ms,
                "note": "k_fedopt_mix (libfedagg_probe.so): k_fedopt_c's exact loads and stores with one add per value "
                        "instead of the arithmetic and no store window; the HBM ceiling of the unwindowed pattern on "
                        "this box (k_fedopt_cw times its stores into a chip-wide window: it can beat it)"}
    res["config"] = (f"BASELINE configs[3]: FedAdam, {K} device-resident fp32 updates x {P} params, m / v in HBM "
                     "(fedopt.py:151-185), one fused launch per round")
    res["steady_f32state"]["vs_steady_ms"] = ms3 / ms2
    res["steady_f32state"]["note"] = ("fp32-state mode (aggregators.fedopt_f32state): m / v / model stored in "
                                      "float32, P*(4K+24) bytes; opt-in, not the reference's dtype flow")
    del ups, old32, out, v, m32, old64, m64, v64, m_out, v_out, out2, old_f, m_f, v_f, m_o32, v_o32, out32
    torch.cuda.empty_cache()
    return res


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(n):
    """``bench.py --gpus N`` outside torch.distributed.run: start one child process per rank with the
    contract's environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT), wait
    for all of them, and return the first failure's exit status (the other ranks are then stopped by
    their exact PIDs). This process only starts children: it never touches the GPU and never execs."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc, live = 0, list(procs)
    while live:
        for pr in list(live):
            r = pr.poll()
            if r is None:
                continue
            live.remove(pr)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for other in live:
                    other.kill()
        time.sleep(0.1)
    return rc


def launch_check(world, rank):
    """--launch-check: the rank set-up alone (gloo rendezvous, one all-reduce, no GPU) — what the CPU
    test of the self-launch runs."""
    dist.init_process_group("gloo")
    t = torch.tensor([rank + 1], dtype=torch.int64)
    dist.all_reduce(t)
    pids = [None] * world
    dist.all_gather_object(pids, (os.getpid(), os.getppid(), int(os.environ["LOCAL_RANK"])))
    if rank == 0:
        print(json.dumps({"launch_check": True, "world": dist.get_world_size(), "rank_sum": int(t[0]),
                          "ranks": pids}), flush=True)
    dist.destroy_process_group()


def global_chunks(geom, K, P_total, dtype, device, seed, sample):
    """THIS rank's chunks (``geom.local``) of the ONE synthetic model every rank and the N = 1 line
    derive from the same seed — base ~ N(0,1), client k = base + 0.01 N(0,1), the exact sequence of
    make_updates(K, P_total, ...) — plus, when ``sample`` > 0, the first ``sample`` params of every
    client on the host (fp32; for bf16 the exact upcasts of the rounded values) for the checker."""
    g = torch.Generator(device=device).manual_seed(seed)
    base = torch.randn(P_total, generator=g, device=device)
    loc, host = [], []
    for _ in range(K):
        u = torch.randn(P_total, generator=g, device=device).mul_(0.01).add_(base)
        if dtype == "bf16":
            u = u.to(torch.bfloat16)
        loc.append(geom.local(u))
        if sample > 0:
            host.append(u[:sample].float().cpu().numpy())
        del u
    del base
    torch.cuda.synchronize(device)
    return loc, host


def gathered_bits(full, device, on_cpu):
    """(min, max) over ranks of the int64 sum of a gathered model's bits: equal when every rank
    holds the same model."""
    bits = full.contiguous().view(torch.int32).to(device).sum(dtype=torch.int64).reshape(1)
    t = torch.cat([bits, -bits])
    t = t.cpu() if on_cpu else t
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return -int(t[1]), int(t[0])


def sample_check(got, host_sample, ns):
    """Bit-for-bit check of the first params of an aggregate against the oracle (numpy, one core) on
    the same clients' values; returns (equal, oracle seconds)."""
    from oracle import numpy_ref as ref  # test infrastructure: the checker only
    S = host_sample[0].size
    t0 = time.perf_counter()
    want = ref.fedavg_flat(host_sample, ns)
    dt = time.perf_counter() - t0
    g = got[:S].cpu().numpy() if isinstance(got, torch.Tensor) else np.asarray(got[:S])
    return bool(np.array_equal(g.view(np.uint32), want.view(np.uint32))), dt


def host_resident_side(a, devs, ns_all, clients=16, sample=1_000_000, rounds=3):
    """The north star's end-to-end rate: the FedAvg PLUG-IN (fedn_amd.aggregators.fedavg.Aggregator,
    the combiner's call shape) over ``clients`` host-resident numpy updates of the model, with its
    devices = the N GPUs of the node (FEDN_AMD_DEVICES' multi-device pipeline: each update packed
    once into pinned memory, each GPU H2D's its parameter slice over its own PCIe link, folds it,
    D2H's its slice of the result into the host model). A session's rounds after the first; the
    first ``sample`` params checked bit-for-bit against the oracle.

    On several devices a second session, ``pinned_decode``, hands over each round's updates as NEW
    arrays in page-locked memory (fedn_amd.helper.pinned_empty — what the plug-in's helper.load
    decodes large npz members into), which the pipeline DMAs in place without packing; the copy into
    them stands in for the decode and is outside the timed round (tools/bench_hostres.py)."""
    from fedn_amd.aggregators import get_aggregator  # noqa: F401
    from fedn_amd.aggregators.fedavg import Aggregator
    from fedn_amd.helper import pinned_empty
    from fedn_amd.updatehandler import MemoryUpdateHandler
    P = a.params
    ns = ns_all[:clients]
    g = torch.Generator(device=devs[0]).manual_seed(a.seed + 11)
    base = torch.randn(P, generator=g, device=devs[0])
    host = []
    for _ in range(clients):
        host.append(torch.randn(P, generator=g, device=devs[0]).mul_(0.01).add_(base).cpu().numpy())
    del base
    S = min(sample, P)
    nbytes = clients * P * 4

    def session(pinned):
        uh = MemoryUpdateHandler()
        agg = Aggregator(uh, devices=list(devs))
        times = []
        for r in range(rounds + 1):
            for k in range(clients):
                u = host[k]
                if pinned:
                    u = pinned_empty(u.shape, u.dtype)
                    u[...] = host[k]
                uh.submit([u], ns[k])
            del u
            t0 = time.perf_counter()
            model, data = agg.combine_models(helper=None)
            if r:
                times.append(time.perf_counter() - t0)
        t = sorted(times)[len(times) // 2]
        exact, _ = sample_check(model[0], [h[:S] for h in host], ns)
        return t, times, exact, data

    t, times, exact, data = session(False)
    out = {"s": t, "value": clients * P / t, "unit": "params/s", "clients": clients, "params": P,
           "devices": len(devs), "GBps_in": nbytes / t / 1e9, "GBps_per_link": nbytes / t / 1e9 / len(devs),
           "rounds_s": times, "bit_exact_on_sample": exact, "sample": f"first {S} params vs oracle/numpy_ref.fedavg_flat",
           "nr_aggregated_models": data.get("nr_aggregated_models"),
           "h2d_path": ("in place (page-locked arrays DMA'd slice by slice to every GPU)" if data.get("bytes_h2d_in_place")
                        else "packed into pinned slots, then H2D"),
           "bytes_h2d_in_place": data.get("bytes_h2d_in_place"), "bytes_h2d_packed": data.get("bytes_h2d_packed"),
           "note": "FedAvg plug-in over pageable host numpy updates (pack -> pinned slot -> H2D, one slice per "
                   "device) -> fold -> D2H into the host model, median of a session's rounds 2..; PCIe-bound; not "
                   "in value"}
    if len(devs) > 1:
        t, times, exact, data = session(True)
        out["pinned_decode"] = {"s": t, "value": clients * P / t, "GBps_in": nbytes / t / 1e9, "rounds_s": times,
                                "bit_exact_on_sample": exact, "bytes_h2d_in_place": data.get("bytes_h2d_in_place"),
                                "bytes_h2d_packed": data.get("bytes_h2d_packed"),
                                "note": "each round's updates new page-locked arrays (helper.pinned_empty, what "
                                        "helper.load decodes into), DMA'd in place"}
    del host
    torch.cuda.empty_cache()
    return out


def main():
    a = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        # no launcher: this process starts the ranks itself (never touching the GPU first)
        raise SystemExit(self_launch(a.gpus))
    world = int(env_world or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.launch_check:
        return launch_check(world, rank)
    # FEDN_AMD_BENCH_ONE_GPU=1: rehearsal of the N>1 code path on a one-GPU box (every rank on
    # cuda:0, gloo instead of RCCL); never used for reported numbers
    rehearsal = os.environ.get("FEDN_AMD_BENCH_ONE_GPU") == "1"
    # FEDN_AMD_BENCH_RCCL_WORLD1=1: the N>1 code path at world size 1 over a real RCCL communicator
    # (every all-gather issued as a collective), so the RCCL calls run on a one-GPU box; never used
    # for reported numbers
    rccl1 = world == 1 and os.environ.get("FEDN_AMD_BENCH_RCCL_WORLD1") == "1"
    device = torch.device("cuda", 0 if rehearsal else local)
    torch.cuda.set_device(device)
    if world > 1 or rccl1:
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)

    from fedn_amd import _abi, ops
    from fedn_amd.sharded import CyclicShardedFedAvg, P2PAllGather
    _abi.load()

    K = a.clients
    P_total = a.params
    in_bytes = 2 if a.dtype == "bf16" else 4
    ns = [int(v) for v in np.random.default_rng(a.seed).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    stream = torch.cuda.current_stream(device)
    extra = {}
    S = min(a.cpu_sample, P_total) if a.cpu_sample > 0 else 0
    base = None

    if world == 1 and not rccl1:
        P = P_total
        ups = make_updates(K, P, a.dtype, device, a.seed)
        agg = torch.empty(P, dtype=torch.float32, device=device)

        def step():
            ops.fedavg_fold(agg, ups, ns, Ns, init=True, stream=stream)

        for _ in range(a.warmup):
            step()
        elapsed, kern_ms = timed_steps(step, a.steps, stream, world, device, rehearsal)
        alg_bytes = K * P * in_bytes + P * 4           # read every update once, write the aggregate once
        workload = f"fedavg_k{K}_p{P}_{a.dtype}"
        kernel = fold_kernel_label(P, in_bytes, K)
        config = {"workload": f"FedAvg {K} clients x {P} params {a.dtype} per GPU (the BASELINE metric's workload, "
                              "north star at 1 GPU; device-resident, one fused fold launch per aggregation)",
                  "clients": K, "params_per_gpu": P, "global_params": P_total,
                  "parallelism": "param-slice shards x1, no data-path collective"}
        scaling = "weak"
        if rank == 0 and S:
            base = cpu_baseline(ups, ns, agg, S)
    else:
        # the fold + gather step: rounds R (--ag-rounds, or the fastest of AG_ROUNDS) and transport
        # (RCCL all-gather, or direct peer copies: P2PAllGather) chosen in the untimed warm-up by
        # max-over-ranks step time — the all-gather over xGMI, not the fold, sets the step at every
        # N > 1, and only the node itself can tell which transport and message size move it fastest
        cands = [a.ag_rounds] if a.ag_rounds > 0 else list(AG_ROUNDS)
        geoms = {R: CyclicShardedFedAvg(P_total, chunk=-(-P_total // (world * R)), collective_at_world1=rccl1)
                 for R in cands}
        Lmax = max(c.local_len for c in geoms.values())
        full_all = torch.empty(max(c.full_len for c in geoms.values()), dtype=torch.float32, device=device)
        transports = {"collective": None}
        engines = {"p2p": "dma", "p2p_kernel": "kernel", "p2p_fused": "fused"}   # P2PAllGather.engine of each
        if a.transport != "collective" and (world > 1 or rccl1):
            try:
                # double-buffered: one fence per step (the exit fence clears the other buffer); ONE set of
                # IPC mappings serves both engines (the engine is switched between steps)
                pa = P2PAllGather(full_all, spare=torch.empty_like(full_all), verify="close")
                for name in engines:
                    if a.transport in ("auto", name):
                        transports[name] = pa
            except Exception as e:  # noqa: BLE001 — reported; the collective stays
                extra["p2p_error"] = f"{type(e).__name__}: {e}"
        if a.transport in engines and a.transport in transports:
            del transports["collective"]

        def use(name):
            tp = transports[name]
            if tp is not None:
                tp.engine = engines[name]
            return tp
        agg_all = torch.empty(Lmax, dtype=torch.float32, device=device)

        def make_step(c, tp, loc, res=None):
            ag = agg_all[:c.local_len]
            out = None if (rehearsal and tp is None) else full_all[:c.full_len]

            def st():
                r = c.fold_allgather(ag, loc, ns, Ns, init=True, out=out, p2p=tp)
                if res is not None:
                    res[0] = r
            return st

        tuned = {}
        if len(cands) * len(transports) > 1:
            scratch = make_updates(K, Lmax, a.dtype, device, a.seed + 1000 * rank + 1)   # timing only
            sums = {}
            for name in transports:
                tp = use(name)
                progress(f"warm-up: transport {name}, rounds {list(geoms)}")
                for R, c in geoms.items():
                    res = [None]
                    st = make_step(c, tp, [u[:c.local_len] for u in scratch], res)
                    for _ in range(2):
                        st()
                    sums[(name, R)] = gathered_bits(res[0], device, rehearsal)
                    el, _ = timed_steps(st, 5, stream, world, device, rehearsal)
                    tuned[f"{name}/R{R}"] = el / 5 * 1e3
            del scratch
            torch.cuda.empty_cache()
            # a transport whose gathered model differs from another's (same geometry, same data) or
            # between ranks is not used: every rank computes the same verdict from all-reduced sums
            bad = {}
            for (name, R), (lo, hi) in sums.items():
                ref_sum = sums.get(("collective", R))
                if lo != hi or (ref_sum is not None and ref_sum != (lo, hi)):
                    bad[name] = "gathered model differs between ranks or from the RCCL all-gather's on the same data"
            # a release grid after peer stores that missed an XCD (sharded.P2PAllGather.check_release):
            # the kernel engines' stores may not have been visible — not used (every rank reads its own
            # records, so the verdict is all-reduced: MAX of the miss flag)
            p2p_objs = {id(t): t for t in transports.values() if t is not None}
            if p2p_objs:
                miss = 0
                for t in p2p_objs.values():
                    try:
                        t.check_release()
                    except Exception:  # noqa: BLE001
                        miss = 1
                flag = torch.tensor([miss], dtype=torch.int32, device="cpu" if rehearsal else device)
                if dist.is_initialized():
                    dist.all_reduce(flag, op=dist.ReduceOp.MAX)
                if int(flag[0]):
                    for name in ("p2p_kernel", "p2p_fused"):
                        if name in transports:
                            bad[name] = "a release grid after its peer stores did not cover every XCD"
            if bad:
                extra["transport_disqualified"] = dict(sorted(bad.items()))
                tuned = {k: v for k, v in tuned.items() if k.split("/R")[0] not in bad}
            best = min(tuned, key=tuned.get)
            tname, R = best.split("/R")[0], int(best.split("/R")[1])
        else:
            tname, R = next(iter(transports)), cands[0]
        tp = use(tname)
        for name in list(transports):
            other = transports[name]
            if name != tname and other is not None and other is not tp:
                transports.pop(name).close(check=False)    # its release records were read in the warm-up
        cyc = geoms[R]
        L = cyc.local_len
        P = L
        # the timed data: this rank's chunks of ONE seeded global model (the N = 1 line's), so that
        # rank 0 checks the gathered model bit-for-bit against the oracle
        progress(f"chose {tname} R={R}; generating this rank's chunks of the global model")
        ups_local, host_sample = global_chunks(cyc, K, P_total, a.dtype, device, a.seed, S if rank == 0 else 0)
        agg = agg_all[:L]
        res = [None]
        step = make_step(cyc, tp, ups_local, res)

        fold_round = cyc.round_folder(agg, ups_local, ns, Ns, True, stream)   # the step's own launches

        def fold_only():
            for i in range(cyc.rounds):
                fold_round(i)

        progress("timed steps")
        for _ in range(a.warmup):
            step()
        elapsed, _ = timed_steps(step, a.steps, stream, world, device, rehearsal)
        full = res[0]
        # every rank ends the step holding the same model: int64 sum of its bits, compared over ranks
        lo_bits, hi_bits = gathered_bits(full, device, rehearsal)
        consistent = lo_bits == hi_bits
        if tp is not None:
            # every release grid after the peer stores covered every XCD (warm-up + timed steps)
            extra["release_check"] = side(tp.check_release)
        for _ in range(2):
            fold_only()
        _, kern_ms = timed_steps(fold_only, a.steps, stream, world, device, rehearsal)
        alg_bytes = K * L * in_bytes + L * 4              # this rank's fold, per step (all rounds)
        workload = f"fedavg_k{K}_p{L}_r{cyc.rounds}_{a.dtype}_rank_of_{world}"
        kernel = (f"{fold_kernel_label(cyc.C, in_bytes, K)} over this rank's {cyc.rounds} chunks of {cyc.C} params "
                  "(fold-only timing; max over ranks)")
        backend = dist.get_backend() if dist.is_initialized() else None
        transport = {"p2p": f"direct peer copies (P2PAllGather: IPC-mapped, double-buffered peer buffers, one DMA copy "
                            f"stream per peer, one {backend} fence per step)",
                     "p2p_kernel": f"direct peer pushes (P2PAllGather engine 'kernel': IPC-mapped, double-buffered peer "
                                   f"buffers, one fa_push kernel per round storing into every peer, one {backend} fence "
                                   "per step)",
                     "p2p_fused": f"fold + push fused (P2PAllGather engine 'fused': each round's fold kernel, "
                                  f"fa_fedavg_fold_push, stores its result into this rank's and every peer's IPC-mapped, "
                                  f"double-buffered model buffer; one {backend} fence per step)"}.get(tname, f"{backend} all_gather_into_tensor on a communication stream")
        config = {"workload": f"FedAvg {K} clients x {P_total} params {a.dtype}, param-sharded block-cyclically over "
                              f"{world} GPUs; each folded round gathered to every GPU while the next round folds, "
                              "inside the timed step (BASELINE configs[2])",
                  "clients": K, "params_per_gpu": L, "global_params": P_total, "rounds": cyc.rounds,
                  "chunk": cyc.C, "parallelism": f"param-slice x{world} + all-gather ({tname})",
                  "transport": transport, "tuned_ms": tuned or None}
        scaling = "strong"
        extra["fold_allgather_ms"] = elapsed / a.steps * 1e3
        extra["allgather_consistent_over_ranks"] = consistent
        if rank == 0 and S:
            progress("oracle check of the gathered model's sample")
            exact, dt = sample_check(full, host_sample, ns)
            base = {"value": K * S / dt, "unit": "params/s", "cores": 1, "kind": "port",
                    "sample": f"{K} clients x {S} fp32 params (the first {S} of the global model's clients); numpy "
                              f"{np.__version__} oracle/numpy_ref.fedavg_flat, single-threaded, {os.cpu_count()} host "
                              "cores present", "seconds": dt,
                    "gpu_bit_exact_on_sample": exact,
                    "gpu_sample_source": "rank 0's copy of the all-gathered model"}
        if not a.no_side:
            extra.update(multi_gpu_side(a, world, rank, device, rehearsal, ns, Ns, K, P_total, agg, ups_local, stream,
                                        rccl1, cyc, host_sample))
        if tp is not None:
            tp.close(check=False)          # the release records are already in the line (release_check)
        if rccl1:
            extra["rccl_world1"] = ("rehearsal: the N>1 path at world size 1 over RCCL (all-gathers issued as "
                                    "collectives); not a reported number")
        ups = ups_local

    achieved = alg_bytes / (kern_ms / 1e3) / 1e9
    traffic, tsrc = pmc_traffic(workload)
    if world == 1 and not rccl1:
        # the model to the host, FEDn's consumer (roundhandler.py:465-468); value excludes it
        host = torch.empty(P, dtype=torch.float32, pin_memory=True)
        for _ in range(2):
            host.copy_(agg, non_blocking=True)
        torch.cuda.synchronize(device)
        t1 = time.perf_counter()
        for _ in range(5):
            host.copy_(agg, non_blocking=True)
        torch.cuda.synchronize(device)
        gh = (time.perf_counter() - t1) / 5
        extra["gather_to_host"] = {"ms": gh * 1e3, "bytes_per_rank": P * 4, "GBps_aggregate": P * 4 / gh / 1e9,
                                   "note": "D2H of the aggregate into pinned host memory; not in value"}
        del host
        if a.achievable and not a.no_side and a.dtype == "f32" and K <= 64:
            extra["access_pattern"] = side(lambda: fedavg_pattern(ups, agg, stream, device, alg_bytes, kern_ms, a))
        if K >= 8 and a.configs1:
            extra["configs1"] = side(lambda: configs1_side(ups[:8], ns[:8], agg, stream, device, in_bytes, a))
        del ups, agg
        torch.cuda.empty_cache()
        if a.achievable and not a.no_side:
            extra["achievable"] = side(lambda: achievable_side(device, achieved_of(alg_bytes, kern_ms)))
        if rank == 0 and a.host_clients > 0 and not a.no_side:
            extra["host_resident"] = side(lambda: host_resident_side(a, [device], ns, clients=a.host_clients))
        if rank == 0 and a.waves_params > 0 and not a.no_side:
            extra["fedopt_waves"] = side(lambda: fedopt_waves_side(a, [device]))
        if rank == 0 and a.fedopt_params > 0:
            extra["fedopt"] = side(lambda: fedopt_side(a.fedopt_params, a.fedopt_clients, device,
                                                       pattern_probe=not a.no_side))
        if rank == 0 and not a.no_side:
            extra["configs0"] = side(lambda: configs0_side(device))

    if rank == 0:
        line = {
            "metric": METRIC, "value": K * P_total / (elapsed / a.steps), "unit": "params/s",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": a.dtype,
            "data": "synthetic: base~N(0,1), client=base+0.01*N(0,1), num_examples~U{1..5000}, device-resident",
            "config": config,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": tsrc,
                         "kernel": kernel, "kernel_ms": kern_ms, "alg_bytes_per_launch": alg_bytes},
            "cpu_baseline": base,
            # the north star's "absolute GB/s and fraction of the HBM roofline" for the whole job: the
            # algorithmic bytes of the 64-client fold over the GLOBAL model (K*P*s_in + P*4) per wall
            # step, against N GPUs' peak (at N > 1 the step includes the all-gather)
            "throughput": {"GBps": (K * P_total * in_bytes + P_total * 4) / (elapsed / a.steps) / 1e9,
                           "peak_GBps": HBM_PEAK_GBS * world,
                           "frac": (K * P_total * in_bytes + P_total * 4) / (elapsed / a.steps) / 1e9
                           / (HBM_PEAK_GBS * world),
                           "note": "whole job, wall time of a step (fold + gather at N > 1) vs N x 8 TB/s"},
        }
        line.update(extra)
        print(json.dumps(line), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def multi_gpu_side(a, world, rank, device, rehearsal, ns, Ns, K, P_total, agg, ups_local, stream, rccl1=False,
                   cyc=None, host_sample=None):
    """The N > 1 measurements beside the line (none of them is in value)."""
    from fedn_amd import ops
    from fedn_amd.sharded import ShardedFedAvg
    out = {}
    on_cpu = rehearsal

    def plain_allgather():
        sh = ShardedFedAvg(P_total, collective_at_world1=rccl1)
        src = torch.zeros(sh.hi - sh.lo, dtype=torch.float32, device=device)
        gsrc = src.cpu() if rehearsal else src
        for _ in range(2):
            sh.allgather(gsrc)
        el, _ = timed_steps(lambda: sh.allgather(gsrc), 5, stream, world, device, on_cpu)
        nbytes = sh.shard * world * 4
        ag_s = el / 5
        return {"ms": ag_s * 1e3, "bytes_in_per_rank": sh.shard * (world - 1) * 4,
                "algbw_GBps": nbytes / ag_s / 1e9, "busbw_GBps": nbytes * (world - 1) / world / ag_s / 1e9,
                "backend": "gloo (rehearsal)" if rehearsal else "rccl",
                "note": f"all-gather of the {P_total}-param fp32 model (one slice per rank), not overlapped; not in value"}

    def gather_to_host():
        """FEDn's consumer (roundhandler.py:465-468) without a device collective: every rank D2H's its
        folded chunks over its own PCIe link straight into the node's ONE shared, page-locked host
        model (CyclicShardedFedAvg.gather_to_host -> sharded.HostGather); rank 0 checks it."""
        fold = lambda: [ops.fedavg_fold(agg[i * cyc.C:(i + 1) * cyc.C],  # noqa: E731
                                        [u[i * cyc.C:(i + 1) * cyc.C] for u in ups_local], ns, Ns, init=True,
                                        stream=stream) for i in range(cyc.rounds)]
        fold()
        got = cyc.gather_to_host(agg)                      # maps + pins the shared host model once
        el, _ = timed_steps(lambda: cyc.gather_to_host(agg), 5, stream, world, device, on_cpu)
        gh = el / 5
        res = {"ms": gh * 1e3, "bytes_per_rank": cyc.local_len * 4, "GBps_aggregate": P_total * 4 / gh / 1e9,
               "path": "sharded.CyclicShardedFedAvg.gather_to_host -> HostGather (shared /dev/shm model, "
                       "fa_host_register, one fa_copy_async per chunk per rank, barrier)",
               "note": "every rank D2H's its chunks into one pinned host model shared by the ranks, all links at "
                       "once; max over ranks; not in value"}
        if rank == 0 and host_sample:
            res["bit_exact_on_sample"] = sample_check(got, host_sample, ns)[0]
        cyc._host_gather.close()
        return res

    def weak():
        # a rehearsal puts every rank on one GPU: each folds a 1/world slice there, so the ranks'
        # updates together take the N = 1 line's HBM, not world times it
        P = -(-P_total // world) if rehearsal else P_total
        ups = make_updates(K, P, a.dtype, device, a.seed + 7 + 1000 * rank)
        agg_w = torch.empty(P, dtype=torch.float32, device=device)
        step = lambda: ops.fedavg_fold(agg_w, ups, ns, Ns, init=True, stream=stream)  # noqa: E731
        for _ in range(2):
            step()
        el, kms = timed_steps(step, a.steps, stream, world, device, on_cpu)
        del ups, agg_w
        torch.cuda.empty_cache()
        return {"value": K * P * world / (el / a.steps), "ms_per_step": el / a.steps * 1e3, "kernel_ms": kms,
                "params_per_gpu": P, "global_params": P * world,
                "note": f"every rank folds its own {P}-param slice of a world x {P} model; no collective; not in value"
                        + ("; REHEARSAL: all ranks on one GPU, each folding a 1/world slice" if rehearsal else "")}

    def in_process():
        """One process (rank 0) drives all N GPUs: each folds its slice of the 64 updates and copies it
        into one pinned host model (the multidev.py layout FEDN_AMD_DEVICES selects)."""
        from fedn_amd.sharded import shard_bounds
        res = None
        if True:
            devs = [torch.device("cuda", 0 if rehearsal else d) for d in range(world)]
            bounds = shard_bounds(P_total, world)
            data = []
            for d, dv in enumerate(devs):
                lo, hi = bounds[d]
                with torch.cuda.device(dv):
                    u = make_updates(K, hi - lo, a.dtype, dv, a.seed + 31 + d)
                    data.append((u, torch.empty(hi - lo, dtype=torch.float32, device=dv)))
            host = torch.empty(P_total, dtype=torch.float32, pin_memory=True)

            def run():
                for d, dv in enumerate(devs):
                    lo, hi = bounds[d]
                    u, ag = data[d]
                    with torch.cuda.device(dv):
                        ops.fedavg_fold(ag, u, ns, Ns, init=True, stream=torch.cuda.current_stream(dv))
                        host[lo:hi].copy_(ag, non_blocking=True)
                for dv in devs:
                    torch.cuda.synchronize(dv)
            run()
            t0 = time.perf_counter()
            for _ in range(5):
                run()
            t = (time.perf_counter() - t0) / 5
            res = {"ms": t * 1e3, "value": K * P_total / t, "devices": len(devs),
                   "note": f"one process, all GPUs: each folds its slice of the {K} device-resident updates and "
                           "D2H's it into one pinned host model (fold + PCIe copy, no collective); not in value"}
            del data, host
            torch.cuda.empty_cache()
        return res

    progress("side: allgather, gather_to_host, weak_scaling")
    out["allgather"] = side(plain_allgather)
    out["gather_to_host"] = side(gather_to_host)
    out["weak_scaling"] = side(weak)
    def fedopt_waves():
        return fedopt_waves_side(a, [torch.device("cuda", 0 if rehearsal else d) for d in range(world)])

    def fedopt_sharded():
        """BASELINE configs[3] on N GPUs: the same FedAdam model (P params, K fp32 updates) sliced over
        the ranks (sharded.ShardedFedOpt's bounds); each rank keeps its slices of the updates, old, m
        and v resident and runs the fused steady-state step on them — no collective (FedOpt state
        never moves); then each rank D2H's its fp64 slice of the new model (FEDn's consumer)."""
        from fedn_amd.sharded import shard_bounds
        P, Kf = a.fedopt_params, a.fedopt_clients
        lo, hi = shard_bounds(P, world)[rank]
        n = hi - lo
        g = torch.Generator(device=device).manual_seed(4 + rank)
        old32 = torch.randn(n, generator=g, device=device)
        fups = [torch.randn(n, generator=g, device=device).mul_(0.01).add_(old32) for _ in range(Kf)]
        fns = [int(v) for v in np.random.default_rng(4).integers(1, 5001, Kf)]
        fNs = [int(v) for v in np.cumsum(fns)]
        out1 = torch.empty(n, dtype=torch.float64, device=device)
        v1 = torch.empty(n, dtype=torch.float64, device=device)
        m1 = torch.empty(n, dtype=torch.float32, device=device)
        ops.fedopt_step(old32, fups, fns, fNs, first=True, final=True, m_out=m1, v_out=v1, out=out1, stream=stream)
        old64, m64 = out1, m1.double()
        del old32, m1
        m_o = torch.empty(n, dtype=torch.float64, device=device)
        v_o = torch.empty(n, dtype=torch.float64, device=device)
        o2 = torch.empty(n, dtype=torch.float64, device=device)
        step = lambda: ops.fedopt_step(old64, fups, fns, fNs, first=True, final=True, m_in=m64, m_out=m_o,  # noqa: E731
                                       v_in=v1, v_out=v_o, out=o2, stream=stream)
        for _ in range(2):
            step()
        el, kms = timed_steps(step, 10, stream, world, device, on_cpu)
        host = torch.empty(n, dtype=torch.float64, pin_memory=True)
        host.copy_(o2, non_blocking=True)
        elh, _ = timed_steps(lambda: host.copy_(o2, non_blocking=True), 5, stream, world, device, on_cpu)
        t = el / 10
        b = n * (4 * Kf + 48)
        del fups, old64, m64, v1, m_o, v_o, o2, out1, host
        torch.cuda.empty_cache()
        return {"ms": t * 1e3, "value": Kf * P / t, "unit": "params/s", "params": P, "clients": Kf,
                "params_per_gpu": n, "kernel_ms": kms, "frac_per_rank": b / (kms / 1e3) / 1e9 / HBM_PEAK_GBS,
                "gather_to_host_ms": elh / 5 * 1e3,
                "note": "BASELINE configs[3] at N GPUs (strong: the same model sliced): FedAdam steady state, "
                        "fp64 old / m / v resident per slice, one fused launch per rank, max over ranks; the "
                        "fp64 model slice's D2H is timed apart; not in value"}

    if a.fedopt_params > 0:
        progress("side: fedopt_sharded")
        out["fedopt_sharded"] = side(fedopt_sharded)
    devs = [torch.device("cuda", 0 if rehearsal else d) for d in range(world)]
    progress("side (rank 0): in_process, host_resident, fedopt_waves")
    ip = side(in_process) if rank == 0 else None     # the other ranks wait (their GPUs are in use)
    hr = (side(lambda: host_resident_side(a, devs, ns, clients=a.host_clients))
          if rank == 0 and a.host_clients > 0 else None)
    fw = side(fedopt_waves) if rank == 0 and a.waves_params > 0 else None
    dist.barrier()
    if rank == 0:
        out["in_process"] = ip
        if hr is not None:
            out["host_resident"] = hr
        if fw is not None:
            out["fedopt_waves"] = fw
    return out


if __name__ == "__main__":
    main()
