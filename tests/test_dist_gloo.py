"""N>1 path on CPU: world_size-2 (and 3) gloo ranks shard a FedAvg by parameter slice,
fold their slices, and reassemble by all-gather / gather; the result must be bit-identical
to the single-process oracle (elementwise independence makes sharding exact).
The per-slice fold here is the oracle (test infrastructure) — the GPU runs libfedagg."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fedn_amd.sharded import ALIGN_ELEMS, ShardedFedAvg, shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_fold(agg, updates, n, N, init):
    from oracle import numpy_ref as ref
    ups = [u.numpy() for u in updates]
    if init:
        out = ref.fedavg_flat(ups, n)    # N recomputed from n in order: same totals
    else:
        raise NotImplementedError
    agg.copy_(torch.from_numpy(out))
    return agg


def _worker(rank, world, port, P, K, seed, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(seed)
        base = rng.standard_normal(P).astype(np.float32)
        ups = [torch.from_numpy((base + 0.01 * rng.standard_normal(P)).astype(np.float32)) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5001, K)]
        Ns = list(np.cumsum(ns))
        sh = ShardedFedAvg(P, fold_fn=_oracle_fold)
        agg = torch.empty(sh.hi - sh.lo, dtype=torch.float32)
        sh.fold(agg, [sh.local(u) for u in ups], ns, Ns, init=True)
        full = sh.allgather(agg)
        host = sh.gather_to_host(agg, dst=0)
        if rank == 0:
            q.put((full.numpy().copy(), host.numpy().copy(), sh.bounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P", [(2, 10_000), (2, 4096), (3, 5_003), (4, 20_011), (8, 70_001)])
def test_sharded_fedavg_gloo(world, P):
    from oracle import numpy_ref as ref
    K, seed = 5, 17
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    pc = mp.start_processes(_worker, args=(world, port, P, K, seed, q), nprocs=world, join=False,
                            start_method="spawn")
    full, host, bounds = q.get(timeout=120)   # drain before joining (queue feeder would block exit)
    while not pc.join(timeout=60):
        pass
    rng = np.random.default_rng(seed)
    base = rng.standard_normal(P).astype(np.float32)
    ups = [(base + 0.01 * rng.standard_normal(P)).astype(np.float32) for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    want = ref.fedavg_flat(ups, ns)
    assert np.array_equal(full.view(np.uint32), want.view(np.uint32))
    assert np.array_equal(host.view(np.uint32), want.view(np.uint32))
    assert bounds[0][0] == 0 and bounds[-1][1] == P


def test_shard_bounds_cover_and_align():
    for P in (1, 1023, 1024, 100_000_000, 12_345_679):
        for n in (1, 2, 4, 8):
            b = shard_bounds(P, n)
            assert b[0][0] == 0 and b[-1][1] == P
            for (lo, hi), (lo2, _) in zip(b, b[1:]):
                assert hi == lo2 and (lo % ALIGN_ELEMS == 0 or lo == P) and (lo2 % ALIGN_ELEMS == 0 or lo2 == P)
            assert all(lo <= hi for lo, hi in b)


def _oracle_fedopt_step(old, updates, n, N, m_in, v_in, params):
    from oracle import numpy_ref as ref
    st = ref.FedOptState()
    st.m = None if m_in is None else [m_in.numpy()]
    st.v = None if v_in is None else [v_in.numpy()]
    out, _ = ref.fedopt_combine(st, [([u.numpy()], k) for u, k in zip(updates, n)], [old.numpy()], params)
    return torch.from_numpy(out[0]), torch.from_numpy(st.m[0]), torch.from_numpy(st.v[0])


def _fedopt_worker(rank, world, port, P, K, seed, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from fedn_amd.sharded import ShardedFedOpt
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(seed)
        old = rng.standard_normal(P).astype(np.float32)
        sh = ShardedFedOpt(P, step_fn=_oracle_fedopt_step)
        params = {"serveropt": "yogi"}
        outs = []
        for r in range(2):
            ups = [torch.from_numpy((old + 0.01 * rng.standard_normal(P)).astype(np.float32)) for _ in range(K)]
            ns = [int(v) for v in rng.integers(1, 5001, K)]
            out = sh.step(sh.local(torch.from_numpy(old)), [sh.local(u) for u in ups], ns, list(np.cumsum(ns)), params)
            full = sh.allgather(out).numpy().copy()
            outs.append(full)
            old = full
        if rank == 0:
            q.put(outs)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P", [(2, 6000), (8, 40_003)])
def test_sharded_fedopt_gloo_two_rounds(world, P):
    """FedOpt state (m, v) stays sharded across rounds; gathered models == single-process oracle."""
    from oracle import numpy_ref as ref
    K, seed = 4, 23
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_fedopt_worker, args=(world, _free_port(), P, K, seed, q), nprocs=world, join=False,
                            start_method="spawn")
    outs = q.get(timeout=120)
    while not pc.join(timeout=60):
        pass
    rng = np.random.default_rng(seed)
    old = rng.standard_normal(P).astype(np.float32)
    st = ref.FedOptState()
    for r in range(2):
        ups = [(old + 0.01 * rng.standard_normal(P)).astype(np.float32) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5001, K)]
        want, _ = ref.fedopt_combine(st, [([u], k) for u, k in zip(ups, ns)], [old], {"serveropt": "yogi"})
        assert outs[r].dtype == want[0].dtype
        assert np.array_equal(outs[r].view(np.uint64), want[0].view(np.uint64)), f"round {r}"
        old = want[0]


def _cyclic_worker(rank, world, port, P, K, chunk, seed, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from fedn_amd.sharded import CyclicShardedFedAvg
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(seed)
        base = rng.standard_normal(P).astype(np.float32)
        ups = [torch.from_numpy((base + 0.01 * rng.standard_normal(P)).astype(np.float32)) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5001, K)]
        cs = CyclicShardedFedAvg(P, chunk=chunk, fold_fn=_oracle_fold)
        agg = torch.empty(cs.local_len, dtype=torch.float32)
        full = cs.fold_allgather(agg, [cs.local(u) for u in ups], ns, list(np.cumsum(ns)), init=True)
        q.put((rank, full.numpy().copy(), cs.owned(), cs.rounds))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,P,chunk", [(2, 10_000, 1024), (3, 5_003, 1024), (2, 3_000, 4096), (3, 9_216, 1024),
                                             (4, 40_001, 2_500), (8, 100_003, 1_571), (8, 2_000, 1_024)])
def test_cyclic_fold_allgather_gloo(world, P, chunk):
    """Block-cyclic shards, per-round fold + all-gather straight into natural order: every
    rank ends with the full model, bit-identical to the single-process oracle. World 4 / 8 are
    the N = 4 / 8 geometries of bench.py --gpus N (ragged last chunk; at (8, 2000, 1024) some
    ranks own nothing)."""
    from oracle import numpy_ref as ref
    K, seed = 4, 29
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_cyclic_worker, args=(world, _free_port(), P, K, chunk, seed, q), nprocs=world,
                            join=False, start_method="spawn")
    res = sorted(q.get(timeout=120) for _ in range(world))
    while not pc.join(timeout=60):
        pass
    rng = np.random.default_rng(seed)
    base = rng.standard_normal(P).astype(np.float32)
    ups = [(base + 0.01 * rng.standard_normal(P)).astype(np.float32) for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    want = ref.fedavg_flat(ups, ns)
    covered = []
    for rank, full, owned, rounds in res:
        assert full.shape == (P,)
        assert np.array_equal(full.view(np.uint32), want.view(np.uint32)), f"rank {rank}"
        covered += [(lo, hi) for lo, hi, _ in owned]
    covered.sort()
    assert covered[0][0] == 0 and covered[-1][1] == P
    assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


def _world1_worker(rank, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from fedn_amd.sharded import CyclicShardedFedAvg
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        rng = np.random.default_rng(23)
        P, K = 9_001, 4
        base = rng.standard_normal(P).astype(np.float32)
        ups = [torch.from_numpy((base + 0.01 * rng.standard_normal(P)).astype(np.float32)) for _ in range(K)]
        ns = [int(v) for v in rng.integers(1, 5001, K)]
        off = CyclicShardedFedAvg(P, chunk=2048, fold_fn=_oracle_fold)
        on = CyclicShardedFedAvg(P, chunk=2048, fold_fn=_oracle_fold, collective_at_world1=True)
        sh = ShardedFedAvg(P, collective_at_world1=True)
        res = []
        for cs in (off, on):
            agg = torch.empty(cs.local_len, dtype=torch.float32)
            res.append(cs.fold_allgather(agg, [cs.local(u) for u in ups], ns, list(np.cumsum(ns)), init=True).numpy())
        q.put((off.collective, on.collective, sh.collective, res[0].copy(), res[1].copy(),
               sh.allgather(torch.from_numpy(res[0])).numpy().copy(), [u.numpy() for u in ups], ns))
    finally:
        dist.destroy_process_group()


def test_collective_at_world1_gloo():
    """collective_at_world1 (the one-GPU rehearsal of the RCCL calls, tests/test_gpu_rccl.py): at
    world size 1 the all-gathers are issued as collectives and give what the local copy gives."""
    from oracle import numpy_ref as ref
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_world1_worker, args=(_free_port(), q), nprocs=1, join=False, start_method="spawn")
    off_c, on_c, sh_c, r_off, r_on, r_sh, ups, ns = q.get(timeout=120)
    while not pc.join(timeout=60):
        pass
    assert (off_c, on_c, sh_c) == (False, True, True)
    want = ref.fedavg_flat(ups, ns)
    for got in (r_off, r_on, r_sh):
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


def _hostgather_worker(rank, world, port, P, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fedn_amd.sharded import HostGather
        sh = ShardedFedAvg(P, fold_fn=lambda *a: None)
        out = []
        for step, dt in enumerate((torch.float32, torch.float32, torch.float64, torch.float32)):
            full = torch.arange(P, dtype=dt) * (step + 1)
            got = sh.gather_to_host(sh.local(full).clone(), dst=0)     # cached per (dst, dtype)
            if rank == 0:
                out.append((str(dt), np.array_equal(got.numpy(), full.numpy()), got.dtype == dt))
            else:
                out.append(got is None)
        hg = HostGather(P, torch.float32, sh.bounds)
        try:
            hg.gather(torch.zeros(sh.hi - sh.lo, dtype=torch.float64))
            out.append("no error")
        except TypeError:
            out.append("TypeError")
        dist.barrier()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_host_gather_dtype_cache_and_entry_barrier():
    """the shared host model is cached per (destination rank, dtype) — a float64 gather after
    float32 ones gets its own buffer, and the float32 one after it is right again — and a slice of the
    wrong dtype raises instead of copying half its bytes; back-to-back gathers (each entered through a
    barrier) return the newest model on rank 0."""
    world, P = 3, 10_007
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_hostgather_worker, args=(world, _free_port(), P, q), nprocs=world, join=False,
                            start_method="spawn")
    res = dict(q.get(timeout=120) for _ in range(world))
    while not pc.join(timeout=60):
        pass
    for dt, same, dtype_ok in res[0][:4]:
        assert same and dtype_ok, dt
    for r in (1, 2):
        assert res[r][:4] == [True] * 4
    assert all(res[r][4] == "TypeError" for r in range(world))


def _one_rank_fails_worker(rank, world, port, P, q):
    """Rank 1 alone fails: its HostGather copy (a piece outside its buffer), its P2PAllGather buffer
    export, then its peer mapping. Every rank must raise at the same point — none left waiting in a
    collective — and the process group must still work afterwards."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fedn_amd import ops, sharded
        from fedn_amd.sharded import HostGather, P2PAllGather
        out = []
        sh = ShardedFedAvg(P, fold_fn=lambda *a: None)
        hg = HostGather(P, torch.float32, sh.bounds)
        local = torch.ones(sh.hi - sh.lo, dtype=torch.float32)
        pieces = [(sh.lo, sh.hi, 5)] if rank == 1 else None        # rank 1: past the end of its slice
        try:
            hg.gather(local, pieces)
            out.append("no error")
        except (ValueError, RuntimeError) as e:
            out.append(type(e).__name__)
        got = hg.gather(local)                                       # the next gather works again
        out.append(bool(rank != 0 or float(got.sum()) == float(P)))

        def handle(t):
            if rank == 1:
                raise OSError("no IPC export here")
            return b"\0" * 64, 0
        ops.ipc_handle, real_handle = handle, ops.ipc_handle
        buf = torch.zeros(8)
        try:
            P2PAllGather(buf)
            out.append("no error")
        except RuntimeError as e:
            out.append("export" if "rank 1 could not export" in str(e) else str(e))
        ops.ipc_handle = lambda t: (b"\0" * 64, 0)

        def ipc_open(h, o, dev):
            if rank == 1:
                raise OSError("no peer mapping here")
            return 4096, 4096
        closed = []
        ops.ipc_open, ops.ipc_close = ipc_open, lambda base, dev=None: closed.append(base)
        try:
            P2PAllGather(buf)
            out.append("no error")
        except (OSError, RuntimeError) as e:
            out.append(type(e).__name__)
        out.append(len(closed))                                      # rank 0 unmapped what it had mapped
        ops.ipc_handle = real_handle
        out.append(sharded._agree(False))
        dist.barrier()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_one_rank_failure_fails_every_rank_without_a_hang():
    """A HostGather copy, a P2P buffer export and a P2P peer mapping that fail on ONE rank raise on
    every rank (the failing rank its own error, the others RuntimeError) — bench.py then falls back to
    the collective on all ranks together instead of hanging in mismatched collectives."""
    world, P = 3, 10_007
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pc = mp.start_processes(_one_rank_fails_worker, args=(world, _free_port(), P, q), nprocs=world, join=False,
                            start_method="spawn")
    res = dict(q.get(timeout=120) for _ in range(world))
    while not pc.join(timeout=60):
        pass
    assert res[1] == ["ValueError", True, "export", "OSError", 0, False]
    assert res[0] == ["RuntimeError", True, "export", "RuntimeError", 2, False]
    assert res[2] == ["RuntimeError", True, "export", "RuntimeError", 2, False]
