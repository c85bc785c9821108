"""The RCCL calls of the N>1 path on the one-GPU box: a world-size-1 "nccl" process group (RCCL
on ROCm) in a child process, with the sharding classes told to issue their all-gathers as
collectives even at world size 1 (``collective_at_world1``). Two ranks cannot share one GPU
under RCCL, so this is how the communicator set-up, ``all_gather_into_tensor`` on the
communication stream and the stream hand-offs of ``CyclicShardedFedAvg.fold_allgather`` run on
real hardware before the driver's 8-GPU run. Results are checked against the oracle."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, {root!r})
    from oracle import numpy_ref as ref
    from fedn_amd.sharded import CyclicShardedFedAvg, ShardedFedAvg

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    rng = np.random.default_rng(7)
    P, K = 3_000_017, 9
    base = rng.standard_normal(P).astype(np.float32)
    ups = [(base + 0.01 * rng.standard_normal(P)).astype(np.float32) for _ in range(K)]
    ns = [int(v) for v in rng.integers(1, 5001, K)]
    want = ref.fedavg_flat(ups, ns)
    cs = CyclicShardedFedAvg(P, chunk=400_000, collective_at_world1=True)
    assert cs.collective and cs.rounds == 8
    dev_ups = [cs.local(torch.from_numpy(u).to(dev)) for u in ups]
    agg = torch.empty(cs.local_len, device=dev)
    for step in range(3):                               # the comm stream is reused across steps
        full = cs.fold_allgather(agg, dev_ups, ns, list(np.cumsum(ns)), init=True)
        torch.cuda.synchronize()
        got = full.cpu().numpy()
        assert got.view(np.uint32).tobytes() == want.view(np.uint32).tobytes(), f"step {{step}}"
    sh = ShardedFedAvg(P, collective_at_world1=True)
    assert sh.collective
    part = torch.from_numpy(want).to(dev)
    g = sh.allgather(part)
    assert torch.equal(g.cpu(), torch.from_numpy(want))
    t = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    dist.destroy_process_group()
    print("RCCL_WORLD1_OK", flush=True)
""")


def test_rccl_world1_fold_allgather():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29561", RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "RCCL_WORLD1_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
