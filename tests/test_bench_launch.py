"""bench.py's own rank launcher (no torch.distributed.run): ``bench.py --gpus N`` with no WORLD_SIZE
in the environment starts N child processes with the contract's environment and waits for them.
CPU-only: ``--launch-check`` runs the rank set-up alone (gloo rendezvous on 127.0.0.1, an
all-reduce, no GPU)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=180, env=env, cwd=ROOT)


def test_self_launch_spawns_ranks_with_gloo():
    r = _run("--gpus", "3", "--launch-check")
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                                   # rank 0 alone prints
    out = json.loads(lines[0])
    assert out["world"] == 3 and out["rank_sum"] == 6
    pids = {p for p, _, _ in out["ranks"]}
    parents = {pp for _, pp, _ in out["ranks"]}
    assert len(pids) == 3 and len(parents) == 1              # three children of one launcher
    assert sorted(lr for _, _, lr in out["ranks"]) == [0, 1, 2]


def test_launched_rank_does_not_relaunch():
    """Under a launcher (WORLD_SIZE set) bench.py is one rank: it must not start children itself."""
    from socket import socket
    s = socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = _run("--gpus", "1", "--launch-check",
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                        "MASTER_PORT": str(port)})
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert out["world"] == 1 and len(out["ranks"]) == 1
    assert out["ranks"][0][1] == os.getpid()                 # the rank is the process started here
