"""The release after peer stores covers every XCD, and says so (include/fedagg.h FA_REL_*).

fa_push / fa_fedavg_fold_push store into other GPUs' memory (sharded.P2PAllGather's kernel and
fused engines); the bytes still in an XCD's L2 must be written back at system scope before the
ranks' fence. HIP promises nothing about which XCDs a grid's workgroups land on, so the release
grid records the XCD each of its workgroups ran on (HW_REG_XCC_ID) and counts every launch that
missed one. These tests read that record on the box's GPU: every launch checked, no miss, the
union of XCDs seen equal to the device's XCD count.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need a HIP device")
    from fedn_amd import _abi
    _abi.load()


def _assert_covered(r, launches):
    from fedn_amd import ops
    nx = ops.device_xccs(DEV)
    assert r["launches"] == launches
    assert r["misses"] == 0
    assert r["expect_mask"] == (1 << nx) - 1
    assert r["seen_mask"] == r["expect_mask"]
    assert r["xcds_seen"] == nx


def test_device_xccs():
    """MI355X in its default single-partition mode: one device of 8 XCDs (gfx950)."""
    from fedn_amd import ops
    nx = ops.device_xccs(DEV)
    props = torch.cuda.get_device_properties(0)
    assert 1 <= nx <= 16
    if "gfx950" in getattr(props, "gcnArchName", "") and props.multi_processor_count == 256:
        assert nx == 8


@pytest.mark.parametrize("launches", [1, 7, 200])
def test_push_release_record(launches):
    """fa_push's release grid: each launch checked, every XCD covered, the bytes still land."""
    from fedn_amd import ops
    st = torch.cuda.current_stream(DEV)
    rec = ops.release_record(DEV)
    src = torch.arange(4096, dtype=torch.int32, device=DEV)
    dsts = [torch.zeros(4096, dtype=torch.int32, device=DEV) for _ in range(3)]
    for _ in range(launches):
        ops.push([d.data_ptr() for d in dsts], src, src.numel() * 4, st, release_rec=rec)
    _assert_covered(ops.read_release_record(rec), launches)
    for d in dsts:
        assert torch.equal(d, src)


def test_fold_push_release_record():
    """fa_fedavg_fold_push: the release runs (and is recorded) only when it stored into peers."""
    from fedn_amd import ops
    P, K = 1 << 20, 9
    g = torch.Generator(device=DEV).manual_seed(3)
    ups = [torch.randn(P, generator=g, device=DEV) for _ in range(K)]
    ns = [int(v) for v in np.random.default_rng(3).integers(1, 5001, K)]
    Ns = [int(v) for v in np.cumsum(ns)]
    want = torch.empty(P, device=DEV)
    ops.fedavg_fold(want, ups, ns, Ns, init=True)
    st = torch.cuda.current_stream(DEV)
    rec = ops.release_record(DEV)
    agg = torch.empty(P, device=DEV)
    peers = [torch.empty(P, device=DEV) for _ in range(2)]
    for _ in range(5):
        ops.fedavg_fold_push(agg.data_ptr(), [u.data_ptr() for u in ups], ns, Ns, P, True,
                             [p.data_ptr() for p in peers], st, DEV, release_rec=rec)
    ops.fedavg_fold_push(agg.data_ptr(), [u.data_ptr() for u in ups], ns, Ns, P, True, [], st, DEV, release_rec=rec)
    _assert_covered(ops.read_release_record(rec), 5)
    for t in [agg] + peers:
        assert torch.equal(t.view(torch.int32), want.view(torch.int32))


def test_release_record_per_stream_concurrent():
    """Two streams, each with its own record, pushing concurrently: both records exact."""
    from fedn_amd import ops
    streams = [torch.cuda.Stream(DEV) for _ in range(2)]
    recs = [ops.release_record(DEV) for _ in streams]
    src = torch.randint(0, 1 << 30, (1 << 18,), dtype=torch.int32, device=DEV)
    dst = [torch.zeros_like(src) for _ in streams]
    torch.cuda.synchronize()
    for _ in range(50):
        for s, r, d in zip(streams, recs, dst):
            ops.push([d.data_ptr()], src, src.numel() * 4, s, release_rec=r)
    for r in recs:
        _assert_covered(ops.read_release_record(r), 50)
    for d in dst:
        assert torch.equal(d, src)


def test_release_record_refused_shapes():
    from fedn_amd import ops
    src = torch.zeros(16, dtype=torch.int32, device=DEV)
    dst = torch.zeros(16, dtype=torch.int32, device=DEV)
    st = torch.cuda.current_stream(DEV)
    with pytest.raises(ValueError, match="release record"):
        ops.push([dst.data_ptr()], src, 64, st, release_rec=torch.zeros(8, dtype=torch.int64, device=DEV))
    with pytest.raises(ValueError, match="release record"):
        ops.push([dst.data_ptr()], src, 64, st, release_rec=torch.zeros(4, dtype=torch.int32, device=DEV))
    with pytest.raises(ValueError, match="release record"):
        ops.push([dst.data_ptr()], src, 64, st, release_rec=torch.zeros(8, dtype=torch.int32))


@pytest.mark.parametrize("engine", ["kernel", "fused"])
def test_p2p_allgather_check_release_world1(engine):
    """P2PAllGather at world size 1 (no peers; both engines still store this rank's own copy as a
    destination and release): check_release reports every launch covered; close() checks it too;
    agg_local holds the folded chunks (what gather_to_host copies)."""
    from fedn_amd.sharded import CyclicShardedFedAvg, P2PAllGather
    P, K = 300_000, 4
    cyc = CyclicShardedFedAvg(P, chunk=65536)
    g = torch.Generator(device=DEV).manual_seed(11)
    ups = [torch.randn(cyc.local_len, generator=g, device=DEV) for _ in range(K)]
    ns = [3, 5, 7, 11]
    Ns = [int(v) for v in np.cumsum(ns)]
    full = torch.empty(cyc.full_len, device=DEV)
    p2p = P2PAllGather(full, spare=torch.empty_like(full), engine=engine)
    agg = torch.empty(cyc.local_len, device=DEV)
    for _ in range(3):
        out = cyc.fold_allgather(agg, ups, ns, Ns, True, p2p=p2p)
    want = torch.empty(cyc.local_len, device=DEV)
    from fedn_amd import ops
    ops.fedavg_fold(want, ups, ns, Ns, init=True)
    assert torch.equal(out.view(torch.int32), want[:P].view(torch.int32))
    assert torch.equal(agg.view(torch.int32), want.view(torch.int32))
    # both engines store this rank's copy of the model as a push destination (the fused fold keeps its
    # running aggregate in agg_local), so every round's launch releases and is recorded
    r = p2p.check_release()
    assert r["launches"] == 3 * cyc.rounds and r["misses"] == 0 and r["xcds_seen"] == r["xcds"]
    p2p.close()


def test_p2p_allgather_checks_every_round_and_fails_the_round_on_a_miss():
    """a session that keeps its P2PAllGather across rounds has each round's release
    records read at that round's fence (verify="round", the default) — not only at close(). A miss
    injected into the record after round 2 fails round 3's exchange right there; with
    verify="close" (bench.py's timed steps) it surfaces at close()."""
    from fedn_amd import _abi
    from fedn_amd.sharded import CyclicShardedFedAvg, P2PAllGather
    P, K = 200_000, 3
    cyc = CyclicShardedFedAvg(P, chunk=65536)
    g = torch.Generator(device=DEV).manual_seed(5)
    ups = [torch.randn(cyc.local_len, generator=g, device=DEV) for _ in range(K)]
    ns, Ns = [2, 3, 4], [2, 5, 9]
    agg = torch.empty(cyc.local_len, device=DEV)
    for verify in ("round", "close"):
        full = torch.empty(cyc.full_len, device=DEV)
        p2p = P2PAllGather(full, spare=torch.empty_like(full), engine="kernel", verify=verify)
        for _ in range(2):
            cyc.fold_allgather(agg, ups, ns, Ns, True, p2p=p2p)
        rec = next(iter(p2p._release.values()))
        rec[_abi.FA_REL_MISSES] += 1                      # a release grid that missed an XCD
        if verify == "round":
            with pytest.raises(_abi.FedAggError, match="did not cover every XCD"):
                cyc.fold_allgather(agg, ups, ns, Ns, True, p2p=p2p)
            p2p.close(check=False)
        else:
            cyc.fold_allgather(agg, ups, ns, Ns, True, p2p=p2p)    # not read until close()
            with pytest.raises(_abi.FedAggError, match="did not cover every XCD"):
                p2p.close()


def test_p2p_allgather_release_count_must_match_launches():
    """A release grid that never ran (or a record reset under it) is a failure too: the records'
    launch count must equal the release grids issued."""
    from fedn_amd import _abi
    from fedn_amd.sharded import CyclicShardedFedAvg, P2PAllGather
    cyc = CyclicShardedFedAvg(100_000, chunk=65536)
    ups = [torch.ones(cyc.local_len, device=DEV)]
    full = torch.empty(cyc.full_len, device=DEV)
    p2p = P2PAllGather(full, engine="kernel", verify="close")
    agg = torch.empty(cyc.local_len, device=DEV)
    cyc.fold_allgather(agg, ups, [1], [1], True, p2p=p2p)
    torch.cuda.synchronize()
    next(iter(p2p._release.values()))[_abi.FA_REL_LAUNCHES] -= 1
    with pytest.raises(_abi.FedAggError, match="release grids recorded"):
        p2p.check_release()
    p2p.close(check=False)


def test_p2p_push_that_stores_nothing_or_fails_leaves_the_count_right():
    """a release is counted only once the ops call succeeded AND launched one. A push of 0
    bytes (fa_push returns before any release grid) and a push refused by its checks (unaligned
    source: FA_EINVAL before launching) must not make every later fence raise 'a release did not run'."""
    from fedn_amd import _abi
    from fedn_amd.sharded import CyclicShardedFedAvg, P2PAllGather
    cyc = CyclicShardedFedAvg(100_000, chunk=65536)
    ups = [torch.ones(cyc.local_len, device=DEV)]
    full = torch.empty(cyc.full_len, device=DEV)
    p2p = P2PAllGather(full, engine="kernel", verify="round")
    agg = torch.empty(cyc.local_len, device=DEV)
    cyc.fold_allgather(agg, ups, [1], [1], True, p2p=p2p)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(DEV))
    src = torch.ones(64, device=DEV)
    p2p.push(0, src[:0], ev, local=True)              # nothing to store: no release grid
    with pytest.raises(_abi.FedAggError):
        p2p.push(0, src[1:5], ev, local=True)         # 4-B offset source: refused before any launch
    cyc.fold_allgather(agg, ups, [1], [1], True, p2p=p2p)   # the next round's fence checks the counts
    r = p2p.check_release()
    assert r["launches"] == 2 * cyc.rounds and r["misses"] == 0
    p2p.close()
