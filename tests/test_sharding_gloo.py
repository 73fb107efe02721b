"""Multi-rank (world_size 2, gloo on CPU) coverage of the matrix-sharded decomposition:
round-robin assignment, packing, and the gather of packed results to rank 0.  The MI355X
engine is replaced by a deterministic CPU stub here; on the GPU box the same code runs with
the HIP engine and the "nccl" (RCCL) backend."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ee274_convexcaldera_llm_quantization_amd import sharding as S


def _stub(batch_items):
    out = []
    for name, m, n, seed in batch_items:
        g = torch.Generator().manual_seed(seed)
        r = 3
        codes = torch.randint(0, 256, (m * n // 4,), generator=g, dtype=torch.uint8)
        L = torch.randn(m, r, generator=g)
        R = torch.randn(r, n, generator=g)
        out.append(S.MatrixResult(name, m, n, r, 2, codes, 1.5 + seed, L, R, 0.02,
                                  {"Q": [0.9, 0.8], "LR": [0.7, 0.6]}))
    return out


def _items():
    shapes = ((8, 16), (8, 16), (8, 16), (8, 16), (24, 16), (24, 16), (16, 24))
    return [(f"model.layers.{l}.p{i}", m, n, l * 7 + i) for l in range(5) for i, (m, n) in enumerate(shapes)]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = S.decompose_sharded(_items(), _stub, rank=rank, world=world, max_batch=2)
        if rank == 0:
            # plain numpy through the queue (tensors would be shared by fd and die with the child)
            q.put([(r.name, r.codes.numpy().copy(), r.L.numpy().copy(), r.R.numpy().copy(), r.Q_scale,
                    r.errors) for r in res])
        else:
            q.put(res)
    finally:
        dist.destroy_process_group()


class _RunAllStub:
    """decompose_batch with the interface of the engine's (sharding.engine_decompose_batch):
    run_all(batches, on_batch_done) -- batches finishing out of order, as interleaved HIP
    streams let them -- and blob_bound(m, n), which enables the overlapped gather."""

    def __call__(self, batch_items):
        return _stub(batch_items)

    def run_all(self, batches, on_batch_done=None):
        res = [_stub(b) for b in batches]
        for j in reversed(range(len(batches))):  # the last batch finishes first
            if on_batch_done is not None:
                on_batch_done(j, res[j])
        return [r for b in res for r in b]

    @staticmethod
    def blob_bound(m, n):
        return S.blob_bound(m, n, 2, 3)


def _worker_overlapped(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        done = []
        res = S.decompose_sharded(_items(), _RunAllStub(), rank=rank, world=world, max_batch=2,
                                  on_batch_done=lambda j, r: done.append(j))
        info = dict(S.LAST_GATHER)
        if rank == 0:
            q.put((rank, info, done, [(r.name, r.codes.numpy().copy(), r.L.numpy().copy(), r.R.numpy().copy(),
                                       r.Q_scale, r.errors) for r in res]))
        else:
            q.put((rank, info, done, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gather_overlapped_world2_gloo():
    """The overlapped gather (one asynchronous gather per batch, issued in batch order as soon
    as the batch and every earlier one finished; metadata gathered at the end) delivers exactly
    what the one-shot gather does, in item order, with batches finishing out of order and the
    ranks holding different numbers of batches (35 matrices over 2 ranks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_overlapped, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = sorted([q.get(timeout=90) for _ in range(2)], key=lambda o: o[0])
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    items = _items()
    plans = [S._plan(items, 2, r, 2) for r in range(2)]
    assert len(plans[0]) != len(plans[1])  # unequal rounds: the shorter rank sends empty rounds
    for rank, info, done, _ in outs:
        assert info["mode"] == "overlapped" and info["rounds"] == max(len(p) for p in plans), info
        assert sorted(done) == list(range(len(plans[rank])))
    assert outs[1][3] is None
    got = outs[0][3]
    assert [g[0] for g in got] == [it[0] for it in items]
    ref = {r.name: r for r in _stub(items)}
    for name, codes, L, R, qs, errs in got:
        assert torch.equal(torch.from_numpy(codes), ref[name].codes) and torch.equal(torch.from_numpy(L), ref[name].L)
        assert torch.equal(torch.from_numpy(R), ref[name].R) and qs == ref[name].Q_scale and errs == ref[name].errors


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_round_robin_balanced_for_llama2_7b():
    items = S.llama2_7b_matrices()
    assert len(items) == 224
    for world in (1, 2, 4, 8):
        counts = []
        for rank in range(world):
            mine = [items[i] for i in S.shard_indices(len(items), world, rank)]
            shapes = sorted((m, n) for _, m, n, _ in mine)
            counts.append(shapes)
        assert all(c == counts[0] for c in counts), world  # identical shape mix on every rank
    assert sorted(i for r in range(8) for i in S.shard_indices(224, 8, r)) == list(range(224))


def test_pack_unpack_roundtrip(tmp_path):
    res = _stub(_items()[:4])
    back = S.unpack_results(S.pack_results(res))
    for a, b in zip(res, back):
        assert a.name == b.name and a.Q_scale == b.Q_scale and a.errors == b.errors
        assert torch.equal(a.codes, b.codes) and torch.equal(a.L, b.L) and torch.equal(a.R, b.R)
    path = str(tmp_path / "res.bin")
    S.save_results(path, res)
    again = S.load_results(path)
    assert [r.name for r in again] == [r.name for r in res]


@pytest.mark.timeout(120)
def test_gather_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=90) for _ in range(2)]
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    got = next(o for o in outs if o is not None)
    assert any(o is None for o in outs)  # non-root ranks return None
    items = _items()
    assert [g[0] for g in got] == [it[0] for it in items]
    ref = {r.name: r for r in _stub(items)}
    for name, codes, L, R, qs, errs in got:
        assert torch.equal(torch.from_numpy(codes), ref[name].codes) and torch.equal(torch.from_numpy(L), ref[name].L)
        assert torch.equal(torch.from_numpy(R), ref[name].R) and qs == ref[name].Q_scale and errs == ref[name].errors


def test_batches_group_by_hessian():
    """h_key adds a grouping key (batches never mix its values); without it, same-shape
    matrices of different layers -- different diagonal Hessians -- share batches (the engine
    reads per-matrix weights, ABI 5)."""
    items = _items()
    seen = []

    def rec(batch_items):
        seen.append([it[0] for it in batch_items])
        return _stub(batch_items)

    layer_of = lambda name: name.split(".")[2]  # noqa: E731  (one Hessian per layer here)
    res = S.decompose_sharded(items, rec, rank=0, world=1, max_batch=8, h_key=layer_of)
    assert [r.name for r in res] == [it[0] for it in items]
    for b in seen:
        assert len({layer_of(n) for n in b}) == 1, b
    # without h_key, same-shape matrices of different layers share batches
    seen.clear()
    S.decompose_sharded(items, rec, rank=0, world=1, max_batch=8)
    assert any(len({layer_of(n) for n in b}) > 1 for b in seen)


def test_resume_skips_finished_matrices(tmp_path):
    items = _items()
    path = str(tmp_path / "rank0.bin")
    first = S.decompose_sharded(items[:10], _stub, rank=0, world=1, max_batch=4, resume_path=path)
    calls = []

    def rec(batch_items):
        calls.extend(it[0] for it in batch_items)
        return _stub(batch_items)

    res = S.decompose_sharded(items, rec, rank=0, world=1, max_batch=4, resume_path=path)
    assert sorted(calls) == sorted(it[0] for it in items[10:])  # only the unfinished ones ran
    assert [r.name for r in res] == [it[0] for it in items]
    ref = {r.name: r for r in _stub(items)}
    for r in res:
        assert torch.equal(r.codes, ref[r.name].codes) and torch.equal(r.L, ref[r.name].L)
    assert [r.name for r in S.load_results(path)] == [it[0] for it in items]
    assert [r.name for r in first] == [it[0] for it in items[:10]]


def test_pack_keeps_padded_grid_and_alignment():
    """n % 4 != 0: packed codes stay on the (m, n_padded) grid; extra["n_padded"] travels
    with them, and every array starts 16-byte aligned (device views need it)."""
    r = S.MatrixResult("x", 5, 7, 2, 2, torch.arange(10, dtype=torch.uint8), 0.5, torch.randn(5, 2),
                       torch.randn(2, 7), 1.0, {"Q": [1.0]}, {"n_padded": 8})
    buf = S.pack_results([r, r])
    back = S.unpack_results(buf)
    assert back[1].extra == {"n_padded": 8} and torch.equal(back[1].codes, r.codes)
    assert torch.equal(back[1].R, r.R) and back[1].R.data_ptr() % 16 == 0


def test_payload_magic_and_version_are_checked():
    """The payload starts with "CQRS" + a format version: a round-2 payload (bare u64 length,
    no magic) or a future version is rejected instead of being misparsed."""
    import struct
    res = _stub(_items()[:2])
    buf = S.pack_results(res)
    assert bytes(buf[:4].numpy().tobytes()) == b"CQRS"
    old = bytearray(buf.numpy().tobytes())
    meta_len = struct.unpack("<Q", bytes(old[8:16]))[0]
    legacy = struct.pack("<Q", meta_len) + bytes(old[16:])   # the round-2 header layout
    with pytest.raises(ValueError, match="magic"):
        S.unpack_results(torch.frombuffer(bytearray(legacy), dtype=torch.uint8))
    future = bytearray(old)
    future[4:8] = struct.pack("<I", 99)
    with pytest.raises(ValueError, match="version 99"):
        S.unpack_results(torch.frombuffer(future, dtype=torch.uint8))
    with pytest.raises(ValueError):
        S.unpack_results(torch.zeros(3, dtype=torch.uint8))


def _worker_async(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # two steps' payloads in flight at once (bench.py: step i's gather under step i + 1),
        # one with the sizes given (no size exchange), one with ragged sizes exchanged
        p1 = torch.arange(64, dtype=torch.int64).to(torch.uint8) + rank
        p2 = torch.full((10 + 7 * rank,), 100 + rank, dtype=torch.uint8)
        g1 = S.gather_to_rank0_async(p1, sizes=[64] * world)
        g2 = S.gather_to_rank0_async(p2)
        p1.zero_()   # the send buffers are copies: the caller may reuse its payload at once
        o1, o2 = g1.wait(), g2.wait()
        q.put((rank, None if o1 is None else [t.numpy().copy() for t in o1],
               None if o2 is None else [t.numpy().copy() for t in o2]))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gather_async_world2_gloo():
    """gather_to_rank0_async (bench.py's N > 1 step gather, overlapped with the next step):
    rank 0 receives every rank's payload in rank order, trimmed to its size; others get None."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_async, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    outs = sorted([q.get(timeout=90) for _ in range(2)], key=lambda o: o[0])
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    (_, o1, o2), (_, n1, n2) = outs
    assert n1 is None and n2 is None
    for r in range(2):
        assert o1[r].tolist() == [(i + r) % 256 for i in range(64)]
        assert o2[r].tolist() == [100 + r] * (10 + 7 * r)
