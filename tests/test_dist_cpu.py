"""Multi-rank path on CPU: gloo, world size 2 (and 3), no GPU.

Checks the sharding invariant (owned ranges tile the (seq, k) space in order)
and the gatherv over torch.distributed with per-rank hit lists produced by the
C oracle on each rank's owned range.
"""

import os
import socket
import sys

import numpy as np
import pytest

from merpcr_amd.dist import HIT_BYTES, as_hits, contig_shards, gather_hits, shard_ranges

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shard_ranges_tile_the_genome():
    lens = [100, 0, 5, 1000, 37]
    for world in (1, 2, 3, 8, 17):
        rs = shard_ranges(lens, world)
        assert rs[0][:1] == (0,) and rs[0][2] == 0
        assert rs[-1][1] == len(lens) and rs[-1][3] == 0
        for a, b in zip(rs[:-1], rs[1:]):
            assert (a[1], a[3]) == (b[0], b[2])


def test_contig_shards_balance_whole_records():
    lens = [250, 10, 10, 200, 190, 5, 0, 180]
    for world in (1, 2, 3, 4, 8, 11):
        rs = contig_shards(lens, world)
        assert len(rs) == world and rs[0][0] == 0 and rs[-1][1] == len(lens)
        assert all(a[1] == b[0] for a, b in zip(rs[:-1], rs[1:]))
        assert all(a <= b for a, b in rs)
    assert contig_shards(lens, 2) == [(0, 4), (4, 8)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from oracle import c_oracle as C
    from oracle import epcr_oracle as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(5)
    seqs = [np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, n)] for n in (40_000, 300, 25_000)]
    p1, p2 = "ACGTTGCAAGCTTAGCA", "GGATCCTTAGGCATCAT"
    amp = (p2 + "ACGT" * 40 + O.revcomp(p1)).encode()
    for s in seqs[::2]:
        for pos in range(100, len(s) - 400, 3001):
            s[pos:pos + len(amp)] = np.frombuffer(amp, dtype=np.uint8)
    table = O.load_sts_lines([f"A\t{p1}\t{p2}\t200\n"], 8, 240)
    prm = O.params(wordsize=8, margin=50)
    whole = C.search(table, seqs, prm)
    # this rank's owned (seq, k) range, restricted from the whole-genome list
    sa, sb, ka, kb = shard_ranges([len(s) for s in seqs], world)[rank]
    key = whole["seq"].astype(np.int64) * (1 << 40) + whole["pos1"].astype(np.int64)
    lo, hi = sa * (1 << 40) + ka, sb * (1 << 40) + kb
    mine = whole[(key >= lo) & (key < hi)]
    buf = torch.from_numpy(np.frombuffer(mine.tobytes() + b"\0" * HIT_BYTES, dtype=np.uint8).copy())
    got = gather_hits(buf, len(mine))
    ok = rank != 0 or as_hits(got).tobytes() == whole.tobytes()
    # contig sharding: this rank searches only its own whole records, indices local to them
    fa, fb = contig_shards([len(s) for s in seqs], world)[rank]
    part = C.search(table, seqs[fa:fb], prm) if fb > fa else whole[:0]
    buf = torch.from_numpy(np.frombuffer(part.tobytes() + b"\0" * HIT_BYTES, dtype=np.uint8).copy())
    got = gather_hits(buf, len(part), seq_base=fa)
    if rank == 0:
        ok = ok and as_hits(got).tobytes() == whole.tobytes()
        q.put((ok, len(whole)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_gloo(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, n = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert ok and n > 10


def _comm_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, ROOT)
    import bench
    comm = bench.agreed_comm(0, rank, world)  # no GPU here: every rank must come back with None
    q.put((rank, comm is None))
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_fallback_is_agreed_without_a_gpu():
    """bench.py's RCCL data plane when a communicator cannot be made (here: no GPU): every
    rank leaves the collective set-up with None (the job then gathers on the host) instead of
    one rank raising while another waits in a broadcast."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got == [(0, True), (1, True)]
