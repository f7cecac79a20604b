"""GPU parity at the benchmark configs' full table scale.

The bench configs c3/c4/c5 use 100k-STS tables (200k records: 195k distinct keys at
W=11, 62k at W=8 with a mean fan-out of 3.2 records per key).  Here the real tables
go through the default kernels over a genome prefix the C oracle scans in seconds
(c3/c4: 40 Mbp, c5: 48 Mbp -- past the ~34 Mbp where the scans' super-step claims turn
dynamic, so c5's split scans each take fresh chunk counters), generated exactly as bench.py does (synth.py: N runs,
soft-masking, every STS planted in both orientations, densely here), and the hit
lists must be byte-identical.  The table regime -- seed fan-out, prefilter pass rate,
bucket tails, full-head deferral, dense_kernel's escape buckets -- is the full-size
one; only the genome is shorter.
"""

import os
import tempfile

import numpy as np
import pytest

from merpcr_amd import MerPCR, _native, synth
from oracle import c_oracle as C
from oracle import epcr_oracle as O

pytestmark = pytest.mark.gpu

_THREADS = max(1, min(16, len(os.sched_getaffinity(0))))


@pytest.mark.parametrize("name,total,records", [("c3", 40_000_000, 3), ("c4", 40_000_000, 3),
                                                ("c5", 48_000_000, 2),
                                                # c2's whole workload: 10k STS x one 250 Mbp record
                                                ("c2", 250_000_000, 1),
                                                # one 300 Mbp record: hits past 2^27 / 2^28 and in the
                                                # record's last kbp (u32 span offsets, exception-run
                                                # directory indices deep in a record)
                                                ("c3", 300_000_000, 1),
                                                # the whole c2-sized record at the c4/c5 tables: the
                                                # IUPAC-head drain and the split-seed scans (two seed
                                                # passes, dynamic claims) over one 250 Mbp record
                                                ("c4", 250_000_000, 1), ("c5", 250_000_000, 1)])
def test_full_table_prefix_vs_c_oracle(name, total, records):
    import torch
    cfg = synth.CONFIGS[name]
    sts = synth.make_sts(cfg["n_sts"], W=cfg["W"], iupac=cfg["iupac"])
    eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"])
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "c.sts")
        with open(p, "w") as fh:
            fh.write(sts.text())
        assert eng.load_sts_file(p)
    assert len(eng.sts_records) == 2 * cfg["n_sts"]
    table = eng.device_table()
    dev = torch.device("cuda", 0)
    names, lens, buf, offs, planted = synth.build_genome_torch(
        total, records, sts, seed=1, N=cfg["N"], M=cfg["M"], W=cfg["W"], nrun=cfg["nrun"], device=dev)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream().cuda_stream
    genome = _native.Genome(0, lens)
    for r, n in enumerate(lens):
        genome.put_device(r, buf.data_ptr() + int(offs[r]), n, stream=stream)
    genome.seal(stream)
    search = _native.Search(table, genome)
    got = search.fetch(search.run(None, stream))
    stats = search.last_stats()
    host = buf.cpu().numpy()
    seqs = [host[int(offs[r]):int(offs[r]) + lens[r]] for r in range(len(lens))]
    otable = O.load_sts_lines(sts.text().splitlines(True), cfg["W"], 240)
    prm = O.params(wordsize=cfg["W"], mismatches=cfg["N"], margin=cfg["M"], iupac_mode=cfg["I"])
    ref = C.search(otable, seqs, prm, _THREADS)
    search.close()
    genome.close()
    assert planted > 10_000 and len(ref) > planted // 2, (planted, len(ref))
    assert stats["windows"] >= 0.9 * total
    assert len(got) == len(ref), (len(got), len(ref), stats)
    assert got.tobytes() == ref.tobytes()
    if records == 1 and total >= 1 << 28:
        pos = got["pos1"].astype(np.int64)
        assert (pos > 1 << 28).sum() > 1000, "no hits deep in the record"
        assert pos.max() > total - 5_000, (int(pos.max()), total)


def test_genome_past_2_32_vs_c_oracle():
    """A 4.5 Gbp genome (c3 table): three records, the first longer than 2^31 bases, the
    last wholly past global base 2^32, amplicons planted on every record's final bases.
    Pins the 33-bit k field of the packed order key (mp_order.hip sort_plan), the high
    words of survivor / tail-reference positions and the hit decode's sequence search."""
    import torch
    cfg = synth.CONFIGS["c3"]
    lens = [2_300_000_000, 1_200_000_000, 1_000_000_000]
    total = sum(lens)
    sts = synth.make_sts(cfg["n_sts"], W=cfg["W"])
    eng = MerPCR(wordsize=cfg["W"], margin=cfg["M"], mismatches=cfg["N"], iupac_mode=cfg["I"])
    with tempfile.TemporaryDirectory() as td:
        p = os.path.join(td, "c.sts")
        with open(p, "w") as fh:
            fh.write(sts.text())
        assert eng.load_sts_file(p)
    table = eng.device_table()
    dev = torch.device("cuda", 0)
    names, lens, buf, offs, planted = synth.build_genome_torch(
        total, len(lens), sts, seed=3, N=cfg["N"], M=cfg["M"], W=cfg["W"], nrun=cfg["nrun"], device=dev, lens=lens)
    n_end = synth.plant_at_ends(buf, offs, lens, sts)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream().cuda_stream
    genome = _native.Genome(0, lens)
    for r, n in enumerate(lens):
        genome.put_device(r, buf.data_ptr() + int(offs[r]), n, stream=stream)
    genome.seal(stream)
    search = _native.Search(table, genome)
    got = search.fetch(search.run(None, stream))
    search.close()
    genome.close()
    host = buf.cpu().numpy()
    del buf
    torch.cuda.empty_cache()
    seqs = [host[int(offs[r]):int(offs[r]) + lens[r]] for r in range(len(lens))]
    otable = O.load_sts_lines(sts.text().splitlines(True), cfg["W"], 240)
    prm = O.params(wordsize=cfg["W"], mismatches=cfg["N"], margin=cfg["M"], iupac_mode=cfg["I"])
    ref = C.search(otable, seqs, prm, _THREADS)
    assert n_end == 3 * len(lens) and planted > 100_000
    assert len(got) == len(ref), (len(got), len(ref))
    assert got.tobytes() == ref.tobytes()
    # coverage of what the case is for
    gstart = np.cumsum([0] + [(n + 63) // 64 * 64 for n in lens[:-1]])
    gpos = gstart[got["seq"].astype(np.int64)] + got["pos1"].astype(np.int64)
    assert (gpos >= 1 << 32).sum() > 1000, "no hits past global base 2^32"
    assert ((got["seq"] == 0) & (got["pos1"] >= 1 << 31)).sum() > 1000, "no hits past 2^31 in record 0"
    for r, n in enumerate(lens):
        sel = got["seq"] == r
        assert int(got["pos2"][sel].max()) == n - 1, (r, n)  # the amplicon on the record's final base
