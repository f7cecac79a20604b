"""Device FASTA ingestion (mp_fasta_load_device) vs the host reader and the reference loop.

The expected side is FASTALoader.load_file_py, the Python restatement of
src/merpcr/io/fasta.py:18-71 (pinned to the reference's recorded loader outputs by
tests/test_host.py), and the native host reader mp_fasta_load.  Inputs are ASCII texts
that stress what the device pass re-implements: universal newlines, str.strip()'s ASCII
whitespace before '>' and around lines, blank lines, empty and '>'-only records, text
before the first header, '>' inside sequence lines, and (large cases) header lines and
records across the 64 KiB compaction tiles.  A non-ASCII byte sends the file to the host
reader, with the same records.
"""

import os
import random

import numpy as np
import pytest

from merpcr_amd import MerPCR, _native
from merpcr_amd.io import fasta as F

pytestmark = pytest.mark.gpu

WS = [" ", "\t", "\x0b", "\x0c", "\x1c", "\x1f"]
NL = ["\n", "\r\n", "\r"]
LETTERS = "ACGTNacgtnUuRYKMSWBDHVXZzj12-*.>"


def _records(recs):
    return [(r.defline, r.sequence, r.label) for r in recs]


def _expected(path):
    try:
        return _records(F.FASTALoader.load_file_py(path))
    except Exception as e:  # noqa: BLE001 - compare exception types
        return type(e)


def _device(path, monkeypatch):
    monkeypatch.setattr(F, "DEVICE_MIN_BYTES", 0)
    try:
        recs = F.FASTALoader.load_file(path, device=0)
        return _records(recs), [type(r).__name__ for r in recs]
    except Exception as e:  # noqa: BLE001
        return type(e), []


def _random_text(rng, n_lines=12, line_max=40):
    out = []
    for _ in range(rng.randint(0, n_lines)):
        kind = rng.random()
        pre = "".join(rng.choice(WS) for _ in range(rng.randint(0, 2))) if rng.random() < 0.3 else ""
        post = "".join(rng.choice(WS) for _ in range(rng.randint(0, 2))) if rng.random() < 0.3 else ""
        if kind < 0.25:
            body = ">" + "".join(rng.choice("abc XYZ_|.\t") for _ in range(rng.randint(1, 12)))
            body = body if body.strip() != ">" else ">x"
        elif kind < 0.35:
            body = ""
        else:
            body = "".join(rng.choice(LETTERS + " ") for _ in range(rng.randint(0, line_max)))
        out.append(pre + body + post + rng.choice(NL))
    if out and rng.random() < 0.5:
        out[-1] = out[-1].rstrip("\r\n")
    return "".join(out)


def test_device_reader_matches_reference_loop(tmp_path, monkeypatch):
    rng = random.Random(4321)
    p = str(tmp_path / "x.fa")
    n_dev = 0
    for i in range(300):
        text = _random_text(rng)
        if not text:
            continue
        with open(p, "wb") as fh:
            fh.write(text.encode("ascii"))
        exp = _expected(p)
        got, kinds = _device(p, monkeypatch)
        if exp is IndexError:  # '>' alone: FASTARecord's label (models.py), as the reference
            assert got is IndexError, (i, text)
            continue
        assert got == exp, (i, text)
        n_dev += kinds.count("DeviceRecord")
    assert n_dev > 100


def test_non_ascii_file_goes_to_the_host_reader(tmp_path, monkeypatch):
    p = str(tmp_path / "u.fa")
    with open(p, "wb") as fh:
        fh.write(">a b\n ACGTſN　\n>c\nacgt\n".encode("utf-8"))
    assert _native.fasta_read_device(p, 0) is None
    got, kinds = _device(p, monkeypatch)
    assert got == _expected(p) and "DeviceRecord" not in kinds


def test_large_file_across_tiles(tmp_path, monkeypatch):
    """~6 MB: ~100 records of random sizes, every line-ending form, header lines with
    leading blanks landing on and across 64 KiB tile boundaries, a text prefix before the
    first header; the device records equal the host reader's byte for byte."""
    rng = random.Random(99)
    parts = ["ACGT junk before any header\r\n", "  \t\n"]
    pos = sum(len(x) for x in parts)
    for r in range(100):
        nl = rng.choice(NL)
        # put some header lines right at / across a tile boundary
        if r % 10 == 3:
            pad = (65536 - pos % 65536) - rng.randint(0, 3)
            if pad > 1:
                parts.append("A" * (pad - 1) + "\n")
                pos += pad
        head = rng.choice(["", " ", "\t ", "\x1c"]) + f">rec{r} descr {rng.random():.3f}" + rng.choice(["", " ", "\t"]) + nl
        parts.append(head)
        pos += len(head)
        for _ in range(rng.randint(0, 1200)):
            body = "".join(rng.choice(LETTERS[:-1]) for _ in range(rng.randint(0, 70)))
            if len(body) > 2 and rng.random() < 0.05:  # a '>' inside a sequence line: dropped
                k = rng.randint(1, len(body) - 1)
                body = body[:k] + ">" + body[k:]
            line = body + rng.choice(NL)
            parts.append(line)
            pos += len(line)
    p = str(tmp_path / "big.fa")
    with open(p, "wb") as fh:
        fh.write("".join(parts).encode("ascii"))
    want = _native.fasta_read(p)
    got = _native.fasta_read_device(p, 0)
    assert got is not None and len(got) == len(want) == 100
    for (dw, sw), (dg, sg) in zip(want, got):
        assert dw == dg
        assert bytes(sw) == sg.host(), dw
    assert sum(len(s) for _, s in got) > 1_000_000
    got_recs, kinds = _device(p, monkeypatch)
    assert set(kinds) == {"DeviceRecord"} and got_recs == _expected(p)


def test_search_from_device_records_matches_host_records(tmp_path, monkeypatch):
    """The engine packs DeviceRecord sequences where they are (mp_genome_put_device) and
    finds exactly the hits of the host-read records; .sequence still gives the str."""
    from tests.test_gpu_parity import _load_sts, _synthetic
    sts_text, seq = _synthetic(31, 300, 400_000, 11, 1, 0, nrun=True)
    p = str(tmp_path / "g.fa")
    with open(p, "w") as fh:
        fh.write(">chrA first\n")
        for i in range(0, 200_000, 60):
            fh.write(seq[i:i + 60] + "\n")
        fh.write("\n>chrB\r\n")
        for i in range(200_000, len(seq), 77):
            fh.write(seq[i:i + 77] + "\r\n")
    res = []
    for dev_min in (0, 1 << 40):
        monkeypatch.setattr(F, "DEVICE_MIN_BYTES", dev_min)
        eng = MerPCR(wordsize=11, mismatches=1)
        assert _load_sts(eng, sts_text, str(tmp_path))
        recs = eng.load_fasta_file(p, on_device=True)
        kinds = {type(r).__name__ for r in recs}
        hits = eng.find_hits(recs)
        res.append((kinds, eng.format_hits(recs, hits), [r.sequence for r in recs]))
    assert res[0][0] == {"DeviceRecord"} and res[1][0] == {"ReaderRecord"}
    assert res[0][1] == res[1][1] and len(res[0][1]) > 50
    assert res[0][2] == res[1][2]
    # the default (API callers that may never search): host records, no device allocation
    monkeypatch.setattr(F, "DEVICE_MIN_BYTES", 0)
    eng = MerPCR(wordsize=11, mismatches=1)
    assert {type(r).__name__ for r in eng.load_fasta_file(p)} == {"ReaderRecord"}
