"""Native FASTA reader (mp_fasta_load) vs the reference's text-mode loop.

The expected side is FASTALoader.load_file_py, the Python restatement of
src/merpcr/io/fasta.py:18-71 (itself pinned to the reference's recorded loader
outputs by tests/test_host.py::test_fasta_loader_matches_reference).  Inputs are
byte strings that stress what the C++ reader re-implements: universal newlines
(also split across read chunks), Python's Unicode whitespace in strip(), the
U+017F keep character, BOMs, blank and header-less lines, invalid UTF-8.
"""

import os
import random

import pytest

from merpcr_amd import _native
from merpcr_amd.io.fasta import FASTALoader

pytestmark = pytest.mark.skipif(not os.path.exists(_native.LIB_PATH), reason="library not built")

WS = [" ", "\t", "\x0b", "\x0c", "\x1c", "\x1f", "\x85", "\xa0", " ", " ", " ",
      " ", " ", " ", "　", "﻿", "​"]
NL = ["\n", "\r\n", "\r"]
LETTERS = "ACGTNacgtnUuRYKMSWBDHVXZzjſ12-*.É中"


def _expected(path):
    try:
        return [(r.defline, r.sequence, r.label) for r in FASTALoader.load_file_py(path)]
    except Exception as e:  # noqa: BLE001 - compare exception types
        return type(e)


def _native_read(path, chunk=0):
    try:
        return [(r.defline, r.sequence, r.label) for r in FASTALoader.load_file(path, _chunk_bytes=chunk)]
    except Exception as e:  # noqa: BLE001
        return type(e)


def _random_text(rng):
    out = []
    for _ in range(rng.randint(0, 12)):
        kind = rng.random()
        pre = "".join(rng.choice(WS) for _ in range(rng.randint(0, 2))) if rng.random() < 0.3 else ""
        post = "".join(rng.choice(WS) for _ in range(rng.randint(0, 2))) if rng.random() < 0.3 else ""
        if kind < 0.25:
            body = ">" + "".join(rng.choice("abc XYZ_|.\t" + "　ſé") for _ in range(rng.randint(1, 12)))
            body = body if body.strip() != ">" else ">x"
        elif kind < 0.35:
            body = ""
        else:
            body = "".join(rng.choice(LETTERS + " ") for _ in range(rng.randint(0, 40)))
        out.append(pre + body + post + rng.choice(NL))
    if out and rng.random() < 0.5:
        out[-1] = out[-1].rstrip("\r\n")  # no final newline
    return "".join(out)


@pytest.mark.parametrize("chunk", [0, 4, 7, 64])
def test_native_matches_python_loop(tmp_path, chunk):
    rng = random.Random(1234 + chunk)
    p = str(tmp_path / "x.fa")
    for i in range(300):
        text = _random_text(rng)
        if not text:
            continue
        with open(p, "wb") as fh:
            fh.write(text.encode("utf-8"))
        exp = _expected(p)
        got = _native_read(p, chunk)
        if isinstance(exp, type) and exp is IndexError:  # '>' alone: FASTARecord label
            assert got is IndexError
            continue
        assert got == exp, (i, text)


@pytest.mark.parametrize("blob", [
    b">a\nAC\xffGT\n", b">a\nACGT\xc5", b">a\nAC\xed\xa0\x80GT\n", b">a\xc0\xaf\nAC\n",
    b">a\nAC\xf4\x90\x80\x80\n", b">a\nAC\xe0\x80\x80\n",
])
def test_invalid_utf8_raises_like_reference(tmp_path, blob):
    p = str(tmp_path / "bad.fa")
    with open(p, "wb") as fh:
        fh.write(blob)
    with pytest.raises(UnicodeDecodeError):
        FASTALoader.load_file_py(p)
    with pytest.raises(UnicodeDecodeError):
        FASTALoader.load_file(p)


def test_crlf_split_across_chunks(tmp_path):
    p = str(tmp_path / "crlf.fa")
    text = ">s1 d\r\nACGT\r\n\r\nGG\r>s2\r\nTT\r\n"
    with open(p, "wb") as fh:
        fh.write(text.encode())
    exp = _expected(p)
    for c in range(4, len(text) + 2):
        assert _native_read(p, c) == exp, c


def test_missing_and_empty(tmp_path):
    with pytest.raises(FileNotFoundError):
        FASTALoader.load_file(str(tmp_path / "nope.fa"))
    p = tmp_path / "empty.fa"
    p.write_bytes(b"")
    assert FASTALoader.load_file(str(p)) == []


def test_reader_records_keep_bytes(tmp_path):
    """Records from the native reader equal the Python loop's FASTARecords; ASCII sequences
    reach the engine's encoder as the reader's bytes (no str round trip), and a record with
    U+017F or a reassigned sequence goes through the str path."""
    import numpy as np
    from merpcr_amd import FASTARecord, MerPCR
    p = tmp_path / "r.fa"
    p.write_text(">a one\nACGTacgtNN\n>b\nACſGT\n>c\n\n", encoding="utf-8")
    got = FASTALoader.load_file(str(p))
    exp = FASTALoader.load_file_py(str(p))
    assert got == exp and exp == got
    assert [repr(r) for r in got] == [repr(FASTARecord(r.defline, r.sequence, r.label)) for r in exp]
    got = FASTALoader.load_file(str(p))
    assert got[0].raw_ascii() == b"ACGTacgtNN" and got[1].raw_ascii() is None
    eng = MerPCR()
    enc = eng.encode_records(got)
    ref = eng.encode_sequences([r.sequence for r in exp])
    assert all(np.array_equal(x, y) for x, y in zip(enc, ref))
    got[0].sequence = "TTTT"
    assert got[0].raw_ascii() is None and np.array_equal(eng.encode_records(got[:1])[0], np.frombuffer(b"TTTT", np.uint8))


def _parallel_read(path, threads):
    try:
        return [(d, s) for d, s in _native.fasta_read(path, 0, threads)]
    except Exception as e:  # noqa: BLE001
        return type(e)


@pytest.mark.parametrize("threads", [2, 3, 7, 16])
def test_parallel_reader_splits(tmp_path, threads):
    """The parallel whole-file reader with more threads than a small file needs: its
    validation, header and filter splits fall inside lines, UTF-8 sequences, CR/LF pairs
    and headers; every split must give the streaming reader's records."""
    rng = random.Random(99 + threads)
    p = str(tmp_path / "x.fa")
    for i in range(300):
        text = _random_text(rng)
        if not text:
            continue
        with open(p, "wb") as fh:
            fh.write(text.encode("utf-8"))
        exp = _native.fasta_read(p, 1 << 20) if _expected(p) is not UnicodeDecodeError else UnicodeDecodeError
        got = _parallel_read(p, threads)
        assert got == exp, (i, text)


def test_parallel_reader_long_lines_and_records(tmp_path):
    """Multi-megabyte single-line and 60-column records, soft-masked, with N runs: the
    parallel reader (default threads, pieces of ~64 KiB and more) equals the streaming one."""
    import numpy as np
    rng = np.random.default_rng(3)
    parts = []
    for r in range(5):
        n = int(rng.integers(1, 3_000_000))
        s = np.frombuffer(b"ACGTNacgtn", np.uint8)[rng.integers(0, 10, n)].tobytes()
        parts.append(f">rec{r} some words\t \n".encode())
        if r % 2:
            parts.append(s + b"\n")
        else:
            parts.append(b"\n".join(s[i:i + 60] for i in range(0, n, 60)) + b"\r\n")
    p = str(tmp_path / "big.fa")
    with open(p, "wb") as fh:
        fh.write(b"".join(parts))
    exp = _native.fasta_read(p, 1 << 20)
    for threads in (0, 5):
        assert _native.fasta_read(p, 0, threads) == exp


def test_reader_records_pickle_and_copy(tmp_path):
    """Records from the native reader serialise as the reference's plain FASTARecord."""
    import copy
    import pickle

    from merpcr_amd.core.models import FASTARecord
    p = tmp_path / "a.fa"
    p.write_text(">s1 first\nACGTNacgt\n>s2\nGGGG\n")
    recs = FASTALoader.load_file(str(p))
    for r in recs:
        for back in (pickle.loads(pickle.dumps(r)), copy.copy(r), copy.deepcopy(r)):
            assert type(back) is FASTARecord
            assert (back.defline, back.sequence, back.label) == (r.defline, r.sequence, r.label)


def test_non_regular_file_streams(tmp_path):
    """A pipe (st_size 0, not mappable) goes through the streaming reader, not an empty mmap."""
    import threading
    fifo = tmp_path / "f.fifo"
    os.mkfifo(fifo)
    text = ">p\nACGT\nTTAA\n>q\nGG\n"

    def writer():
        with open(fifo, "w") as fh:
            fh.write(text)

    th = threading.Thread(target=writer)
    th.start()
    got = [(d, bytes(s)) for d, s in _native.fasta_read(str(fifo), 0)]
    th.join()
    assert got == [(">p", b"ACGTTTAA"), (">q", b"GG")]
