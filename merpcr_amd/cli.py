"""Command line, behaviour-identical to the reference's (src/merpcr/cli.py).

me-PCR style ``X=value`` arguments are rewritten to ``-X value`` (cli.py:19-62),
the same validators and defaults apply (cli.py:79-214), and the exit code is 0
on success, 1 on any failure (cli.py:217-266).
"""

import argparse
import logging
import sys
import threading
from typing import List

from .core.engine import (DEFAULT_IUPAC_MODE, DEFAULT_MARGIN, DEFAULT_MISMATCHES, DEFAULT_PCR_SIZE,
                          DEFAULT_THREADS, DEFAULT_THREE_PRIME_MATCH, DEFAULT_WORDSIZE, MerPCR)

DEFAULT_MAX_STS_LINE_LENGTH = 1022
_MEPCR_FLAGS = "MNWXTQZISO"


def convert_mepcr_arguments(args: List[str]) -> List[str]:
    """Rewrite me-PCR ``M=50`` style arguments; ``P=`` is dropped, ``-help`` -> ``--help``."""
    out: List[str] = []
    for arg in args:
        if len(arg) >= 3 and arg[1] == "=" and arg[0] in _MEPCR_FLAGS + "P":
            if arg[0] != "P":
                out.extend(["-" + arg[0], arg[2:]])
        elif arg == "-help":
            out.append("--help")
        else:
            out.append(arg)
    return out


def setup_logging(quiet: int, debug: bool) -> None:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s - %(levelname)s - %(message)s")
    logger = logging.getLogger("merpcr")
    if debug:
        logger.setLevel(logging.DEBUG)
    elif quiet == 0:
        logger.setLevel(logging.INFO)
    else:
        logger.setLevel(logging.WARNING)


def _bounded(name, lo, hi=None, fmt=None):
    def check(value):
        v = int(value)
        if v < lo or (hi is not None and v > hi):
            raise argparse.ArgumentTypeError(fmt.format(v=v))
        return v
    check.__name__ = name
    return check


margin_type = _bounded("margin_type", 0, 10000, "Margin must be between 0-10000, got {v}")
mismatch_type = _bounded("mismatch_type", 0, 10, "Mismatches must be between 0-10, got {v}")
wordsize_type = _bounded("wordsize_type", 3, 16, "Word size must be between 3-16, got {v}")
threads_type = _bounded("threads_type", 1, None, "Threads must be > 0, got {v}")
pcr_size_type = _bounded("pcr_size_type", 1, 10000, "PCR size must be between 1-10000, got {v}")
sts_line_length_type = _bounded("sts_line_length_type", 1, None, "STS line length must be > 0, got {v}")


def create_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="merPCR - Modern Electronic Rapid PCR (MI355X engine)",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("sts_file", type=str, help="STS file (tab-delimited)")
    p.add_argument("fasta_file", type=str, help="FASTA sequence file")
    p.add_argument("-M", "--margin", type=margin_type, default=DEFAULT_MARGIN,
                   help=f"Margin (default: {DEFAULT_MARGIN})")
    p.add_argument("-N", "--mismatches", type=mismatch_type, default=DEFAULT_MISMATCHES,
                   help=f"Number of mismatches allowed (default: {DEFAULT_MISMATCHES})")
    p.add_argument("-W", "--wordsize", type=wordsize_type, default=DEFAULT_WORDSIZE,
                   help=f"Word size (default: {DEFAULT_WORDSIZE})")
    p.add_argument("-T", "--threads", type=threads_type, default=DEFAULT_THREADS,
                   help=f"Number of threads (default: {DEFAULT_THREADS})")
    p.add_argument("-X", "--three-prime-match", type=int, default=DEFAULT_THREE_PRIME_MATCH,
                   help="Number of 3'-ward bases in which to disallow mismatches "
                        f"(default: {DEFAULT_THREE_PRIME_MATCH})")
    p.add_argument("-O", "--output", type=str, default=None, help="Output file name (default: stdout)")
    p.add_argument("-Q", "--quiet", type=int, choices=[0, 1], default=1,
                   help="Quiet flag (0=verbose, 1=quiet)")
    p.add_argument("-Z", "--default-pcr-size", type=pcr_size_type, default=DEFAULT_PCR_SIZE,
                   help=f"Default PCR size (default: {DEFAULT_PCR_SIZE})")
    p.add_argument("-I", "--iupac", type=int, choices=[0, 1], default=DEFAULT_IUPAC_MODE,
                   help="IUPAC flag (0=don't honor IUPAC ambiguity symbols, 1=honor IUPAC symbols)")
    p.add_argument("-S", "--max-sts-line-length", type=sts_line_length_type,
                   default=DEFAULT_MAX_STS_LINE_LENGTH,
                   help=f"Max. line length for the STS file (default: {DEFAULT_MAX_STS_LINE_LENGTH})")
    p.add_argument("-v", "--version", action="version", version="merPCR version 1.0.0")
    p.add_argument("--debug", action="store_true", help="Enable debug logging")
    p.add_argument("--device", type=int, default=None, help="HIP device index (default: 0)")
    p.add_argument("--gpus", type=_bounded("gpus_type", 1, None, "GPUs must be > 0, got {v}"), default=1,
                   help="search on this many GPUs (devices --device, --device+1, ...): the sequences' "
                        "positions are split among them and the hits gathered over RCCL")
    p.add_argument("--emulate-chunks", action="store_true",
                   help="with -T > 1, reproduce the reference's per-chunk output (duplicate overlap "
                        "hits) instead of the exact single-chunk result")
    return p


def main(argv: List[str] = None) -> int:
    args = create_parser().parse_args(convert_mepcr_arguments(sys.argv[1:] if argv is None else argv))
    setup_logging(args.quiet, args.debug)
    logger = logging.getLogger("merpcr")
    try:
        eng = MerPCR(wordsize=args.wordsize, margin=args.margin, mismatches=args.mismatches,
                     three_prime_match=args.three_prime_match, iupac_mode=args.iupac,
                     default_pcr_size=args.default_pcr_size, threads=args.threads,
                     max_sts_line_length=args.max_sts_line_length, device=args.device,
                     emulate_chunks=args.emulate_chunks,
                     devices=[(args.device or 0) + i for i in range(args.gpus)] if args.gpus > 1 else None)
        # the HIP runtime starts on a thread beside the STS parse, and the device tables are
        # built beside the FASTA read (native calls release the GIL)
        from . import _native
        warm = None
        try:
            _native.lib()  # loaded once, here, before the threads use it
            warm = threading.Thread(target=_native.device_count, daemon=True)
            warm.start()
        except Exception:  # noqa: BLE001 -- no library: search() reports it in its turn
            warm = None
        if not eng.load_sts_file(args.sts_file):
            logger.error(f"Failed to load STS file: {args.sts_file}")
            return 1
        prep = None
        if warm is not None:
            prep = threading.Thread(target=eng.prepare_device, daemon=True)
            prep.start()
        try:
            # the CLI searches what it reads: large ASCII files are ingested on the GPU
            records = eng.load_fasta_file(args.fasta_file, on_device=True)
        finally:
            if prep is not None:
                prep.join()
            if warm is not None:
                warm.join()
        if not records:
            logger.error(f"Failed to load FASTA file: {args.fasta_file}")
            return 1
        n = eng.search(records, args.output)
        logger.info(f"Search complete: {n} hits found")
        return 0
    except Exception as e:  # cli.py:260-266: any failure -> exit 1
        logger.error(f"Error: {str(e)}")
        if args.debug:
            import traceback
            traceback.print_exc()
        return 1


if __name__ == "__main__":
    sys.exit(main())
