"""python -m merpcr_amd (reference: src/merpcr/__main__.py)."""

from .cli import main

if __name__ == "__main__":
    raise SystemExit(main())
