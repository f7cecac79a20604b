"""CPU oracle for parity tests (test infrastructure only; see epcr_oracle.py)."""
