"""Parity oracle (test infrastructure only -- see md2_oracle.py header)."""
