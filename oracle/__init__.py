"""CPU oracle (test infrastructure only) -- see csmom_oracle.py."""
