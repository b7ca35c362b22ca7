"""CPU oracle (test infrastructure only; see kge_oracle.py)."""
