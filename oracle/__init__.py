"""CPU oracle package -- test infrastructure only (see oracle/gsdr_oracle.h)."""
