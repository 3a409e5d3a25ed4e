"""TEST INFRASTRUCTURE ONLY: the CPU restatement of the reference codec (parity oracle)."""
