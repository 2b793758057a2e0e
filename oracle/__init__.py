"""CPU oracle for the DS2 hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker (or as the timed CPU baseline).  The
product path (deepspeech.pytorch_amd/ds2amd) never imports it and has no CPU
fallback.  Pinning: see oracle/ds2_oracle.py header and tests/golden/.
"""
