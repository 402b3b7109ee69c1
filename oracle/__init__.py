"""Test infrastructure only: the CPU checker (scalar C restatement) and the AVX2 port used
as bench.py's CPU baseline.  Only tests/, __graft_entry__.smoke() and bench.py import it."""
