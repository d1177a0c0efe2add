"""ORACLE — test infrastructure only (see miner_oracle.py header).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
