"""CPU oracle for the scan-result hot path — TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker. See semantics.py for what each function restates and how it is pinned.
"""
