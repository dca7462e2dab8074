"""CPU oracle for the uam_path_planning hot path.  TEST INFRASTRUCTURE, NOT PRODUCT.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
as the checker (and the timed CPU baseline), never as the thing measured or shipped.
Parity pinned against golden vectors recorded from the reference (tests/golden/).
"""
