"""CPU oracle for the xsknf checksummer path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / reported CPU baseline.  The product
(xsknf_amd/) never imports it.
"""
