"""Test infrastructure only: CPU restatements of the reference's hot path
(the checker, never the product).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this package."""
