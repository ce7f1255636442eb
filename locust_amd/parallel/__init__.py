"""Distribution: launcher, hosts files, per-rank runners (replaces Distributor/slave.py)."""
