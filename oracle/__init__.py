"""CPU oracle -- TEST INFRASTRUCTURE ONLY (checker, never the thing measured or shipped).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import anything from this package.
"""
