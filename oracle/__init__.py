"""TEST INFRASTRUCTURE ONLY -- the CPU oracle for charpt parity tests.

Nothing in the product (``replicatinggpt_amd``) may import this package.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use it, and only as the
checker / the timed CPU baseline -- never as the thing measured or shipped.

Parity status: PINNED.  Every function here is checked against golden vectors produced by
running the reference ``GPT1.py`` itself in the build container (tests/golden/make_golden.py,
tests/test_oracle_golden.py).
"""
