"""CPU oracle for the unfolded D-ADMM forward — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / the CPU baseline, never as the product path.

Parity status: unpinned by reference outputs (the reference's tests hold no vectors for this path
and running the reference was denied here); pinned by known-answer tests derived
from the reference source and by its shipped data fixtures. See ``oracle/dadmm_oracle.c``.
"""
from .oracle import *  # noqa: F401,F403
