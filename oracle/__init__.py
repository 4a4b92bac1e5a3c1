"""CPU oracle for the OpenR SPF path — TEST INFRASTRUCTURE ONLY.

Restates /root/reference/openr/decision/LinkState.cpp:398-419, 762-882 in C
(spf_oracle.c). Imported only by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py; never by the product package openr_amd.
"""
from .oracle import Oracle, OracleGraph, SpfRun, U64_MAX, build, default_threads, delta_digest  # noqa: F401
