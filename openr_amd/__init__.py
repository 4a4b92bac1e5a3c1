"""openr_amd — MI355X-native SPF engine for OpenR's Decision module.

The product is the HIP engine behind the C-ABI in include/openr_spf.h
(openr_amd/csrc, built to openr_amd/lib/libopenr_spf.so). This package holds
its Python binding (``engine``) and the topology/CSR mirror (``topology``).
There is no CPU fallback: importing ``engine`` without the built library, or
creating an engine without a GPU, raises.
"""
__all__ = ["engine", "topology"]
