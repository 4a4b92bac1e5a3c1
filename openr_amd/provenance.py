"""Build provenance of the native libraries.

Each library / test binary embeds a build id ``"<hash> <file> <file> ..."`` (Makefile
``build_id``): the first 16 hex digits of sha256 over the concatenated source files it
was built from, followed by those files (paths relative to the repository root). A
binary is accepted only if the same hash over the same files of THIS tree matches, so a
run cannot silently use a library built from other sources (e.g. a stale .so shipped to
a GPU box). Set OPENR_ALLOW_STALE_BUILD=1 to downgrade the error to a warning while
iterating on sources locally.
"""
from __future__ import annotations

import hashlib
import os
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class StaleBuildError(ImportError):
    pass


def source_hash(files) -> str:
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(ROOT, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def check_build_id(build_id: str, what: str) -> str:
    """Raise StaleBuildError unless ``build_id`` matches the sources in this tree."""
    parts = build_id.split()
    if len(parts) < 2:
        raise StaleBuildError(f"{what}: no build id ({build_id!r}); rebuild with make")
    want, files = parts[0], parts[1:]
    missing = [f for f in files if not os.path.exists(os.path.join(ROOT, f))]
    got = source_hash(files) if not missing else "missing:" + ",".join(missing)
    if got != want:
        msg = (f"{what} was built from other sources (embedded {want}, tree {got}); "
               f"rebuild: python -c 'import __graft_entry__ as g; g.build()'")
        if os.environ.get("OPENR_ALLOW_STALE_BUILD") == "1":
            warnings.warn(msg)
        else:
            raise StaleBuildError(msg)
    return want
