"""The engine library is keyed on a hash of its sources and flags (janus_amd/_lib.py), not on file
times: editing a source's content forces a rebuild, touching it does not, and a library that
carries another hash (or none: a foreign build) is rejected at load.  No GPU needed."""
import os
import shutil
import time

import pytest

from janus_amd import _lib


@pytest.fixture()
def tree(tmp_path):
    csrc = tmp_path / "csrc"
    inc = tmp_path / "include"
    shutil.copytree(_lib.CSRC, csrc)
    shutil.copytree(_lib.INCLUDE, inc)
    return csrc, inc


def test_hash_follows_content_not_mtime(tree):
    csrc, inc = tree
    h0 = _lib.source_hash(csrc, inc)
    f = csrc / "keccak.h"
    os.utime(f, (time.time() + 100, time.time() + 100))  # touch: same bytes
    assert _lib.source_hash(csrc, inc) == h0
    f.write_bytes(f.read_bytes() + b"\n// edited\n")        # content change
    assert _lib.source_hash(csrc, inc) != h0
    h1 = _lib.source_hash(csrc, inc)
    (inc / "prio3gpu.h").write_bytes((inc / "prio3gpu.h").read_bytes() + b"\n")
    assert _lib.source_hash(csrc, inc) != h1
    assert _lib.source_hash(csrc, inc, flags=_lib.FLAGS + ("-DX=1",)) != \
        _lib.source_hash(csrc, inc)


def test_foreign_and_stale_libraries_need_rebuild(tmp_path):
    want = "ab" * 32
    foreign = tmp_path / "foreign.so"
    foreign.write_bytes(os.urandom(4096))
    assert _lib.embedded_hash(foreign) is None
    assert _lib.needs_rebuild(foreign, want)
    stale = tmp_path / "stale.so"
    stale.write_bytes(b"\x7fELF" + _lib.HASH_MARKER + b"cd" * 32 + b"\0" + os.urandom(64))
    assert _lib.embedded_hash(stale) == "cd" * 32
    assert _lib.needs_rebuild(stale, want)
    good = tmp_path / "good.so"
    good.write_bytes(b"\x7fELF" + _lib.HASH_MARKER + want.encode() + b"\0")
    assert not _lib.needs_rebuild(good, want)
    assert _lib.needs_rebuild(tmp_path / "missing.so", want)


def test_built_library_carries_the_sources_hash():
    if not _lib.LIB_PATH.exists():
        pytest.skip("engine library not built")
    assert _lib.embedded_hash(_lib.LIB_PATH) == _lib.source_hash()
