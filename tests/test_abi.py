"""CPU-side checks of the C ABI: the library builds/loads and exports every symbol the header
declares (no compute calls: there is no GPU here)."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def header_symbols(names=("prio3gpu.h", "prio3gpu_test.h")):
    text = "".join((ROOT / "include" / n).read_text() for n in names)
    return sorted(set(re.findall(r"\b(prio3gpu_[a-z0-9_]+)\s*\(", text)))


def test_header_and_wrapper_agree():
    from janus_amd._lib import EXPORTED, TEST_EXPORTED
    assert sorted(EXPORTED) == header_symbols(("prio3gpu.h",))
    assert sorted(TEST_EXPORTED) == header_symbols(("prio3gpu_test.h",))


def test_product_header_declares_no_test_hooks():
    """The product ABI (what Janus binds) carries no test or device-memory helpers, and the engine
    reads no environment variable (every switch is a context option or a prio3gpu_test_* call)."""
    prod = header_symbols(("prio3gpu.h",))
    assert not [s for s in prod if s.startswith("prio3gpu_test_") or s in
                ("prio3gpu_dev_alloc", "prio3gpu_dev_free", "prio3gpu_memcpy")]
    for src in ("engine.hip", "codec.cpp", "hpke.cpp"):
        assert "getenv" not in (ROOT / "janus_amd" / "csrc" / src).read_text(), src


def test_library_exports_all_symbols():
    from janus_amd._lib import LIB_PATH, lib
    if not LIB_PATH.exists():
        pytest.skip("library not built")
    l = lib()
    for name in header_symbols():
        assert hasattr(l, name), name


def test_nm_exports():
    import subprocess
    from janus_amd._lib import LIB_PATH
    if not LIB_PATH.exists():
        pytest.skip("library not built")
    out = subprocess.run(["nm", "-D", "--defined-only", str(LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    syms = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [s for s in header_symbols() if s not in syms]
    assert not missing, missing
