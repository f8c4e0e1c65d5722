"""CPU-side checks of the C ABI: the library builds/loads and exports every symbol the header
declares (no compute calls: there is no GPU here)."""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def header_symbols():
    text = (ROOT / "include" / "prio3gpu.h").read_text()
    return sorted(set(re.findall(r"\b(prio3gpu_[a-z0-9_]+)\s*\(", text)))


def test_header_and_wrapper_agree():
    from janus_amd._lib import EXPORTED
    assert sorted(EXPORTED) == header_symbols()


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
