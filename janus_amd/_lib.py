"""Loader for the in-tree HIP library `janus_amd/lib/libprio3gpu.so` (C ABI: include/prio3gpu.h).

There is no CPU fallback: if the library is missing or cannot be loaded, every entry point raises.
Build it with `python -c "import __graft_entry__ as g; g.build()"` (hipcc, gfx950).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent
LIB_DIR = ROOT / "lib"
LIB_PATH = LIB_DIR / "libprio3gpu.so"
# Tuning experiments may point at another build of the same library (still the HIP engine).
if os.environ.get("PRIO3GPU_LIB"):
    LIB_PATH = Path(os.environ["PRIO3GPU_LIB"]).resolve()
CSRC = ROOT / "csrc"
INCLUDE = ROOT.parent / "include"

_lib = None


class Prio3GpuError(RuntimeError):
    pass


class InvalidMessage(Prio3GpuError):
    """The whole request is invalid (Janus `Error::InvalidMessage`, DAP "invalidMessage"):
    duplicate report IDs, a non-empty Prio3 aggregation parameter (aggregator.rs:1588-1605)."""


class EmptyAggregation(Prio3GpuError):
    """An aggregation job without reports (Janus `Error::EmptyAggregation`, aggregator.rs:1851-1863)."""


E_INVALID_MESSAGE = -7

SOURCES = ("engine.hip", "codec.cpp", "hpke.cpp")
FLAGS = ("--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared")
LIBS = ("-lrccl", "-lcrypto")
HASH_MARKER = b"PRIO3GPU_BUILD_HASH="


def source_hash(csrc: Path = CSRC, include: Path = INCLUDE, flags=FLAGS) -> str:
    """SHA-256 (hex) over the engine's sources, its headers and the compiler flags: the build key
    (file mtimes are not: a tree copied to another machine keeps its library only if the
    contents it was built from are unchanged)."""
    import hashlib
    h = hashlib.sha256()
    files = ([csrc / s for s in SOURCES] + sorted(csrc.glob("*.h"))
             + [include / "prio3gpu.h", include / "prio3gpu_test.h"])
    for p in files:
        h.update(p.name.encode() + b"\0" + p.read_bytes() + b"\0")
    h.update(" ".join(flags + LIBS).encode())
    return h.hexdigest()


def embedded_hash(path: Path = LIB_PATH):
    """The build hash a library carries (its `prio3gpu_build_id` marker), read from the file
    without loading it; None if the file is missing or carries no marker (a foreign library)."""
    try:
        data = Path(path).read_bytes()
    except OSError:
        return None
    i = data.find(HASH_MARKER)
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i + len(HASH_MARKER):j].decode(errors="replace")


def needs_rebuild(path: Path = LIB_PATH, want=None) -> bool:
    return embedded_hash(path) != (want or source_hash())


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile the HIP engine for gfx950 into janus_amd/lib/libprio3gpu.so, unless the library
    there was built from exactly these sources and flags (its embedded build hash)."""
    want = source_hash()
    if not force and not needs_rebuild(LIB_PATH, want):
        return LIB_PATH
    LIB_DIR.mkdir(exist_ok=True)
    tmp = LIB_PATH.with_suffix(".so.tmp")
    cmd = (["hipcc"] + list(FLAGS) + [f'-DPRIO3GPU_BUILD_HASH="{want}"', "-o", str(tmp)]
           + [str(CSRC / s) for s in SOURCES] + list(LIBS))
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


def _declare(lib):
    c = ctypes
    P = c.c_void_p
    u8p = c.c_void_p
    sigs = {
        "prio3gpu_ctx_create": (c.c_int, [c.c_int, c.c_uint32, c.c_uint32, c.c_uint32, c.c_char_p,
                                          c.c_int, c.POINTER(P)]),
        "prio3gpu_ctx_create2": (c.c_int, [c.c_int, c.c_uint32, c.c_uint32, c.c_uint32,
                                           c.c_char_p, c.c_int, c.c_int, c.POINTER(P)]),
        "prio3gpu_ctx_destroy": (c.c_int, [P]),
        "prio3gpu_ctx_set_async": (c.c_int, [P, c.c_int]),
        "prio3gpu_ctx_set_option": (c.c_int, [P, c.c_char_p, c.c_int64]),
        "prio3gpu_ctx_wait": (c.c_int, [P, P]),
        "prio3gpu_ctx_mark": (c.c_int, [P, c.POINTER(c.c_int)]),
        "prio3gpu_ctx_wait_mark": (c.c_int, [P, P, c.c_int]),
        "prio3gpu_prepare_init_xof": (c.c_int, [P, P, c.c_size_t, u8p, u8p, u8p, u8p]),
        "prio3gpu_prepare_init_query": (c.c_int, [P, P, c.c_size_t, u8p, u8p]),
        "prio3gpu_prepare_init_weights": (c.c_int, [P, P, c.c_size_t, u8p]),
        "prio3gpu_ctx_sizes": (c.c_int, [P, P]),
        "prio3gpu_ctx_sync": (c.c_int, [P]),
        "prio3gpu_ctx_stream": (P, [P]),
        "prio3gpu_state_create": (c.c_int, [P, c.c_int, c.c_size_t, c.POINTER(P)]),
        "prio3gpu_state_destroy": (c.c_int, [P]),
        "prio3gpu_state_set_input_pitch": (c.c_int, [P, c.c_size_t]),
        "prio3gpu_agg_create": (c.c_int, [P, c.c_uint32, c.POINTER(P)]),
        "prio3gpu_agg_destroy": (c.c_int, [P]),
        "prio3gpu_agg_reset": (c.c_int, [P]),
        "prio3gpu_agg_read": (c.c_int, [P, c.c_uint32, u8p, c.POINTER(c.c_uint64)]),
        "prio3gpu_agg_merge_bytes": (c.c_int, [P, c.c_uint32, u8p, c.c_uint64]),
        "prio3gpu_agg_update_reports": (c.c_int, [P, c.c_size_t, u8p, P, u8p, P]),
        "prio3gpu_agg_read_reports": (c.c_int, [P, c.c_uint32, u8p, c.POINTER(c.c_uint64),
                                                c.POINTER(c.c_uint64)]),
        "prio3gpu_prepare_init": (c.c_int, [P, P, c.c_size_t, u8p, u8p, u8p, u8p, u8p]),
        "prio3gpu_prepare_shares_to_prepare_message": (c.c_int, [P, c.c_size_t, u8p, u8p, u8p, u8p]),
        "prio3gpu_prepare_next": (c.c_int, [P, P, c.c_size_t, u8p, u8p, u8p, P, P]),
        "prio3gpu_helper_init": (c.c_int, [P, P, c.c_size_t, u8p, u8p, u8p, u8p, P, u8p, u8p, P]),
        "prio3gpu_random_size": (c.c_int, [P]),
        "prio3gpu_shard": (c.c_int, [P, P, c.c_size_t, u8p, P, u8p, u8p, u8p, u8p]),
        "prio3gpu_comm_unique_id": (c.c_int, [u8p]),
        "prio3gpu_comm_init": (c.c_int, [u8p, c.c_int, c.c_int, c.c_int, c.POINTER(P)]),
        "prio3gpu_comm_destroy": (c.c_int, [P]),
        "prio3gpu_agg_allreduce": (c.c_int, [P, P, P, P]),
        "prio3gpu_agg_epoch_merge": (c.c_int, [P, P, P, P, c.c_uint32, P]),
        "prio3gpu_prof_enable": (c.c_int, [P, c.c_int]),
        "prio3gpu_prof_read": (c.c_int, [P, P, P, c.c_int]),
        "prio3gpu_prof_kernel_name": (c.c_char_p, [c.c_int]),
        "prio3gpu_test_squeeze": (c.c_int, [c.c_int, P, c.c_size_t, c.c_uint32, u8p, c.c_int]),
        "prio3gpu_test_flp_query": (c.c_int, [P, c.c_size_t, u8p, u8p, u8p, u8p, u8p, u8p]),
        "prio3gpu_dev_alloc": (c.c_int, [P, c.c_size_t, c.POINTER(P)]),
        "prio3gpu_dev_free": (c.c_int, [P, P]),
        "prio3gpu_memcpy": (c.c_int, [P, P, P, c.c_size_t]),
        "prio3gpu_test_hpke_set_ifma": (c.c_int, [c.c_int]),
        "prio3gpu_last_error": (c.c_char_p, []),
        "prio3gpu_build_hash": (c.c_char_p, []),
        "prio3gpu_unshard": (c.c_int, [P, u8p, c.c_size_t, c.c_uint64, u8p, P]),
        # DAP codec edge (host-only, codec.cpp)
        "prio3gpu_decode_agg_init_req": (c.c_int, [u8p, c.c_size_t, c.c_int, u8p, P, P, c.c_size_t,
                                                   c.POINTER(c.c_size_t)]),
        "prio3gpu_gather_prepare_inits": (c.c_int, [P, u8p, P, c.c_size_t, u8p, u8p, u8p, u8p]),
        "prio3gpu_apply_faults": (c.c_int, [c.c_size_t, u8p, u8p]),
        "prio3gpu_batch_aggregation_merge": (c.c_int, [c.c_uint32, c.c_size_t, P, P]),
        "prio3gpu_check_agg_init_req": (c.c_int, [u8p, P, c.c_size_t, c.c_uint64]),
        "prio3gpu_decode_plaintext_input_shares": (c.c_int, [P, u8p, P, c.c_size_t, c.c_int, u8p,
                                                             u8p]),
        "prio3gpu_encode_agg_job_resp": (c.c_int, [u8p, u8p, c.c_uint32, u8p, c.c_size_t, u8p,
                                                   c.c_size_t, c.POINTER(c.c_size_t)]),
        "prio3gpu_encode_agg_init_req": (c.c_int, [c.c_int, u8p, u8p, c.c_uint32, c.c_size_t, u8p,
                                                   P, u8p, c.c_uint32, u8p, u8p, P, u8p, P, u8p,
                                                   c.c_uint32, u8p, u8p, c.c_size_t,
                                                   c.POINTER(c.c_size_t)]),
        "prio3gpu_decode_agg_job_resp": (c.c_int, [u8p, c.c_size_t, P, c.c_size_t,
                                                   c.POINTER(c.c_size_t)]),
        "prio3gpu_gather_helper_resps": (c.c_int, [P, u8p, P, c.c_size_t, u8p, c.c_size_t, u8p,
                                                   u8p]),
        # HPKE on host threads (hpke.cpp)
        "prio3gpu_hpke_open": (c.c_int, [c.c_uint16, c.c_uint16, c.c_uint16, u8p, c.c_size_t, u8p,
                                         c.c_size_t, u8p, c.c_size_t, u8p, c.c_size_t, u8p,
                                         c.c_size_t, u8p, c.c_size_t, u8p, c.c_size_t,
                                         c.POINTER(c.c_size_t)]),
        "prio3gpu_hpke_seal": (c.c_int, [c.c_uint16, c.c_uint16, c.c_uint16, u8p, c.c_size_t, u8p,
                                         c.c_size_t, u8p, c.c_size_t, u8p, c.c_size_t, u8p,
                                         c.c_size_t, u8p, c.c_size_t, c.POINTER(c.c_size_t), u8p,
                                         c.c_size_t, c.POINTER(c.c_size_t)]),
        "prio3gpu_hpke_public_key": (c.c_int, [c.c_uint16, u8p, c.c_size_t, u8p, c.c_size_t,
                                               c.POINTER(c.c_size_t)]),
        "prio3gpu_x25519_batch": (c.c_int, [u8p, u8p, c.c_size_t, u8p, c.c_int]),
        "prio3gpu_hpke_open_report_shares": (c.c_int, [u8p, P, c.c_size_t, P, c.c_size_t,
                                                       c.c_uint8, c.c_uint8, u8p, P, c.c_size_t,
                                                       u8p, P, u8p, c.c_int]),
    }
    for name, (res, args) in sigs.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return sigs


# Every symbol include/prio3gpu.h declares (the product ABI; checked by tests/test_abi.py).
EXPORTED = [
    "prio3gpu_ctx_create", "prio3gpu_ctx_create2", "prio3gpu_ctx_destroy", "prio3gpu_ctx_sizes",
    "prio3gpu_ctx_sync", "prio3gpu_ctx_set_async", "prio3gpu_ctx_set_option", "prio3gpu_ctx_wait",
    "prio3gpu_ctx_mark",
    "prio3gpu_ctx_wait_mark",
    "prio3gpu_prepare_init_xof", "prio3gpu_prepare_init_query", "prio3gpu_prepare_init_weights",
    "prio3gpu_ctx_stream", "prio3gpu_state_create", "prio3gpu_state_destroy",
    "prio3gpu_state_set_input_pitch",
    "prio3gpu_agg_create", "prio3gpu_agg_destroy", "prio3gpu_agg_reset", "prio3gpu_agg_read",
    "prio3gpu_agg_merge_bytes", "prio3gpu_agg_update_reports", "prio3gpu_agg_read_reports",
    "prio3gpu_prepare_init",
    "prio3gpu_prepare_shares_to_prepare_message", "prio3gpu_prepare_next", "prio3gpu_helper_init",
    "prio3gpu_random_size", "prio3gpu_shard", "prio3gpu_comm_unique_id", "prio3gpu_comm_init", "prio3gpu_comm_destroy",
    "prio3gpu_agg_allreduce", "prio3gpu_agg_epoch_merge", "prio3gpu_prof_enable",
    "prio3gpu_prof_read",
    "prio3gpu_prof_kernel_name",
    "prio3gpu_last_error", "prio3gpu_build_hash", "prio3gpu_unshard", "prio3gpu_decode_agg_init_req", "prio3gpu_gather_prepare_inits",
    "prio3gpu_apply_faults", "prio3gpu_check_agg_init_req", "prio3gpu_batch_aggregation_merge",
    "prio3gpu_decode_plaintext_input_shares", "prio3gpu_encode_agg_job_resp",
    "prio3gpu_encode_agg_init_req", "prio3gpu_decode_agg_job_resp", "prio3gpu_gather_helper_resps",
    "prio3gpu_hpke_open", "prio3gpu_hpke_seal", "prio3gpu_hpke_public_key",
    "prio3gpu_hpke_open_report_shares", "prio3gpu_x25519_batch",
]
# The test / benchmark hooks of include/prio3gpu_test.h (same library, not part of the product ABI).
TEST_EXPORTED = [
    "prio3gpu_test_squeeze", "prio3gpu_test_flp_query", "prio3gpu_dev_alloc", "prio3gpu_dev_free",
    "prio3gpu_memcpy", "prio3gpu_test_hpke_set_ifma",
]


def lib():
    """The loaded HIP library; raises Prio3GpuError when it is absent (no fallback)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise Prio3GpuError(f"HIP library not built: {LIB_PATH} (run __graft_entry__.build())")
        if not os.environ.get("PRIO3GPU_LIB"):  # A/B variants name their own build
            got, want = embedded_hash(LIB_PATH), source_hash()
            if got != want:
                raise Prio3GpuError(f"stale or foreign library {LIB_PATH}: build hash {got} is "
                                    f"not the sources' {want} (run __graft_entry__.build())")
        try:
            l = ctypes.CDLL(str(LIB_PATH))
        except OSError as e:
            raise Prio3GpuError(f"cannot load {LIB_PATH}: {e}") from e
        _declare(l)
        _lib = l
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().prio3gpu_last_error().decode(errors="replace")
        cls = InvalidMessage if rc == E_INVALID_MESSAGE else Prio3GpuError
        raise cls(f"{what} failed ({rc}): {msg}")
