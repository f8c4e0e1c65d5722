"""ctypes binding of oracle/prio3_ref.c (C restatement of prio 0.15.1 Prio3).

TEST INFRASTRUCTURE / CPU BASELINE ONLY (see prio3_ref.c header).  Used by tests/ to generate
synthetic report batches quickly and by bench.py's `cpu_baseline` leg.  PARITY UNPINNED (no prio
0.15.1 source or vectors in this container); cross-checked against oracle/prio3.py in tests.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "build" / "libprio3ref.so"
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
        l = ctypes.CDLL(str(LIB))
        P = ctypes.c_void_p
        l.p3ref_new.restype = P
        l.p3ref_new.argtypes = [ctypes.c_int, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, P]
        l.p3ref_free.argtypes = [P]
        l.p3ref_sizes.argtypes = [P, P]
        l.p3ref_gen.restype = ctypes.c_int
        l.p3ref_gen.argtypes = [P, P, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_size_t,
                                ctypes.c_int, P, P, P, P, P]
        l.p3ref_synth.restype = ctypes.c_int
        l.p3ref_synth.argtypes = [P, P, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_size_t,
                                  ctypes.c_int, P, P, P]
        l.p3ref_prepare_batch.restype = ctypes.c_longlong
        l.p3ref_prepare_batch.argtypes = [P, ctypes.c_size_t, ctypes.c_int] + [P] * 10
        _lib = l
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class Prio3Ref:
    def __init__(self, kind, verify_key, bits=0, length=0, chunk=0):
        vk = np.frombuffer(bytes(verify_key), dtype=np.uint8).copy()
        self._h = lib().p3ref_new(kind, bits, length, chunk, _p(vk))
        if not self._h:
            raise ValueError("bad Prio3 parameters")
        s = np.zeros(8, dtype=np.uint32)
        lib().p3ref_sizes(self._h, _p(s))
        (self.es, self.leader_len, self.helper_len, self.public_len, self.prep_len,
         self.msg_len, self.agg_len, self.random_size) = [int(x) for x in s]
        self.kind, self.length = kind, length

    def __del__(self):
        if getattr(self, "_h", None):
            lib().p3ref_free(self._h)
            self._h = None

    def gen(self, cfg_id: bytes, start: int, n: int, threads: int = 0):
        """n synthetic reports (SURVEY §8(d) recipe) -> dict of report-major uint8 arrays."""
        threads = threads or (os.cpu_count() or 1)
        cid = np.frombuffer(cfg_id, dtype=np.uint8).copy()
        out = dict(
            nonces=np.zeros((n, 16), np.uint8),
            public=np.zeros((n, self.public_len), np.uint8),
            leader_in=np.zeros((n, self.leader_len), np.uint8),
            helper_in=np.zeros((n, self.helper_len), np.uint8),
            meas=np.zeros((n, self.length if self.kind in (2, 4) else 1), np.uint64),
        )
        lib().p3ref_gen(self._h, _p(cid), len(cfg_id), start, n, threads, _p(out["nonces"]),
                        _p(out["public"]) if self.public_len else None, _p(out["leader_in"]),
                        _p(out["helper_in"]), _p(out["meas"]))
        return out

    def synth(self, cfg_id: bytes, start: int, n: int, threads: int = 0):
        """Inputs only (nonces, client randomness, measurements) for n synthetic reports."""
        threads = threads or (os.cpu_count() or 1)
        cid = np.frombuffer(cfg_id, dtype=np.uint8).copy()
        out = dict(nonces=np.zeros((n, 16), np.uint8),
                   rand=np.zeros((n, self.random_size), np.uint8),
                   meas=np.zeros((n, self.length if self.kind in (2, 4) else 1), np.uint64))
        lib().p3ref_synth(self._h, _p(cid), len(cfg_id), start, n, threads, _p(out["nonces"]),
                          _p(out["rand"]), _p(out["meas"]))
        return out

    def prepare_batch(self, nonces, public, leader_in, helper_in, threads=1, outputs=True):
        """Leader + helper prepare + aggregate for every report (the bench unit)."""
        n = nonces.shape[0]
        res = dict(agg_l=np.zeros(self.agg_len, np.uint8), agg_h=np.zeros(self.agg_len, np.uint8))
        if outputs:
            res.update(lprep=np.zeros((n, self.prep_len), np.uint8),
                       hprep=np.zeros((n, self.prep_len), np.uint8),
                       msgs=np.zeros((n, max(1, self.msg_len)), np.uint8),
                       status=np.zeros(n, np.uint8))
        cnt = lib().p3ref_prepare_batch(
            self._h, n, threads, _p(nonces), _p(public) if self.public_len else None,
            _p(leader_in), _p(helper_in), _p(res.get("lprep")), _p(res.get("hprep")),
            _p(res.get("msgs")) if self.msg_len else None, _p(res.get("status")),
            _p(res["agg_l"]), _p(res["agg_h"]))
        res["count"] = int(cnt)
        if outputs and not self.msg_len:
            res["msgs"] = res["msgs"][:, :0]
        return res
