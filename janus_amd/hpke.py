"""HPKE for the aggregate-init path, host side: the Python mirror of Janus's
`core/src/hpke.rs` over the native RFC 9180 implementation in libprio3gpu.so
(janus_amd/csrc/hpke.cpp; C ABI include/prio3gpu.h).

  Label / HpkeApplicationInfo        core/src/hpke.rs:44-77
  seal / open                        core/src/hpke.rs:158-202
  generate_hpke_config_and_private_key   core/src/hpke.rs:204-231
  HpkeKeypair                        core/src/hpke.rs:233-255
  open_report_shares                 the helper's per-report open loop, batched over host threads
                                     (aggregator/src/aggregator.rs:1634-1700)

Errors: `HpkeError` where hpke::open / hpke::seal return `Error::Hpke`, `ValueError` for an
unsupported suite (`Error::InvalidConfiguration`).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from ._lib import lib

# HpkeKemId / HpkeKdfId / HpkeAeadId (messages/src/lib.rs)
KEM_X25519_HKDF_SHA256, KEM_P256_HKDF_SHA256 = 0x20, 0x10
KDF_HKDF_SHA256, KDF_HKDF_SHA384, KDF_HKDF_SHA512 = 1, 2, 3
AEAD_AES128GCM, AEAD_AES256GCM, AEAD_CHACHA20POLY1305 = 1, 2, 3
# Role (messages/src/lib.rs:495-500)
ROLE_COLLECTOR, ROLE_CLIENT, ROLE_LEADER, ROLE_HELPER = 0, 1, 2, 3

_E_HPKE, _E_UNSUPPORTED, _E_CAPACITY = -5, -6, -4


class HpkeError(Exception):
    pass


class Label:
    INPUT_SHARE = b"dap-07 input share"
    AGGREGATE_SHARE = b"dap-07 aggregate share"


def application_info(label: bytes, sender_role: int, recipient_role: int) -> bytes:
    """HpkeApplicationInfo::new (core/src/hpke.rs:64-77)."""
    return bytes(label) + bytes([sender_role, recipient_role])


@dataclass(frozen=True)
class HpkeConfig:
    id: int
    kem_id: int
    kdf_id: int
    aead_id: int
    public_key: bytes


@dataclass(frozen=True)
class HpkeKeypair:
    config: HpkeConfig
    private_key: bytes


def _buf(b: bytes):
    return ctypes.c_char_p(bytes(b)) if b else None


def _rc(rc: int, what: str) -> None:
    if rc == _E_UNSUPPORTED:
        raise ValueError(f"{what}: unsupported HPKE suite")
    if rc == _E_HPKE:
        raise HpkeError(f"{what} failed")
    if rc != 0:
        raise RuntimeError(f"{what}: error {rc}")


def public_key(kem_id: int, private_key: bytes) -> bytes:
    out = ctypes.create_string_buffer(65)
    ln = ctypes.c_size_t()
    _rc(lib().prio3gpu_hpke_public_key(kem_id, _buf(private_key), len(private_key), out, 65,
                                       ctypes.byref(ln)), "public key")
    return out.raw[:ln.value]


def generate_hpke_config_and_private_key(config_id: int, kem_id: int = KEM_X25519_HKDF_SHA256,
                                         kdf_id: int = KDF_HKDF_SHA256,
                                         aead_id: int = AEAD_AES128GCM) -> HpkeKeypair:
    for _ in range(64):  # P-256: rejection-sample a scalar in [1, n)
        sk = os.urandom(32)
        try:
            pk = public_key(kem_id, sk)
        except HpkeError:
            continue
        return HpkeKeypair(HpkeConfig(config_id, kem_id, kdf_id, aead_id, pk), sk)
    raise HpkeError("key generation failed")


def seal(config: HpkeConfig, info: bytes, plaintext: bytes, aad: bytes,
         ephemeral_private_key: Optional[bytes] = None):
    """-> (config id, encapsulated key, payload) = HpkeCiphertext fields."""
    enc = ctypes.create_string_buffer(65)
    ct = ctypes.create_string_buffer(len(plaintext) + 16)
    el, cl = ctypes.c_size_t(), ctypes.c_size_t()
    ske = ephemeral_private_key
    _rc(lib().prio3gpu_hpke_seal(config.kem_id, config.kdf_id, config.aead_id,
                                 _buf(config.public_key), len(config.public_key), _buf(ske),
                                 len(ske) if ske else 0, _buf(info), len(info), _buf(aad),
                                 len(aad), _buf(plaintext), len(plaintext), enc, 65,
                                 ctypes.byref(el), ct, len(ct), ctypes.byref(cl)), "HPKE seal")
    return config.id, enc.raw[:el.value], ct.raw[:cl.value]


def open_(keypair: HpkeKeypair, info: bytes, enc: bytes, payload: bytes, aad: bytes) -> bytes:
    c = keypair.config
    n = max(0, len(payload) - 16)
    pt = ctypes.create_string_buffer(max(1, n))
    ln = ctypes.c_size_t()
    _rc(lib().prio3gpu_hpke_open(c.kem_id, c.kdf_id, c.aead_id, _buf(keypair.private_key),
                                 len(keypair.private_key), _buf(c.public_key), len(c.public_key),
                                 _buf(enc), len(enc), _buf(info), len(info), _buf(aad), len(aad),
                                 _buf(payload), len(payload), pt, n, ctypes.byref(ln)),
        "HPKE open")
    return pt.raw[:ln.value]


class _Keypair(ctypes.Structure):
    _fields_ = [("config_id", ctypes.c_uint8), ("kem_id", ctypes.c_uint16),
                ("kdf_id", ctypes.c_uint16), ("aead_id", ctypes.c_uint16),
                ("public_key", ctypes.c_void_p), ("public_key_len", ctypes.c_uint32),
                ("private_key", ctypes.c_void_p), ("private_key_len", ctypes.c_uint32)]


def _keypairs(kps: Sequence[HpkeKeypair]):
    arr = (_Keypair * max(1, len(kps)))()
    keep = []
    for i, kp in enumerate(kps):
        pk = ctypes.create_string_buffer(kp.config.public_key, len(kp.config.public_key))
        sk = ctypes.create_string_buffer(kp.private_key, len(kp.private_key))
        keep += [pk, sk]
        c = kp.config
        arr[i] = _Keypair(c.id, c.kem_id, c.kdf_id, c.aead_id, ctypes.addressof(pk), len(pk.raw),
                          ctypes.addressof(sk), len(sk.raw))
    return arr, keep


def input_share_aad(task_id: bytes, report_id: bytes, time: int, public_share: bytes) -> bytes:
    """InputShareAad encoding (messages/src/lib.rs:1790-1827)."""
    return (bytes(task_id) + bytes(report_id) + int(time).to_bytes(8, "big")
            + len(public_share).to_bytes(4, "big") + bytes(public_share))


def open_report_shares(task_id: bytes, req, task_keys: Sequence[HpkeKeypair],
                       global_keys: Sequence[HpkeKeypair] = (),
                       status: Optional[np.ndarray] = None, threads: int = 0,
                       recipient_role: int = ROLE_HELPER):
    """Open every encrypted input share of a decoded AggregationJobInitializeReq
    (`janus_amd.codec.AggInitReq`) on `threads` host threads (0: all cores).

    -> (plaintexts uint8 array, offsets (n + 1), status); report i's PlaintextInputShare is
    plaintexts[offsets[i]:offsets[i+1]] -- the input of codec.decode_plaintext_input_shares_raw.
    Status 3 = HpkeUnknownConfigId, 4 = HpkeDecryptError (aggregator.rs:1634-1700)."""
    n = req.n
    st = np.zeros(n, np.uint8) if status is None else status
    offs = np.zeros(n + 1, np.uint64)
    tid = np.frombuffer(bytes(task_id), np.uint8).copy()
    assert tid.size == 32, "TaskId is 32 bytes"
    tk, keep_t = _keypairs(task_keys)
    gk, keep_g = _keypairs(global_keys)
    L = lib()
    _rc(L.prio3gpu_hpke_open_report_shares(tid.ctypes.data, tk, len(task_keys), gk,
                                           len(global_keys), ROLE_CLIENT, recipient_role,
                                           req.raw.ctypes.data, req.views, n, None,
                                           offs.ctypes.data, st.ctypes.data, threads), "size")
    pts = np.zeros(max(1, int(offs[-1])), np.uint8)
    _rc(L.prio3gpu_hpke_open_report_shares(tid.ctypes.data, tk, len(task_keys), gk,
                                           len(global_keys), ROLE_CLIENT, recipient_role,
                                           req.raw.ctypes.data, req.views, n, pts.ctypes.data,
                                           offs.ctypes.data, st.ctypes.data, threads),
        "open report shares")
    del keep_t, keep_g
    return pts, offs, st
