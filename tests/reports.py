"""Synthetic report batches + expected transcripts from the CPU oracle (test infrastructure).

`make_batch` runs the oracle's Client::shard and the full VdafTranscript (core/src/test_util/
mod.rs:87-233 `run_vdaf`) for n deterministic synthetic reports (SURVEY.md §8(d) input recipe) and
packs them into the report-major byte arrays the C ABI takes.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List

import numpy as np

from oracle import prio3 as O


CONFIGS = {
    "count": dict(kind=0, ctor=lambda: O.Prio3.new_count(), bits=0, length=0, chunk=0),
    "sum8": dict(kind=1, ctor=lambda: O.Prio3.new_sum(8), bits=8, length=0, chunk=0),
    "sum32": dict(kind=1, ctor=lambda: O.Prio3.new_sum(32), bits=32, length=0, chunk=0),
    # bits not a power of two (calls != m / 2) and the extremes of the Sum query loop
    "sum5": dict(kind=1, ctor=lambda: O.Prio3.new_sum(5), bits=5, length=0, chunk=0),
    "sum1": dict(kind=1, ctor=lambda: O.Prio3.new_sum(1), bits=1, length=0, chunk=0),
    # the paired Sum query's edges: m = 4 (generic loop), m = 8 (one 4-iteration window), m = 32
    "sum2": dict(kind=1, ctor=lambda: O.Prio3.new_sum(2), bits=2, length=0, chunk=0),
    "sum4": dict(kind=1, ctor=lambda: O.Prio3.new_sum(4), bits=4, length=0, chunk=0),
    "sum16": dict(kind=1, ctor=lambda: O.Prio3.new_sum(16), bits=16, length=0, chunk=0),
    "sum64": dict(kind=1, ctor=lambda: O.Prio3.new_sum(64), bits=64, length=0, chunk=0),
    "sumvec_small": dict(kind=2, ctor=lambda: O.Prio3.new_sum_vec(2, 10, 3), bits=2, length=10,
                         chunk=3),
    "countvec15": dict(kind=2, ctor=lambda: O.Prio3.new_sum_vec(1, 15, 3), bits=1, length=15,
                       chunk=3),
    "sumvec_8_1000": dict(kind=2, ctor=lambda: O.Prio3.new_sum_vec(8, 1000, 89), bits=8,
                          length=1000, chunk=89),
    # chunk > 64 shapes for k_flp_wires_mfma: an odd number of calls with a padded last call, a
    # chunk that is a multiple of 32 (no spare column), 65 columns (one in the last tile)
    "sumvec_odd_calls": dict(kind=2, ctor=lambda: O.Prio3.new_sum_vec(1, 650, 100), bits=1,
                             length=650, chunk=100),
    "sumvec_chunk128": dict(kind=2, ctor=lambda: O.Prio3.new_sum_vec(1, 1000, 128), bits=1,
                            length=1000, chunk=128),
    "sumvec_chunk65": dict(kind=2, ctor=lambda: O.Prio3.new_sum_vec(3, 300, 65), bits=3,
                           length=300, chunk=65),
    "hist4": dict(kind=3, ctor=lambda: O.Prio3.new_histogram(4, 2), bits=0, length=4, chunk=2),
    # ParallelSum with ONE gadget call (the batched inversion, the backward block and the MM
    # powers at their smallest) and with three
    "sumvec_calls1": dict(kind=2, ctor=lambda: O.Prio3.new_sum_vec(1, 1, 1), bits=1, length=1,
                          chunk=1),
    "hist_calls1": dict(kind=3, ctor=lambda: O.Prio3.new_histogram(2, 2), bits=0, length=2,
                        chunk=2),
    "sumvec_calls3": dict(kind=2, ctor=lambda: O.Prio3.new_sum_vec(3, 4, 4), bits=3, length=4,
                          chunk=4),
    "hist256": dict(kind=3, ctor=lambda: O.Prio3.new_histogram(256, 16), bits=0, length=256,
                    chunk=16),
    # FixedPointBoundedL2VecSum (Janus Prio3FixedPoint{16,32,64}BitBoundedL2VecSum { length })
    "fp16_3": dict(kind=4, ctor=lambda: O.Prio3.new_fixedpoint_boundedl2_vec_sum(16, 3), bits=16,
                   length=3, chunk=0),
    "fp32_5": dict(kind=4, ctor=lambda: O.Prio3.new_fixedpoint_boundedl2_vec_sum(32, 5), bits=32,
                   length=5, chunk=0),
    "fp64_4": dict(kind=4, ctor=lambda: O.Prio3.new_fixedpoint_boundedl2_vec_sum(64, 4), bits=64,
                   length=4, chunk=0),
    "fp16_300": dict(kind=4, ctor=lambda: O.Prio3.new_fixedpoint_boundedl2_vec_sum(16, 300),
                     bits=16, length=300, chunk=0),
    "fp16_5000": dict(kind=4, ctor=lambda: O.Prio3.new_fixedpoint_boundedl2_vec_sum(16, 5000),
                      bits=16, length=5000, chunk=0),
}


@dataclass
class Batch:
    name: str
    vdaf: O.Prio3
    verify_key: bytes
    n: int
    measurements: list
    nonces: np.ndarray
    public: np.ndarray
    leader_in: np.ndarray
    helper_in: np.ndarray
    leader_prep: np.ndarray
    helper_prep: np.ndarray
    prep_msg: np.ndarray
    leader_out: np.ndarray
    helper_out: np.ndarray
    rand: np.ndarray = None


def _pack(rows: List[bytes], width: int) -> np.ndarray:
    if width == 0:
        return np.zeros((len(rows), 0), dtype=np.uint8)
    return np.frombuffer(b"".join(rows), dtype=np.uint8).reshape(len(rows), width).copy()


def make_batch(name: str, n: int, cfg_id: bytes = None, start: int = 0, xof=None) -> Batch:
    """`xof`: oracle XOF class (default XofShake128; O.XofTurboShake128 for the VDAF-08+ mode)."""
    cfg = CONFIGS[name]
    v = cfg["ctor"]()
    if xof is not None:
        v.xof = xof
    cfg_id = cfg_id if cfg_id is not None else name.encode()
    vk = O.synth_verify_key(cfg_id)
    keys = ["public_share", "leader_input_share", "helper_input_share", "leader_prep_share",
            "helper_prep_share", "prep_msg", "leader_out_share", "helper_out_share"]
    cols = {k: [] for k in keys}
    nonces, meas, rands = [], [], []
    for i in range(start, start + n):
        nonce, m, rand = O.synth_report(v, cfg_id, i)
        t = O.run_vdaf(v, vk, nonce, m, rand)
        nonces.append(nonce)
        meas.append(m)
        rands.append(rand)
        for k in keys:
            cols[k].append(t[k])
    es = v.fld.ENCODED_SIZE
    return Batch(
        name=name, vdaf=v, verify_key=vk, n=n, measurements=meas,
        nonces=_pack(nonces, 16),
        public=_pack(cols["public_share"], v.public_share_len()),
        leader_in=_pack(cols["leader_input_share"], v.leader_input_share_len()),
        helper_in=_pack(cols["helper_input_share"], v.helper_input_share_len()),
        leader_prep=_pack(cols["leader_prep_share"], v.prep_share_len()),
        helper_prep=_pack(cols["helper_prep_share"], v.prep_share_len()),
        prep_msg=_pack(cols["prep_msg"], v.prep_msg_len()),
        leader_out=_pack(cols["leader_out_share"], v.typ.OUTPUT_LEN * es),
        helper_out=_pack(cols["helper_out_share"], v.typ.OUTPUT_LEN * es),
        rand=_pack(rands, v.random_size()),
    )


def meas_array(b: Batch) -> np.ndarray:
    """Measurements as the (n, words) array prio3gpu_shard takes (uint64; FixedPoint vectors:
    int64 raw two's-complement entries)."""
    from oracle.prio3 import FixedPointBoundedL2VecSum
    if isinstance(b.vdaf.typ, FixedPointBoundedL2VecSum):
        return np.array(b.measurements, dtype=np.int64)
    if isinstance(b.measurements[0], list):
        return np.array(b.measurements, dtype=np.uint64)
    return np.array(b.measurements, dtype=np.uint64).reshape(-1, 1)


def expected_aggregate(b: Batch, which: str, mask=None, slots=None, slot=0) -> bytes:
    """Sum of the selected reports' output shares (oracle Aggregator::aggregate)."""
    v = b.vdaf
    outs = b.leader_out if which == "leader" else b.helper_out
    sel = []
    for r in range(b.n):
        if mask is not None and not mask[r]:
            continue
        if slots is not None and slots[r] != slot:
            continue
        sel.append(v.fld.decode_vec(outs[r].tobytes()))
    return v.fld.encode_vec(v.aggregate(sel)), len(sel)


def plaintext_sum(b: Batch, mask=None):
    """What unshard(aggregate) must equal (integration_tests/tests/common/mod.rs:225-398)."""
    from oracle.prio3 import Count, FixedPointBoundedL2VecSum, Histogram, Sum, SumVec
    typ = b.vdaf.typ
    ms = [m for r, m in enumerate(b.measurements) if mask is None or mask[r]]
    if isinstance(typ, FixedPointBoundedL2VecSum):
        # exact: sum of the fixed-point values (integers / 2^(bits-1)) as floats
        sums = [sum(col) for col in zip(*ms)] if ms else [0] * typ.entries
        return [s * 2.0 ** (1 - typ.bits) for s in sums]
    if isinstance(typ, (Count, Sum)):
        return sum(ms)
    if isinstance(typ, SumVec):
        return [sum(col) for col in zip(*ms)] if ms else [0] * typ.length
    if isinstance(typ, Histogram):
        out = [0] * typ.length
        for m in ms:
            out[m] += 1
        return out
    raise TypeError(typ)
