"""The FLP query's degenerate branches, reached through prio3gpu_test_flp_query (crafted query /
joint randomness instead of SHAKE128 output), compared with the oracle's direct flp_query
(oracle/prio3.py, prio 0.15.1 flp.rs Type::query restated):

  * a query point t with t^m == 1 (t = 1, t = a primitive m-th root and a power of it): prio's
    query fails ("invalid query randomness"), Janus maps it to VdafPrepError (error.rs:240-300);
  * a joint-rand element r with r^m == 1 (r = 1, r = alpha_m^k): k_flp_query_lane's closed-form
    gadget sum G(y) = y (y^calls - 1) / (y - 1) divides by zero there and takes its separate
    loop; the ParallelSum kernels' powers of r wrap;
  * r = 0 (every range-check term vanishes).

Parity of these values is pinned only against the oracle restatement (parity unpinned vs prio
0.15.1, as everywhere: DESIGN.md §2)."""
import ctypes

import numpy as np
import pytest

from oracle import prio3 as O

pytestmark = pytest.mark.gpu

NAMES = ["count", "sum8", "sum5", "sum64", "sumvec_small", "countvec15", "hist4", "hist256"]


def _m(typ):
    return O.gadget_m(typ.gadgets[0])


def _run(v, leader_in, t, jr, part):
    from janus_amd._lib import check, lib
    n = leader_in.shape[0]
    s = v.sizes
    prep = np.zeros((n, s.prep_share), np.uint8)
    st = np.zeros(n, np.uint8)
    P = lambda a: ctypes.c_void_p(a.ctypes.data) if a is not None else None
    check(lib().prio3gpu_test_flp_query(v._ctx, n, P(np.ascontiguousarray(leader_in)),
                                        P(np.ascontiguousarray(t)),
                                        P(np.ascontiguousarray(jr)) if jr is not None else None,
                                        P(np.ascontiguousarray(part)), P(prep), P(st)),
          "test_flp_query")
    return prep, st


@pytest.mark.parametrize("name", NAMES)
def test_crafted_query_and_joint_randomness_match_oracle(name):
    from janus_amd.prio3 import Prio3Gpu
    from tests.reports import CONFIGS, make_batch
    b = make_batch(name, 3)
    c = CONFIGS[name]
    v = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                 chunk_length=c["chunk"])
    ov = b.vdaf
    fld, typ = ov.fld, ov.typ
    p, es, m = fld.MODULUS, fld.ENCODED_SIZE, _m(typ)
    alpha = fld.root(m.bit_length() - 1)
    jr_len = typ.JOINT_RAND_LEN
    rs = [None] if jr_len == 0 else [1, pow(alpha, 5, p), 0, 0x1234567]
    ts = [0x0123456789ABCDEF % p, 1, alpha, pow(alpha, 3, p)]
    rows_in, rows_t, rows_jr, want, want_st = [], [], [], [], []
    part = bytes(range(16))
    for i in range(b.n):
        share = ov.decode_input_share(0, b.leader_in[i].tobytes())
        for t in ts:
            for r in rs:
                jr = [] if r is None else [r] + [(r * 7 + k) % p for k in range(1, jr_len)]
                rows_in.append(b.leader_in[i])
                rows_t.append(np.frombuffer(fld.encode_vec([t]), np.uint8))
                rows_jr.append(np.frombuffer(fld.encode_vec(jr), np.uint8) if jr_len else None)
                try:
                    ver = O.flp_query(typ, share.meas_share, share.proof_share, [t], jr, ov.SHARES)
                    want.append(fld.encode_vec(ver) + (part if ov.uses_jr else b""))
                    want_st.append(0)
                except ValueError:
                    want.append(None)
                    want_st.append(5)
    n = len(rows_in)
    prep, st = _run(v, np.stack(rows_in), np.stack(rows_t),
                    np.stack(rows_jr) if jr_len else None,
                    np.frombuffer(part * n, np.uint8).reshape(n, 16))
    assert st.tolist() == want_st
    for k in range(n):
        if want[k] is not None:
            assert prep[k].tobytes() == want[k], (name, k)
    assert want_st.count(5) == b.n * 3 * len(rs)  # t = 1, alpha, alpha^3: roots of unity
