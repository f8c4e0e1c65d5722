"""k_flp_wires_mfma (byte-limb convolution on v_mfma_i32_32x32x32_i8, janus_amd/csrc/wires_mfma.h;
chunk > 64) and k_flp_wires_cols (lane per column; chunk <= 64) against the VALU wire pass
k_flp_wires (engine options wires_mfma = wires_cols = 0), which the oracle transcripts pin
(tests/test_gpu_parity.py runs every config through the default kernels).

Here: many random leader shares per shape, so the exact-integer path sees thousands of random
weights and elements (top bytes near 0xFF, all-zero and all-0xFF words, padding in the last call,
odd call counts, columns past the last 32-column tile), and non-canonical elements in every
position class.  Prep shares must be byte-identical and the same reports rejected."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# (bits, length, chunk): calls, columns per last tile
# (kind, bits, length, chunk); SumVec = 2, Histogram = 3
SHAPES = [(2, 8, 1000, 89),   # 90 calls, last call 79 of 89 columns; 3 tiles, 25 in the last
          (2, 1, 650, 100),   # 7 calls (odd: a zero-weight padding call), 4 tiles
          (2, 1, 1000, 128),  # 8 calls, 4 full tiles (no spare column)
          (2, 3, 300, 65),    # 14 calls, a 1-column last tile
          (2, 2, 3000, 300),  # 20 calls, 10 tiles, 4 waves looping over them
          # short rows (chunk <= 64): k_flp_wires_cols
          (3, 0, 256, 16),    # Histogram256 (BASELINE config C): 16 calls; v needs sum x
          (3, 0, 100, 10),    # Histogram, 10 calls
          (2, 4, 100, 32),    # 13 calls (odd), a full 32-column tile
          (2, 1, 300, 24)]    # 13 calls, padding in the last call


def _vdaf(kind, bits, length, chunk, monkeypatch, mfma, vk=bytes(range(16))):
    """mfma: the default wire passes; else the VALU k_flp_wires for every shape."""
    from janus_amd.prio3 import Prio3Gpu
    v = Prio3Gpu(kind, vk, bits=bits, length=length, chunk_length=chunk)
    if not mfma:
        v.set_option("wires_mfma", 0)
        v.set_option("wires_cols", 0)
    return v


def _random_shares(rng, n, s, meas_len, extremes):
    lin = rng.integers(0, 256, size=(n, s.leader_input_share), dtype=np.uint8)
    el = lin[:, :meas_len * 16].reshape(n, meas_len, 16)
    el[:, :, 15] &= 0x7F  # canonical (< p) unless planted below
    if extremes:
        # elements whose every byte is 0x00 / 0x7F.. / p - 1 (the largest canonical value)
        el[0, :, :] = 0
        el[1, :, :] = 0xFF
        el[1, :, 15] = 0x7F
        pm1 = (2**128 - 28 * 2**64).to_bytes(16, "little")
        el[2, :, :] = np.frombuffer(pm1, np.uint8)
    return lin


@pytest.mark.parametrize("shape", SHAPES,
                         ids=lambda s: ("sumvec_%d_%d_%d" % s[1:]) if s[0] == 2 else
                         "histogram_%d_%d" % s[2:])
def test_mfma_wires_match_valu(shape, monkeypatch):
    kind, bits, length, chunk = shape
    rng = np.random.default_rng(chunk)
    vm = _vdaf(kind, bits, length, chunk, monkeypatch, True)
    vv = _vdaf(kind, bits, length, chunk, monkeypatch, False)
    s = vm.sizes
    meas_len = bits * length if kind == 2 else length
    n = 640
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    pub = rng.integers(0, 256, size=(n, s.public_share), dtype=np.uint8)
    lin = _random_shares(rng, n, s, meas_len, extremes=True)
    # non-canonical elements: first, last, a tile boundary, the last column of a call
    bad = {5: 0, 9: meas_len - 1, 17: min(32, meas_len - 1), 33: chunk - 1,
           65: meas_len // 2}
    for r, e in bad.items():
        lin[r, e * 16:(e + 1) * 16] = 0xFF
    # >= p but top word != 2^32 - 1 cannot exist; p itself (top word 2^32 - 1) is non-canonical
    lin[77, 16 * 3:16 * 4] = np.frombuffer((2**128 - 28 * 2**64 + 1).to_bytes(16, "little"), np.uint8)
    # canonical elements the one-compare pre-filter flags (top word 2^32 - 1, value < p)
    lin[90, 16 * 7:16 * 8] = np.frombuffer((2**128 - 29 * 2**64).to_bytes(16, "little"), np.uint8)
    bad[77] = 3
    lpm, stm = vm.prepare_init(vm.new_state(0, n), nonces, pub, lin)
    lpv, stv = vv.prepare_init(vv.new_state(0, n), nonces, pub, lin)
    np.testing.assert_array_equal(stm, stv)
    for r in range(n):
        assert stm[r] == (8 if r in bad else 0), (r, stm[r])
    ok = stm == 0
    np.testing.assert_array_equal(lpm[ok], lpv[ok])


def test_mfma_wires_helper_path(monkeypatch):
    """The helper's expanded share (k_expand output, the fused helper_init path) through both
    wire kernels: identical prep messages and aggregates for real reports."""
    from tests.reports import make_batch
    b = make_batch("sumvec_8_1000", 6)
    out = []
    for mfma in (True, False):
        v = _vdaf(2, 8, 1000, 89, monkeypatch, mfma, b.verify_key)
        hs = v.new_state(1, b.n)
        agg = v.new_aggregate(1)
        msgs, st = v.helper_init(hs, b.nonces, b.public, b.helper_in, b.leader_prep, agg=agg)
        assert (st == 0).all()
        np.testing.assert_array_equal(msgs, b.prep_msg)
        a, cnt = agg.read(0)
        out.append((bytes(a), cnt))
    assert out[0] == out[1]


# (bits, entries): FixedPoint16 / 32 take both matrix-core passes (k_fpv_wires0_mfma over 4 call
# ranges, k_fpv_wires1_mfma over the raw bits); FixedPoint64 takes k_fpv_wires0_mfma and the VALU
# k_fpv_wires1
FP_SHAPES = [(16, 300), (16, 5000), (16, 37), (32, 50), (64, 20)]


@pytest.mark.parametrize("shape", FP_SHAPES, ids=lambda s: "fp%d_%d" % s)
def test_fpvec_mfma_wires_match_valu(shape):
    """FixedPoint wire passes on the matrix cores (fpvec_mfma.h) against the VALU k_fpv_wires0 /
    k_fpv_wires1 (wires_mfma = 0): random canonical leader shares (all-zero, all-0x7F.. and p - 1
    rows among them) and non-canonical elements in several position classes; identical prep
    shares and the same reports rejected."""
    from janus_amd.prio3 import Prio3Gpu
    bits, entries = shape
    vk = bytes(range(16))
    vm = Prio3Gpu.new_fixedpoint_boundedl2_vec_sum(bits, entries, vk)
    vv = Prio3Gpu.new_fixedpoint_boundedl2_vec_sum(bits, entries, vk)
    vv.set_option("wires_mfma", 0)
    s = vm.sizes
    rng = np.random.default_rng(bits * 100003 + entries)
    n = 96
    nel = (s.leader_input_share - 16) // 16  # measurement + proof elements, then the blind
    meas_len = bits * entries + 2 * bits - 2
    nonces = rng.integers(0, 256, size=(n, 16), dtype=np.uint8)
    pub = rng.integers(0, 256, size=(n, s.public_share), dtype=np.uint8)
    lin = rng.integers(0, 256, size=(n, s.leader_input_share), dtype=np.uint8)
    el = lin[:, :nel * 16].reshape(n, nel, 16)
    el[:, :, 15] &= 0x7F
    el[0, :meas_len, :] = 0
    el[1, :meas_len, :] = 0xFF
    el[1, :meas_len, 15] = 0x7F
    el[2, :meas_len, :] = np.frombuffer((2**128 - 28 * 2**64).to_bytes(16, "little"), np.uint8)
    bad = {5: 0, 9: meas_len - 1, 17: 31, 33: meas_len // 2, 41: bits * entries}
    for r, e in bad.items():
        lin[r, e * 16:(e + 1) * 16] = 0xFF
    # canonical elements the pre-filter flags (top word 2^32 - 1, value < p)
    lin[50, 16 * 7:16 * 8] = np.frombuffer((2**128 - 29 * 2**64).to_bytes(16, "little"), np.uint8)
    lpm, stm = vm.prepare_init(vm.new_state(0, n), nonces, pub, lin)
    lpv, stv = vv.prepare_init(vv.new_state(0, n), nonces, pub, lin)
    np.testing.assert_array_equal(stm, stv)
    for r in range(n):
        assert stm[r] == (8 if r in bad else 0), (r, stm[r])
    ok = stm == 0
    np.testing.assert_array_equal(lpm[ok], lpv[ok])
