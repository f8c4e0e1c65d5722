"""tools/gen_keccak_asm.py's bank-aware inline-assembly Keccak-f[1600] (a round-5 A/B study, measured
no faster and not part of the engine): the generated instructions, interpreted on
32-bit integers, equal a plain Keccak-f[1600], which is itself pinned by hashlib's SHAKE128."""
import hashlib
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gen():
    spec = importlib.util.spec_from_file_location("gen_keccak_asm",
                                                  os.path.join(ROOT, "tools", "gen_keccak_asm.py"))
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)
    return g


def test_reference_keccak_matches_shake128():
    g = _gen()
    st = [0] * 25
    st[0] ^= 0x1F
    st[20] ^= 0x8000000000000000
    out = g.keccak_f_ref(st)
    assert b"".join(x.to_bytes(8, "little") for x in out[:4]) == hashlib.shake_128(b"").digest(32)


def test_generated_asm_is_keccak_f(tmp_path):
    g = _gen()
    out = str(tmp_path / "keccak_asm.h")
    g.main(out)
    for seed in (1, 2, 3):
        assert g.selftest(path=out, seed=seed)
        assert g.selftest_rolled(path=out, seed=seed)
