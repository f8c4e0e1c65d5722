"""The Field128 inversion the FLP kernels use (janus_amd/csrc/inv128.h: batched Bernstein-Yang
divsteps) against x^(p-2) mod p, the exponentiation prio 0.15.1 inverts with (src/fp.rs).  The
same source the device compiles is built here for the host with g++ (no GPU needed)."""
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = (1 << 128) - 28 * (1 << 64) + 1


@pytest.fixture(scope="module")
def inv_bin(tmp_path_factory):
    out = tmp_path_factory.mktemp("inv128") / "inv128_host"
    subprocess.run(["g++", "-O2", "-std=c++17", "-Wall", "-o", str(out),
                    os.path.join(ROOT, "tests", "native", "inv128_host.cpp")], check=True)
    return str(out)


def test_inverse_matches_exponentiation(inv_bin):
    rng = random.Random(128)
    xs = [0, 1, 2, 3, P - 1, P - 2, (P + 1) // 2, 1 << 64, (1 << 64) - 1, 1 << 127,
          28 * (1 << 64) - 1, P - (1 << 64), (1 << 96) + 7]
    xs += [rng.randrange(1, P) for _ in range(20000)]
    xs += [rng.randrange(1, 1 << 32) for _ in range(500)]          # short values
    xs += [P - rng.randrange(1, 1 << 32) for _ in range(500)]      # near p
    inp = "".join(f"{x:032x}\n" for x in xs).encode()
    out = subprocess.run([inv_bin], input=inp, capture_output=True, check=True).stdout.split()
    assert len(out) == len(xs)
    for x, y in zip(xs, out):
        want = pow(x, P - 2, P) if x else 0
        assert int(y, 16) == want, hex(x)
