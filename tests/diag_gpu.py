"""Diagnostic (not collected by pytest): field-by-field comparison of GPU prep shares vs oracle.

python tests/diag_gpu.py [config ...]
"""
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from tests.reports import CONFIGS, make_batch  # noqa: E402


def split(v, row):
    es = v.fld.ENCODED_SIZE
    vl = v.VERIFIER_LEN
    ver = [int.from_bytes(row[i * es:(i + 1) * es].tobytes(), "little") for i in range(vl)]
    part = row[vl * es:].tobytes()
    return ver, part


def main(names):
    from janus_amd.prio3 import Prio3Gpu
    for name in names:
        n = 4 if name != "sumvec_8_1000" else 2
        b = make_batch(name, n)
        c = CONFIGS[name]
        g = Prio3Gpu(c["kind"], b.verify_key, bits=c["bits"], length=c["length"],
                     chunk_length=c["chunk"])
        for agg_id, inp, exp in ((0, b.leader_in, b.leader_prep), (1, b.helper_in, b.helper_prep)):
            st = g.new_state(agg_id, n)
            got, status = g.prepare_init(st, b.nonces, b.public, inp)
            ok = np.array_equal(got, exp)
            print(f"{name} agg{agg_id}: match={ok} status={status.tolist()}")
            if not ok:
                for r in range(min(n, 2)):
                    gv, gp = split(b.vdaf, got[r])
                    ev, ep = split(b.vdaf, exp[r])
                    print(f"  r{r} part match={gp == ep}  v match={gv[0] == ev[0]} "
                          f"p(t) match={gv[-1] == ev[-1]}  wires match="
                          f"{sum(x == y for x, y in zip(gv[1:-1], ev[1:-1]))}/{len(ev) - 2}")
                    print(f"     got v={gv[0]:x} pt={gv[-1]:x}\n     exp v={ev[0]:x} pt={ev[-1]:x}")


if __name__ == "__main__":
    main(sys.argv[1:] or ["count", "sum8", "hist4", "sumvec_small", "hist256"])
