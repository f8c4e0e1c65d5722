"""Generates tests/golden/prio3_transcripts.json: VdafTranscript fields (core/src/test_util/mod.rs:
50-83) for deterministic synthetic reports, computed by the CPU oracle (oracle/prio3.py).

PARITY UNPINNED: the reference (prio 0.15.1, not vendored) cannot be run here, so these vectors pin
our VDAF-07 restatement against regressions and pin the GPU path to it; they are not reference
outputs.  Large byte strings (> 4 KiB) are stored as SHA-256 digests.

python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from tests.reports import CONFIGS  # noqa: E402
from oracle import prio3 as O  # noqa: E402

SETS = [("count", 4), ("sum8", 3), ("sum32", 2), ("sumvec_small", 3), ("countvec15", 2),
        ("hist4", 3), ("hist256", 2), ("sumvec_8_1000", 1), ("fp16_3", 3), ("fp32_5", 2),
        ("fp64_4", 2)]
FIELDS = ["public_share", "leader_input_share", "helper_input_share", "leader_prep_share",
          "helper_prep_share", "prep_msg", "leader_out_share", "helper_out_share"]


def enc(b: bytes):
    if len(b) > 4096:
        return {"sha256": hashlib.sha256(b).hexdigest(), "len": len(b)}
    return b.hex()


def main():
    out = {"vdaf": "Prio3 (draft-irtf-cfrg-vdaf-07 / prio 0.15.1 restatement)", "configs": []}
    for name, n in SETS:
        cfg = CONFIGS[name]
        v = cfg["ctor"]()
        cid = f"golden-{name}".encode()
        vk = O.synth_verify_key(cid)
        reports = []
        lo, ho = [], []
        for i in range(n):
            nonce, m, rand = O.synth_report(v, cid, i)
            t = O.run_vdaf(v, vk, nonce, m, rand)
            rep = {"nonce": nonce.hex(), "measurement": m, "rand": rand.hex()}
            rep.update({k: enc(t[k]) for k in FIELDS})
            reports.append(rep)
            lo.append(v.fld.decode_vec(t["leader_out_share"]))
            ho.append(v.fld.decode_vec(t["helper_out_share"]))
        out["configs"].append({
            "name": name, "kind": cfg["kind"], "bits": cfg["bits"], "length": cfg["length"],
            "chunk_length": cfg["chunk"], "verify_key": vk.hex(), "cfg_id": cid.hex(),
            "reports": reports,
            "leader_agg_share": enc(v.fld.encode_vec(v.aggregate(lo))),
            "helper_agg_share": enc(v.fld.encode_vec(v.aggregate(ho))),
            "unsharded": v.unshard([v.aggregate(lo), v.aggregate(ho)], n),
        })
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "prio3_transcripts.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
