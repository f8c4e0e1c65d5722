"""Extract the RFC 9180 base-mode vectors the reference's HPKE test uses into a small fixture.

Source (data, read at generation time only): core/src/test-vectors.json, consumed by
core/src/hpke.rs:539-615 (`decrypt_test_vectors`), which keeps mode 0 and the KEMs Janus supports
(X25519HkdfSha256 0x20, P256HkdfSha256 0x10) and opens each encryption whose nonce is the base
nonce (single-shot HPKE).  Run: python tests/golden/make_hpke_vectors.py /root/reference
"""
import json
import os
import sys

ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
src = json.load(open(os.path.join(ref, "core", "src", "test-vectors.json")))
out = []
for tv in src:
    if tv["mode"] != 0 or tv["kem_id"] not in (0x10, 0x20) or tv["aead_id"] == 0xFFFF:
        continue
    for e in tv["encryptions"]:
        if e["nonce"] != tv["base_nonce"]:
            continue
        out.append({k: tv[k] for k in ("kem_id", "kdf_id", "aead_id", "info", "enc", "pkRm",
                                        "skRm")} | {"aad": e["aad"], "ct": e["ct"], "pt": e["pt"]})
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hpke_rfc9180_vectors.json")
json.dump(out, open(path, "w"), indent=1)
print(f"{len(out)} vectors -> {path}")
