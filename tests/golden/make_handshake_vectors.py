#!/usr/bin/env python3
"""Extract the Noise_*_25519_ChaChaPoly_BLAKE2b test vectors of the reference
(/root/reference/tests/vectors/*.json, cacophony/snow format: data, not code)
into tests/golden/handshake_vectors.tsv for tests/cpp/handshake_test.cpp.
Runs only in the build container (the reference is not on the GPU box).

One line per vector, tab-separated, '-' for an absent field:
  protocol_name init_prologue init_psks init_static init_ephemeral
  init_remote_static resp_prologue resp_psks resp_static resp_ephemeral
  resp_remote_static handshake_hash messages
psks: comma-separated hex; messages: comma-separated payload:ciphertext hex.
"""
import glob
import json
import os

VEC_DIR = "/root/reference/tests/vectors"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "handshake_vectors.tsv")
FIELDS = ["init_prologue", "init_psks", "init_static", "init_ephemeral", "init_remote_static",
          "resp_prologue", "resp_psks", "resp_static", "resp_ephemeral", "resp_remote_static",
          "handshake_hash"]


def main():
    files = sorted(glob.glob(os.path.join(VEC_DIR, "Noise_*_25519_ChaChaPoly_BLAKE2b*.json")))
    if not files:
        raise SystemExit("no vectors under %s (build container only)" % VEC_DIR)
    rows = []
    for f in files:
        v = json.load(open(f))
        row = [v["protocol_name"]]
        for k in FIELDS:
            x = v.get(k)
            if x is None:
                row.append("-")
            elif isinstance(x, list):
                row.append(",".join(x) if x else "-")
            else:
                row.append(x if x else "-")
        row.append(",".join("%s:%s" % (m["payload"] or "", m["ciphertext"]) for m in v["messages"]))
        rows.append("\t".join(row))
    with open(OUT, "w") as fh:
        fh.write("\n".join(rows) + "\n")
    print("%d vectors -> %s" % (len(rows), OUT))


if __name__ == "__main__":
    main()
