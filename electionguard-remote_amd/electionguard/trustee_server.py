"""Remote decrypting trustee process — ``RunRemoteDecryptingTrustee.main``
(src/main/java/electionguard/decrypt/RunRemoteDecryptingTrustee.java:58-120), GPU-backed.

    python -m electionguard.trustee_server --trusteeFile guardian1.json [--port 0]

One process per guardian, one GPU per process (pin it with HIP_VISIBLE_DEVICES).  Prints
``PORT <n>`` once serving; exits after the mediator's ``finish`` RPC (:274-276).  The
trustee file is this build's JSON restatement of the key-ceremony output (the reference
reads it with upstream ``readTrustee``, :90 — record I/O is out of scope).
"""
from __future__ import annotations

import argparse
import json
import sys


def load_trustee_file(path):
    from .keyceremony import GuardianKeys

    d = json.loads(open(path).read())
    g = GuardianKeys(d["id"], d["x"], [int(a, 16) for a in d["coeffs"]], [int(k, 16) for k in d["commitments"]],
                     {}, {k: (int(v[0], 16), bytes.fromhex(v[1]), bytes.fromhex(v[2]))
                          for k, v in d["backups_from"].items()})
    comm = {k: [int(x, 16) for x in v] for k, v in d["all_commitments"].items()}
    return g, comm


def write_trustee_file(path, g, all_commitments):
    json.dump({"id": g.gid, "x": g.x, "coeffs": [hex(a) for a in g.coeffs],
               "commitments": [hex(k) for k in g.commitments],
               # the other guardians' shares travel only as their encrypted backups
               "backups_from": {k: [hex(c0), c1.hex(), c2.hex()] for k, (c0, c1, c2) in g.backups_from.items()},
               "all_commitments": {k: [hex(x) for x in v] for k, v in all_commitments.items()}},
              open(path, "w"))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--trusteeFile", required=True)
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=600.0)
    a = ap.parse_args(argv)
    from .core import productionGroup
    from .decrypt import DecryptingTrustee
    from .remote import DecryptingTrusteeServer

    group = productionGroup(a.device)
    g, comm = load_trustee_file(a.trusteeFile)
    srv = DecryptingTrusteeServer(group, DecryptingTrustee(group, g, comm), port=a.port).start()
    print(f"PORT {srv.port}", flush=True)
    ok = srv.wait(a.timeout)
    srv.stop()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
