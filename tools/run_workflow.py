"""End-to-end remote workflow — ``RunRemoteWorkflowTest.main``
(src/test/java/electionguard/workflow/RunRemoteWorkflowTest.java:83-192) on the GPU path:

  1 key ceremony (in-process; commitments, Schnorr proofs and share backups made and
    checked on the GPU)                     2 encrypt ballots (GPU)
  3 accumulate tally + verify ballots (GPU)
  4 remote decryption: one trustee PROCESS per available guardian over gRPC on localhost,
    missing guardians compensated (RunRemoteDecryptionTest.java:63-136)
  5 check the decrypted counts against the plaintext votes (the reference only prints)

    python tools/run_workflow.py -nguardians 3 -quorum 3 -nballots 25            # configs[0]
    python tools/run_workflow.py -nguardians 5 -quorum 3 -navailable 3 -nballots 100   # configs[3]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-nguardians", type=int, default=3)
    ap.add_argument("-quorum", type=int, default=3)
    ap.add_argument("-navailable", type=int, default=0)
    ap.add_argument("-nballots", type=int, default=25)
    ap.add_argument("-ngpus", type=int, default=1, help="trustee k runs on GPU k % ngpus")
    a = ap.parse_args()
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.core import productionGroup
    from electionguard.decrypt import Decryption
    from electionguard.keyceremony import key_ceremony, verify_backups, verify_commitment_proofs
    from electionguard.remote import RemoteDecryptingTrusteeProxy
    from electionguard.trustee_server import write_trustee_file

    t_all = time.time()
    G = productionGroup(0)
    navail = a.navailable or a.quorum
    t = time.time()
    gk, K = key_ceremony(G, a.nguardians, a.quorum)
    comm = {g.gid: g.commitments for g in gk}
    kc_ok = all(verify_commitment_proofs(G, [k for g in gk for k in g.commitments], [pr for g in gk for pr in g.proofs]))
    kc_ok = kc_ok and all(all(verify_backups(G, g, comm).values()) for g in gk)
    print(f"*** keyCeremony {a.nguardians} guardians quorum {a.quorum} {time.time() - t:.3f} s, proofs+backups valid = {kc_ok}")
    if not kc_ok:
        return 1
    key = ElectionKey(G, K)
    qbar = int.from_bytes(os.urandom(32), "big") % G.q
    man = Manifest(4, 5, 1)
    rng = np.random.default_rng()
    votes = random_votes(rng, man, a.nballots)
    t = time.time()
    eb = batch_encryption(G, key, qbar, man, votes, random_scalars(rng, (a.nballots, man.nsel, 4), G.q),
                          random_scalars(rng, (a.nballots, man.n_contests), G.q))
    print(f"*** encryptBallots {a.nballots} ballots {time.time() - t:.3f} s")
    t = time.time()
    ok_s, ok_c, tally = Verifier(G, key, qbar, man).verify(eb)
    print(f"*** verify+accumTally {time.time() - t:.3f} s, all valid = {bool(ok_s.all() and ok_c.all())}")
    tmp = Path(tempfile.mkdtemp(prefix="eg_trustees_"))
    procs, proxies = [], []
    try:
        for k, g in enumerate(gk[:navail]):
            f = tmp / f"{g.gid}.json"
            write_trustee_file(f, g, comm)
            env = dict(os.environ, HIP_VISIBLE_DEVICES=str(k % a.ngpus), PYTHONPATH=str(ROOT / "electionguard-remote_amd"))
            p = subprocess.Popen([sys.executable, "-m", "electionguard.trustee_server", "--trusteeFile", str(f)],
                                 stdout=subprocess.PIPE, text=True, env=env)
            procs.append(p)
        for p, g in zip(procs, gk[:navail]):
            line = p.stdout.readline().strip()
            if not line.startswith("PORT "):
                raise RuntimeError(f"trustee {g.gid} failed to start: {line!r}")
            proxies.append(RemoteDecryptingTrusteeProxy(g.gid, f"127.0.0.1:{line.split()[1]}", g.x, g.public_key))
        t = time.time()
        dec = Decryption(G, qbar, proxies, [g.gid for g in gk[navail:]], {g.gid: g.public_key for g in gk})
        counts = dec.decrypt(tally, a.nballots)
        print(f"*** remote decryption ({navail} trustees, {a.nguardians - navail} missing) {time.time() - t:.3f} s")
        expected = votes.reshape(a.nballots, man.n_contests, man.spc)[:, :, : man.n_selections].sum(axis=0).reshape(-1)
        ok = counts == [int(x) for x in expected]
        print(json.dumps({"counts": counts, "expected": [int(x) for x in expected], "match": ok,
                          "all_took_s": round(time.time() - t_all, 3)}))
        for px in proxies:
            px.finish(ok)
        for p in procs:
            p.wait(timeout=60)
        return 0 if ok and ok_s.all() and ok_c.all() else 1
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


if __name__ == "__main__":
    sys.exit(main())
