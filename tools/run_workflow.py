"""End-to-end remote workflow — ``RunRemoteWorkflowTest.main``
(src/test/java/electionguard/workflow/RunRemoteWorkflowTest.java:83-192) on the GPU path:

  1 key ceremony (in-process; commitments, Schnorr proofs and share backups made and
    checked on the GPU)                     2 encrypt ballots (GPU)
  3 accumulate tally + verify ballots (GPU)
  4 remote decryption: one trustee PROCESS per available guardian over gRPC on localhost,
    missing guardians compensated (RunRemoteDecryptionTest.java:63-136)
  5 check the decrypted counts against the plaintext votes (the reference only prints)
  6 with -nspoiled k: the first k ballots are spoiled -- verified but not tallied, then each is
    decrypted through the same remote trustees (RunRemoteDecryptor.java:264-269, -decryptSpoiled)
    and must decrypt to its own votes

    python tools/run_workflow.py -nguardians 3 -quorum 3 -nballots 25            # configs[0]
    python tools/run_workflow.py -nguardians 5 -quorum 3 -navailable 3 -nballots 100   # configs[3]
    python tools/run_workflow.py -nballots 1000000                                      # configs[2] tally size
    python tools/run_workflow.py -ncontests 20 -nballots 1000000                        # configs[4] manifest
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
    ap.add_argument("-ncontests", type=int, default=4)
    ap.add_argument("-nselections", type=int, default=5, help="real selections per contest (+1 placeholder)")
    ap.add_argument("-fbwindow", type=int, default=8, help="fixed-base radix window bits for K (8 = LOW_MEMORY_USE)")
    ap.add_argument("-chunk", type=int, default=65536,
                    help="ballots per encrypt+verify batch; batch tallies are multiplied (bounded memory)")
    ap.add_argument("-nspoiled", type=int, default=0, help="spoiled ballots (the first k; at most one chunk)")
    a = ap.parse_args()
    if a.nspoiled > min(a.chunk, a.nballots):
        ap.error("-nspoiled must fit in the first chunk")
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.core import productionGroup
    from electionguard.decrypt import Decryption, verify_decryption_record
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
    key = ElectionKey(G, K, window_bits=a.fbwindow)
    qbar = int.from_bytes(os.urandom(32), "big") % G.q
    man = Manifest(a.ncontests, a.nselections, 1)
    rng = np.random.default_rng()
    ver = Verifier(G, key, qbar, man)
    expected = np.zeros(man.n_real, dtype=np.int64)
    tally, t_enc, t_ver, t_gen, all_ok = None, 0.0, 0.0, 0.0, True
    spoiled, spoiled_votes = None, None
    for b0 in range(0, a.nballots, a.chunk):
        nb = min(a.chunk, a.nballots - b0)
        t = time.time()
        votes = random_votes(rng, man, nb)
        sn = random_scalars(rng, (nb, man.nsel, 4), G.q)
        cn = random_scalars(rng, (nb, man.n_contests), G.q)
        cast = np.ones(nb, bool)
        if b0 == 0:
            cast[: a.nspoiled] = False
        real = votes.reshape(nb, man.n_contests, man.spc)[:, :, : man.n_selections].reshape(nb, man.n_real)
        expected += real[cast].sum(axis=0, dtype=np.int64)
        if b0 == 0 and a.nspoiled:
            spoiled_votes = real[~cast]
        t_gen += time.time() - t
        t = time.time()
        eb = batch_encryption(G, key, qbar, man, votes, sn, cn)
        t_enc += time.time() - t
        if b0 == 0 and a.nspoiled:
            spoiled = eb.slice(0, a.nspoiled)
        t = time.time()
        ok_s, ok_c, part = ver.verify(eb, cast=None if cast.all() else cast)
        all_ok = all_ok and bool(ok_s.all() and ok_c.all())
        tally = part if tally is None else G.multP_batch(tally.reshape(-1, 512), part.reshape(-1, 512)).reshape(part.shape)
        t_ver += time.time() - t
        if a.nballots > a.chunk:
            print(f"    {b0 + nb}/{a.nballots} ballots: encrypt {t_enc:.1f} s, verify+tally {t_ver:.1f} s", flush=True)
    print(f"*** encryptBallots {a.nballots} ballots ({man.nsel} selections each) {t_enc:.3f} s "
          f"({a.nballots / max(t_enc, 1e-9):.0f} ballots/s; host nonce generation {t_gen:.1f} s untimed)")
    print(f"*** verify+accumTally {t_ver:.3f} s ({a.nballots / max(t_ver, 1e-9):.0f} ballots/s), all valid = {all_ok}",
          flush=True)
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
        rec = dec.decrypt_record(tally, a.nballots)
        counts = rec.counts
        print(f"*** remote decryption ({navail} trustees, {a.nguardians - navail} missing) {time.time() - t:.3f} s")
        t = time.time()
        rv = verify_decryption_record(G, qbar, rec, {g.gid: g.public_key for g in gk}, comm)
        print(f"*** verify decryption record {time.time() - t:.3f} s: {rv}")
        ok = counts == [int(x) for x in expected]
        spoiled_ok, rvs = True, {}
        if spoiled is not None:
            t = time.time()
            srec = dec.decrypt_ballots_record(spoiled, man)
            plain = np.array([-1 if c is None else c for c in srec.counts]).reshape(-1, man.n_real)
            spoiled_ok = bool(np.array_equal(plain, spoiled_votes))
            t_dec, t = time.time() - t, time.time()
            rvs = verify_decryption_record(G, qbar, srec, {g.gid: g.public_key for g in gk}, comm,
                                           max_count=man.votes_allowed)
            print(f"*** decryptBallot x {a.nspoiled} spoiled ({a.nspoiled * man.n_real} selections, one remote batch "
                  f"per trustee) {t_dec:.3f} s, its record verified in {time.time() - t:.3f} s: plaintexts match = "
                  f"{spoiled_ok}, record = {rvs}")
        print(json.dumps({"counts": counts, "expected": [int(x) for x in expected], "match": ok and spoiled_ok,
                          "record_checks": rv, "spoiled": a.nspoiled, "spoiled_match": spoiled_ok,
                          "spoiled_record_checks": rvs,
                          "all_took_s": round(time.time() - t_all, 3)}))
        ok = ok and spoiled_ok and all(rvs.values())
        for px in proxies:
            px.finish(ok)
        for p in procs:
            p.wait(timeout=60)
        return 0 if ok and all_ok and all(rv.values()) else 1
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


if __name__ == "__main__":
    sys.exit(main())
