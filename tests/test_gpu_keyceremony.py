"""Key-ceremony arithmetic on the GPU (RunRemoteKeyCeremony.java:200-233):
Schnorr proofs of the coefficient commitments and the recipients' backup checks, against
the oracle restatement (oracle/eg_oracle.py: schnorr_prove / schnorr_verify /
verify_backup_share).  Proof bytes use random nonces, so they are pinned by verification
(the upstream pre-image is unpinned)."""
import random

import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


def test_schnorr_proofs_gpu_vs_oracle(group):
    from electionguard.keyceremony import key_ceremony, verify_commitment_proofs
    og = O.production_group()
    gk, _ = key_ceremony(group, 5, 3, seed=404)
    Ks = [K for g in gk for K in g.commitments]
    prs = [pr for g in gk for pr in g.proofs]
    # GPU-made proofs verify under the CPython oracle
    for K, (c, v) in zip(Ks, prs):
        assert O.schnorr_verify(og, K, O.GenericProof(c, v))
    assert verify_commitment_proofs(group, Ks, prs) == [True] * len(Ks)
    # oracle-made proofs verify on the GPU; tampering is rejected exactly where the oracle rejects
    rng = random.Random(5)
    a = rng.randrange(1, og.q)
    K = og.gPowP(a)
    good = O.schnorr_prove(og, a, K, rng.randrange(1, og.q))
    cases = [(K, (good.c, good.v)),
             (K, (good.c, (good.v + 1) % og.q)),
             (K, ((good.c + 1) % og.q, good.v)),
             (og.multP(K, og.g), (good.c, good.v)),
             (og.p - 1, (good.c, good.v)),            # not in the order-q subgroup
             (K, (good.c, og.q)),                      # response out of range
             (Ks[3], prs[4])]                          # another commitment's proof
    want = [O.schnorr_verify(og, k, O.GenericProof(c, v)) for k, (c, v) in cases]
    assert want == [True, False, False, False, False, False, False]
    assert verify_commitment_proofs(group, [k for k, _ in cases], [pr for _, pr in cases]) == want


def test_backup_verification_gpu_vs_oracle(group):
    from electionguard.keyceremony import backup_label, key_ceremony, verify_backups
    og = O.production_group()
    gk, _ = key_ceremony(group, 4, 3, seed=77)
    comm = {g.gid: g.commitments for g in gk}
    for g in gk:
        assert verify_backups(group, g, comm) == {l: True for l in comm if l != g.gid}
    # a well-formed backup (valid MAC) of a WRONG share fails only the commitment check
    ora = {g.gid: O.Guardian(g.gid, g.x, g.coeffs, g.commitments) for g in gk}
    tgt, src = gk[2], gk[0]
    wrong = (O.poly_eval(src.coeffs, tgt.x, og.q) + 1) % og.q
    tgt.backups_from[src.gid] = O.backup_encrypt(og, tgt.public_key, wrong, 12345,
                                                 backup_label(src.gid, tgt.gid))
    assert not O.verify_backup_share(og, wrong, ora[src.gid], tgt.x)
    assert O.verify_backup_share(og, O.poly_eval(gk[1].coeffs, tgt.x, og.q), ora[gk[1].gid], tgt.x)
    # a corrupted MAC fails to open
    c0, c1, c2 = tgt.backups_from[gk[3].gid]
    tgt.backups_from[gk[3].gid] = (c0, bytes([c1[0] ^ 4]) + c1[1:], c2)
    assert verify_backups(group, tgt, comm) == {src.gid: False, gk[1].gid: True, gk[3].gid: False}
