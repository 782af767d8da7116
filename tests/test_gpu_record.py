"""GPU: election-record verification (record.verify_election_record, the reference's
``Verifier(record, 11).verify()`` step, RunRemoteWorkflowTest.java:179-182): an honest
5-guardian / quorum-3 record with 2 missing guardians passes every check, and each
tampering fails the check that covers it (and only the checks that depend on it)."""
import copy

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def election(group):
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.decrypt import DecryptingTrustee, Decryption
    from electionguard.keyceremony import key_ceremony
    from electionguard.record import ElectionRecord, GuardianRecord
    gk, K = key_ceremony(group, 5, 3, seed=77)
    man = Manifest(2, 3, 1)
    rng = np.random.default_rng(77)
    nb = 12
    votes = random_votes(rng, man, nb)
    qbar = 0xABCDEF
    key = ElectionKey(group, K)
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), group.q),
                          random_scalars(rng, (nb, man.n_contests), group.q))
    _, _, tally = Verifier(group, key, qbar, man).verify(eb)
    comm = {g.gid: g.commitments for g in gk}
    avail = [DecryptingTrustee(group, g, comm) for g in gk[:3]]
    drec = Decryption(group, qbar, avail, [g.gid for g in gk[3:]], {g.gid: g.public_key for g in gk}) \
        .decrypt_record(tally, nb)
    rec = ElectionRecord(man, qbar, K, [GuardianRecord(g.gid, g.x, list(g.commitments), list(g.proofs)) for g in gk],
                         eb, tally, drec)
    expected = votes.reshape(nb, man.n_contests, man.spc)[:, :, : man.n_selections].sum(axis=0).reshape(-1)
    return rec, [int(x) for x in expected]


def test_honest_record_passes(group, election):
    from electionguard.record import verify_election_record
    rec, expected = election
    assert rec.decryption.counts == expected
    res = verify_election_record(group, rec)
    assert all(res.values()), res


def _failed(res):
    return sorted(k for k, v in res.items() if not v)


def test_tampered_records_fail_their_check(group, election):
    from electionguard.ballot import EncryptedBallots
    from electionguard.record import verify_election_record
    rec, _ = election
    p = group.p

    bad = copy.copy(rec)
    g0 = copy.deepcopy(rec.guardians[0])
    c, v = g0.proofs[1]
    g0.proofs[1] = (c, (v + 1) % group.q)
    bad.guardians = [g0] + rec.guardians[1:]
    assert _failed(verify_election_record(group, bad)) == ["guardian_proofs"]

    bad = copy.copy(rec)
    bad.joint_key = rec.joint_key * group.g % p
    # the ballots were encrypted under the real K, so their proofs fail under the wrong one too
    assert _failed(verify_election_record(group, bad)) == ["ballots", "joint_key"]

    bad = copy.copy(rec)
    rp = rec.ballots.rproof.copy()
    rp[5, 2, 1, 7] ^= 0x10
    bad.ballots = EncryptedBallots(rec.ballots.cts, rp, rec.ballots.cproof)
    assert _failed(verify_election_record(group, bad)) == ["ballots"]

    bad = copy.copy(rec)
    et = rec.encrypted_tally.copy()
    et[[0, 1]] = et[[1, 0]]   # two selections' totals swapped
    bad.encrypted_tally = et
    assert _failed(verify_election_record(group, bad)) == ["decryption.texts", "tally"]

    bad = copy.copy(rec)
    bad.decryption = copy.deepcopy(rec.decryption)
    bad.decryption.counts[3] += 1
    assert _failed(verify_election_record(group, bad)) == ["decryption.tally"]


def test_structurally_bad_records_report_false_instead_of_raising(group, election):
    """empty commitment lists, out-of-range counts, x-coordinates that disagree
    with the key ceremony, too few available guardians."""
    from electionguard.record import verify_election_record
    rec, _ = election

    bad = copy.copy(rec)
    g0 = copy.deepcopy(rec.guardians[0])
    g0.commitments, g0.proofs = [], []
    bad.guardians = [g0] + rec.guardians[1:]
    res = verify_election_record(group, bad)
    assert not res["guardian_proofs"] and not res["joint_key"]

    for c in (-1, rec.ballots.n + 1, 2.5):
        bad = copy.copy(rec)
        bad.decryption = copy.deepcopy(rec.decryption)
        bad.decryption.counts[0] = c
        assert _failed(verify_election_record(group, bad)) == ["decryption.tally"]

    bad = copy.copy(rec)
    bad.guardians = [copy.deepcopy(g) for g in rec.guardians]
    bad.guardians[1].x = 9   # the ceremony's x for guardian 2 differs from the record's
    assert "decryption.quorum" in _failed(verify_election_record(group, bad))

    bad = copy.copy(rec)
    bad.decryption = copy.deepcopy(rec.decryption)
    gone = sorted(bad.decryption.direct)[0]
    del bad.decryption.direct[gone]   # 2 available < quorum 3, and gone is neither available nor missing
    assert "decryption.quorum" in _failed(verify_election_record(group, bad))


def test_record_with_spoiled_ballots(group):
    """A record with 3 spoiled ballots of 12 (RunRemoteDecryptor.java:264-269): the tally covers the
    9 cast ones, the spoiled ballots' decryption covers exactly their real selections and passes
    every share check with plaintexts <= votesAllowed; claiming a spoiled ballot as cast breaks
    the tally, and a tampered spoiled plaintext breaks only the spoiled record's B == M g^t."""
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.decrypt import DecryptingTrustee, Decryption
    from electionguard.keyceremony import key_ceremony
    from electionguard.record import ElectionRecord, GuardianRecord, verify_election_record
    gk, K = key_ceremony(group, 5, 3, seed=78)
    man = Manifest(2, 3, 1)
    rng = np.random.default_rng(78)
    nb = 12
    votes = random_votes(rng, man, nb)
    qbar = 0xABCDE0
    key = ElectionKey(group, K)
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), group.q),
                          random_scalars(rng, (nb, man.n_contests), group.q))
    cast = np.ones(nb, bool)
    cast[[1, 6, 11]] = False
    _, _, tally = Verifier(group, key, qbar, man).verify(eb, cast=cast)
    comm = {g.gid: g.commitments for g in gk}
    dec = Decryption(group, qbar, [DecryptingTrustee(group, g, comm) for g in gk[:3]], [g.gid for g in gk[3:]],
                     {g.gid: g.public_key for g in gk})
    drec = dec.decrypt_record(tally, int(cast.sum()))
    srec = dec.decrypt_ballots_record(eb.slice(0, nb).cts[~cast], man)
    real = votes.reshape(nb, man.n_contests, man.spc)[:, :, : man.n_selections].reshape(nb, man.n_real)
    assert drec.counts == [int(x) for x in real[cast].sum(axis=0)]
    assert np.array_equal(np.array(srec.counts).reshape(-1, man.n_real), real[~cast])
    rec = ElectionRecord(man, qbar, K, [GuardianRecord(g.gid, g.x, list(g.commitments), list(g.proofs)) for g in gk],
                         eb, tally, drec, cast=cast, spoiled_decryption=srec)
    res = verify_election_record(group, rec)
    assert all(res.values()) and "spoiled.tally" in res, res
    bad = copy.copy(rec)
    bad.cast = np.ones(nb, bool)  # the spoiled ballots claimed as cast
    assert "tally" in _failed(verify_election_record(group, bad))
    bad = copy.copy(rec)
    bad.spoiled_decryption = copy.deepcopy(srec)
    bad.spoiled_decryption.counts[4] = 1 - bad.spoiled_decryption.counts[4]
    assert _failed(verify_election_record(group, bad)) == ["spoiled.tally"]
    bad = copy.copy(rec)
    bad.spoiled_decryption = None
    assert _failed(verify_election_record(group, bad)) == ["spoiled.decryption", "spoiled.texts"]
