"""GPU: the Montgomery-multiply counts of the op programs k_pow runs, pinned per unit of
work (eg_ctx_profile_end counts them from the programs of the timed launches):

* verifier, 4 x (5+1) manifest: per selection the alpha job's 462 + 2 W and the beta job's
  462 + 3 W (256-step squaring chain, 5 for w = B^189, 3 x 11 subset products of the 4-row,
  3-block comb, 2 x (21 + 63) comb evaluation, then 2 or 3 fixed-base terms of
  W = ceil(256 / window bits) table windows each), per contest 148 + W (A) and 148 + 2 W (B)
  gathered combs: 24,944 MM per ballot at the bench's 22-bit tables (W = 12), 27,584 at the
  default 8-bit ones (W = 32) (round 2's 5-row, 2-block comb, EG_SEL_COMB=52: 465 + ... and
  25,088);
* trustee share: 434 MM for the constant-time 4-row comb pair (A^s, A^u) + 102 for g^u
  from g's shared comb table.
The verdicts of the profiled batches are checked too (the counts are of real work)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu



def verify_mm_per_ballot(window_bits: int) -> int:
    W = -(-256 // window_bits)
    return 24 * ((462 + 2 * W) + (462 + 3 * W)) + 4 * ((148 + W) + (148 + 2 * W))


TRUSTEE_MM_PER_TEXT = (224 + 2 * 11 + 2 * (31 + 63)) + (1 + 51 * 2 - 1)


def test_verifier_mm_per_ballot(group):
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.keyceremony import key_ceremony
    assert verify_mm_per_ballot(22) == 24944 and verify_mm_per_ballot(8) == 27584
    man = Manifest(4, 5, 1)
    _, K = key_ceremony(group, 3, 3, seed=5)
    key = ElectionKey(group, K)
    rng = np.random.default_rng(9)
    nb = 300
    eb = batch_encryption(group, key, 77, man, random_votes(rng, man, nb),
                          random_scalars(rng, (nb, man.nsel, 4), group.q), random_scalars(rng, (nb, man.n_contests), group.q))
    V = Verifier(group, key, 77, man)
    V.verify(eb.slice(0, 1))  # warm-up: key registration and job tables outside the window
    group.profile_begin()
    ok_s, ok_c, _ = V.verify(eb)
    kp = group.profile_end()
    assert ok_s.all() and ok_c.all()
    assert kp.mont_ops == nb * verify_mm_per_ballot(key.window_bits), kp


def test_verifier_comb52_same_verdicts_and_tally(group, monkeypatch):
    """EG_SEL_COMB=52 (read at context creation) puts the selection jobs back on round 2's
    5-row, 2-block comb: its op programs cost 465 + 2 W / 465 + 3 W per alpha / beta job (25,088
    MM per ballot at W = 12), and its verdicts and tally equal the default 4 x 3 comb's, on
    honest ballots and with one tampered proof."""
    from electionguard.ballot import (ElectionKey, EncryptedBallots, Manifest, Verifier, batch_encryption,
                                      random_scalars, random_votes)
    from electionguard.core import GroupContext
    from electionguard.keyceremony import key_ceremony
    monkeypatch.setenv("EG_SEL_COMB", "52")
    g52 = GroupContext(group.p, group.q, group.g, device=group.device)
    man = Manifest(4, 5, 1)
    _, K = key_ceremony(group, 3, 3, seed=6)
    rng = np.random.default_rng(10)
    nb = 200
    eb = batch_encryption(group, ElectionKey(group, K), 77, man, random_votes(rng, man, nb),
                          random_scalars(rng, (nb, man.nsel, 4), group.q), random_scalars(rng, (nb, man.n_contests), group.q))
    rp = eb.rproof.copy()
    rp[17, 5, 1, 3] ^= 0x40
    bad = EncryptedBallots(eb.cts, rp, eb.cproof)
    W = -(-256 // 8)
    for G in (group, g52):
        V = Verifier(G, ElectionKey(G, K), 77, man)
        V.verify(eb.slice(0, 1))  # warm-up outside the profile window
        G.profile_begin()
        ok_s, ok_c, tally = V.verify(eb)
        kp = G.profile_end()
        assert ok_s.all() and ok_c.all()
        per_job = (465, 465) if G is g52 else (462, 462)
        assert kp.mont_ops == nb * (24 * ((per_job[0] + 2 * W) + (per_job[1] + 3 * W)) + 4 * ((148 + W) + (148 + 2 * W))), kp
        ok_s2, ok_c2, _ = V.verify(bad, with_tally=False)
        assert np.argwhere(~ok_s2).tolist() == [[17, 5]] and ok_c2.all()
        if G is group:
            ref_tally = tally
        else:
            assert np.array_equal(tally, ref_tally)


def test_trustee_mm_per_text(group):
    from electionguard.ballot import random_scalars
    from electionguard.decrypt import partial_decrypt_batch
    assert TRUSTEE_MM_PER_TEXT == 536
    rng = np.random.default_rng(4)
    n = 700
    R = random_scalars(rng, (n,), group.q)
    pads = group.gPowP_batch(R)
    texts = np.ascontiguousarray(np.stack([pads, pads], axis=1))
    nonces = random_scalars(rng, (n,), group.q)
    s = 0x1234567890ABCDEF
    partial_decrypt_batch(group, s, 99, texts[:2], nonces[:2])  # warm-up: g's shared comb table
    group.profile_begin()
    M, _ = partial_decrypt_batch(group, s, 99, texts, nonces)
    kp = group.profile_end()
    assert kp.mont_ops == n * TRUSTEE_MM_PER_TEXT, kp
    for i in (0, n // 2, n - 1):
        P = int.from_bytes(pads[i].tobytes(), "big")
        assert int.from_bytes(M[i].tobytes(), "big") == pow(P, s, group.p), i
