"""GPU: the BASELINE.json configurations at one GPU's full share, checked through
size-independent properties (the CPU oracle cannot redo them in a test's time):

* configs[4]'s manifest (20 x 5): 10,000 ballots, device-resident as bench.py runs them.  Every
  verdict is valid; the tally decrypts (joint secret, BSGS dLog) to exactly the per-selection
  vote sums; and the two-rank fold (each half verified alone, partial tallies multiplied mod p as
  electionguard.distributed.gather_fold_tally does on rank 0) equals the single tally.

configs[2] and configs[4] at their full 1M ballots (8 shards of 125,000, the 8-part fold,
threshold decryption through DecryptingTrustees) are tests/test_gpu_config_1M.py; they subsume the
one-rank 125k-shard tests this file held until round 5.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(group, contests, selections, nb, seed, trustees=False):
    from electionguard.ballot import (ElectionKey, Manifest, Verifier, batch_encryption_device, random_scalars,
                                      random_votes)
    from electionguard.decrypt import dlog_g_batch
    from electionguard.distributed import gather_fold_tally
    from electionguard.keyceremony import key_ceremony
    man = Manifest(contests, selections, 1)
    gk, K = key_ceremony(group, 5 if trustees else 3, 3, seed=seed)
    key = ElectionKey(group, K, window_bits=16)
    rng = np.random.default_rng(seed)
    votes = random_votes(rng, man, nb)
    dv = group.to_device(votes)
    dsn = group.to_device(random_scalars(rng, (nb, man.nsel, 4), group.q))
    dcn = group.to_device(random_scalars(rng, (nb, man.n_contests), group.q))
    cts = group.device_empty((nb, man.nsel, 2, 512))
    rp = group.device_empty((nb, man.nsel, 4, 32))
    cp = group.device_empty((nb, man.n_contests, 2, 32))
    qbar = 0xC0FFEE + seed
    batch_encryption_device(group, key, qbar, man, nb, dv.ptr, dsn.ptr, dcn.ptr,
                            cts.ptr, rp.ptr, cp.ptr)
    del dsn, dcn
    V = Verifier(group, key, qbar, man)

    def verify(a, b):
        oks = group.device_zeros((b - a, man.nsel))
        okc = group.device_zeros((b - a, man.n_contests))
        tal = group.device_zeros((man.n_real, 2, 512))
        V.verify_device(cts[a:b].ptr, rp[a:b].ptr, cp[a:b].ptr, b - a, oks.ptr,
                        okc.ptr, tal.ptr)
        group.sync()
        return group.all_nonzero(oks) and group.all_nonzero(okc), tal

    ok, tally = verify(0, nb)
    assert ok, "honest ballots rejected"
    T = tally.download()
    want = votes.reshape(nb, man.n_contests, man.spc)[:, :, :man.n_selections].sum(axis=0).reshape(-1)
    if trustees:  # the trustees' shares: 3 of 5 guardians available, 2 compensated
        from electionguard.decrypt import DecryptingTrustee, Decryption
        comm = {g.gid: g.commitments for g in gk}
        dec = Decryption(group, qbar, [DecryptingTrustee(group, g, comm) for g in gk[:3]],
                         [g.gid for g in gk[3:]], {g.gid: g.public_key for g in gk})
        counts = dec.decrypt(T, nb)
    else:  # the joint secret (quorum = all 3 guardians): t = dLog_g(beta / alpha^S)
        S = sum(int(g.secret) for g in gk) % group.q
        M = group.powP_batch(np.ascontiguousarray(T[:, 0]), [S] * man.n_real)
        gt = group.multP_batch(np.ascontiguousarray(T[:, 1]), group.multInv_batch(M))
        counts = dlog_g_batch(group, gt, nb)
    assert counts == [int(x) for x in want]
    # two-rank shard fold == the single tally
    h = nb // 2 + 17
    ok_a, t_a = verify(0, h)
    ok_b, t_b = verify(h, nb)
    assert ok_a and ok_b

    class TwoRanks:  # the gather's result for world = 2, as gather_fold_tally folds it on rank 0
        @staticmethod
        def is_initialized():
            return False

    parts = np.stack([t_a.download(), t_b.download()])          # (world, n_real, 2, 512)
    g = np.ascontiguousarray(np.transpose(parts, (1, 2, 0, 3))).reshape(-1, 512)
    folded = group.prodP_groups(g, man.n_real * 2, 2).reshape(man.n_real, 2, 512)
    assert np.array_equal(folded, T)
    assert gather_fold_tally(TwoRanks, T, group.prodP_groups).tobytes() == T.tobytes()  # world 1: identity
    # the same fold in libeg_hip (eg_tally_allgather_fold without a communicator: the local parts)
    d2 = group.to_device(parts)
    assert np.array_equal(group.tally_allgather_fold(d2, 2, man.n_real * 2).reshape(man.n_real, 2, 512), T)


def test_config4_shape_100_selections(group):
    _run(group, 20, 5, 10_000, 23)
