"""GPU: the 1M-ballot BASELINE configurations at full size on ONE MI355X, end to end.

* configs[4] -- "Large manifest 100 selections/ballot x 1M ballots: full-pipeline
  encrypt/verify/tally/decrypt" -- its N = 1 point: 1,000,000 ballots of 20 contests x (5+1)
  selections.
* configs[2] -- "verify + homomorphic tally 1M ballots sharded by ballot, RCCL all-gather of
  partial products" -- the same 1M ballots of 4 x (5+1), as its 8 ranks would shard them.

Both follow RunRemoteWorkflowTest.main (RunRemoteWorkflowTest.java:140-182): device encryption
(batchEncryption, :140-141), verify + tally (Verifier / runAccumulateBallots, :151, :179-182), then
threshold decryption through 5 DecryptingTrustees with 2 missing (direct + compensated shares with
proofs, RunRemoteDecryptingTrustee.java:189-193, :227-232; Decryption.decrypt,
RunRemoteDecryptor.java:261-262) and decryptBallot of spoiled ballots (:264-269).

The 1M ballots are processed as 8 shards of 125,000 -- configs[2]/[4]'s per-GPU share on 8 GPUs
-- and the 8 partial tallies are folded by ``eg_tally_allgather_fold`` over the 8 parts, the fold
rank 0 runs after the RCCL all-gather (here without a communicator: the all-gather's output is
laid out by hand).  The CPU oracle cannot redo 1M ballots in a test's time, so parity is through
size-independent properties: every verdict valid, the fold equal to the sequential product of the
shard tallies, the decrypted counts EXACTLY the plaintext vote sums over the cast ballots, every
decryption-record check (share proofs, recovery keys, quorum, B = M g^t), and every spoiled
ballot decrypting to its own votes; in the 4 x (5+1) run, three records of the last shard tampered
(a range-proof response, a contest challenge, a non-residue pad) flip exactly their verdicts on
a re-verify of all 125,000 ballots.  (The oracle pins the same kernels at small sizes:
test_gpu_golden.py, test_gpu_benchconfig.py, test_gpu_fullsize.py.)

Host nonce generation for shard k+1 overlaps the GPU's work on shard k (ctypes releases the GIL).
"""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHARDS = 8
SHARD = 125_000


def _shard_inputs(seed, k, man, q):
    from electionguard.ballot import random_scalars, random_votes
    rng = np.random.default_rng([seed, k])
    votes = random_votes(rng, man, SHARD)
    return votes, random_scalars(rng, (SHARD, man.nsel, 4), q), random_scalars(rng, (SHARD, man.n_contests), q)


def _tamper_last_shard(group, man, ver, cts, rp, cp, oks, okc, tal):
    """Full-size tamper detection on the last shard (125,000 ballots, re-verified on the device):
    one selection's range-proof response, one contest proof's challenge, and one ciphertext's pad
    multiplied by p - 1 (an element with an order-2 component: not a residue, so its range proof, its
    residue test and its contest's aggregate all fail).  Exactly these verdicts flip; every other of
    the shard's flags stays valid."""
    b1, s1 = 12_345, 3
    b2, c2 = 54_321, man.n_contests - 1
    b3, s3 = 99_999, man.spc + 1  # a selection of contest 1
    r = rp[b1:b1 + 1].download()
    r[0, s1, 1, 31] ^= 1
    rp[b1:b1 + 1].upload(r)
    c = cp[b2:b2 + 1].download()
    c[0, c2, 0, 5] ^= 0x40
    cp[b2:b2 + 1].upload(c)
    e = cts[b3:b3 + 1].download()
    alpha = int.from_bytes(e[0, s3, 0].tobytes(), "big")
    e[0, s3, 0] = np.frombuffer((alpha * (group.p - 1) % group.p).to_bytes(512, "big"), np.uint8)
    cts[b3:b3 + 1].upload(e)
    oks.zero()
    okc.zero()
    ver.verify_device(cts.ptr, rp.ptr, cp.ptr, SHARD, oks.ptr, okc.ptr, tal.ptr)
    group.sync()
    fs, fc = oks.download().reshape(SHARD, man.nsel), okc.download().reshape(SHARD, man.n_contests)
    bad_s = {tuple(x) for x in np.argwhere(fs == 0)}
    bad_c = {tuple(x) for x in np.argwhere(fc == 0)}
    assert bad_s == {(b1, s1), (b3, s3)}, bad_s
    assert bad_c == {(b2, c2), (b3, s3 // man.spc)}, bad_c


def _full_pipeline_1M(group, contests, seed, nspoiled, say=print, tamper=False):
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption_device
    from electionguard.decrypt import Decryption, DecryptingTrustee, verify_decryption_record
    from electionguard.keyceremony import key_ceremony, verify_backups, verify_commitment_proofs
    t_all = time.time()
    man = Manifest(contests, 5, 1)
    gk, K = key_ceremony(group, 5, 3, seed=seed)
    comm = {g.gid: g.commitments for g in gk}
    assert all(verify_commitment_proofs(group, [k for g in gk for k in g.commitments],
                                        [pr for g in gk for pr in g.proofs]))
    assert all(all(verify_backups(group, g, comm).values()) for g in gk)
    key = ElectionKey(group, K, window_bits=16)
    qbar = (0x1_000_000 + seed) % group.q
    ver = Verifier(group, key, qbar, man)
    # device buffers for one shard, reused by all 8
    dv = group.device_empty((SHARD, man.nsel))
    dsn = group.device_empty((SHARD, man.nsel, 4, 32))
    dcn = group.device_empty((SHARD, man.n_contests, 32))
    cts = group.device_empty((SHARD, man.nsel, 2, 512))
    rp = group.device_empty((SHARD, man.nsel, 4, 32))
    cp = group.device_empty((SHARD, man.n_contests, 2, 32))
    oks = group.device_empty((SHARD, man.nsel))
    okc = group.device_empty((SHARD, man.n_contests))
    tal = group.device_empty((man.n_real, 2, 512))
    cast = np.ones(SHARD, np.uint8)
    cast[:nspoiled] = 0
    dcast = group.to_device(cast)
    expected = np.zeros(man.n_real, np.int64)
    parts, spoiled_cts, spoiled_votes = [], None, None
    t_enc = t_ver = 0.0
    with ThreadPoolExecutor(1) as ex:
        nxt = ex.submit(_shard_inputs, seed, 0, man, group.q)
        for k in range(SHARDS):
            votes, sn, cn = nxt.result()
            if k + 1 < SHARDS:
                nxt = ex.submit(_shard_inputs, seed, k + 1, man, group.q)
            real = votes.reshape(SHARD, man.n_contests, man.spc)[:, :, :man.n_selections].reshape(SHARD, man.n_real)
            m = cast.astype(bool) if k == 0 else slice(None)
            expected += real[m].sum(axis=0, dtype=np.int64)
            dv.upload(votes)
            dsn.upload(sn)
            dcn.upload(cn)
            del sn, cn
            t = time.time()
            batch_encryption_device(group, key, qbar, man, SHARD, dv.ptr, dsn.ptr, dcn.ptr, cts.ptr, rp.ptr, cp.ptr)
            group.sync()
            t_enc += time.time() - t
            t = time.time()
            oks.zero()
            okc.zero()
            ver.verify_device(cts.ptr, rp.ptr, cp.ptr, SHARD, oks.ptr, okc.ptr, tal.ptr,
                              dcast.ptr if k == 0 else None)
            group.sync()
            ok = group.all_nonzero(oks) and group.all_nonzero(okc)
            t_ver += time.time() - t
            assert ok, f"honest ballots rejected in shard {k}"
            parts.append(tal.download())
            if k == 0 and nspoiled:
                spoiled_cts = cts[0:nspoiled].download()
                spoiled_votes = real[:nspoiled]
            say(f"  shard {k + 1}/{SHARDS}: {(k + 1) * SHARD} ballots, encrypt {t_enc:.1f} s, verify+tally {t_ver:.1f} s")
    if tamper:  # (the last shard's tally is already in parts)
        _tamper_last_shard(group, man, ver, cts, rp, cp, oks, okc, tal)
        say("  tampered last shard: exactly the 4 expected verdicts flipped")
    del cts, rp, cp, dsn, dcn, dv, oks, okc
    # rank 0's fold after the all-gather: parts laid out (world, n_real * 2, 512) as ncclAllGather leaves them
    gathered = np.ascontiguousarray(np.stack(parts)).reshape(SHARDS, man.n_real * 2, 512)
    tally = group.tally_allgather_fold(group.to_device(gathered), SHARDS, man.n_real * 2).reshape(man.n_real, 2, 512)
    seq = parts[0].reshape(-1, 512)
    for p in parts[1:]:
        seq = group.multP_batch(seq, p.reshape(-1, 512))
    assert np.array_equal(tally.reshape(-1, 512), seq), "all-gather fold != sequential product of the shard tallies"
    # threshold decryption: 3 of 5 guardians available, 2 compensated
    pub = {g.gid: g.public_key for g in gk}
    xs = {g.gid: g.x for g in gk}
    t = time.time()
    dec = Decryption(group, qbar, [DecryptingTrustee(group, g, comm) for g in gk[:3]], [g.gid for g in gk[3:]], pub)
    rec = dec.decrypt_record(tally, SHARDS * SHARD)
    t_dec = time.time() - t
    assert rec.counts == [int(x) for x in expected], "decrypted tally != plaintext vote sums"
    rv = verify_decryption_record(group, qbar, rec, pub, comm, guardian_xs=xs, quorum=3)
    assert all(rv.values()), rv
    if nspoiled:
        srec = dec.decrypt_ballots_record(spoiled_cts, man)
        plain = np.array([-1 if c is None else c for c in srec.counts]).reshape(nspoiled, man.n_real)
        assert np.array_equal(plain, spoiled_votes), "a spoiled ballot did not decrypt to its votes"
        rvs = verify_decryption_record(group, qbar, srec, pub, comm, guardian_xs=xs, quorum=3,
                                       max_count=man.votes_allowed)
        assert all(rvs.values()), rvs
    n = SHARDS * SHARD
    say(f"{contests}x(5+1), {n} ballots ({nspoiled} spoiled) on one GPU: encrypt {t_enc:.1f} s "
          f"({n / t_enc:.0f}/s), verify+tally {t_ver:.1f} s ({n / t_ver:.0f}/s), threshold decryption "
          f"{t_dec:.2f} s, all {time.time() - t_all:.1f} s; counts exact, record checks {rv}")


def _say(capsys):
    """Progress straight to the terminal, past pytest's capture: a 3-minute test must not look hung
    to a runner that watches the output."""
    def say(msg):
        with capsys.disabled():
            print(msg, flush=True)
    return say


@pytest.mark.timeout(420)
def test_config4_1M_ballots_100_selections_full_pipeline(group, capsys):
    """configs[4] at N = 1: 1M ballots x 20 x (5+1), encrypt -> verify + tally -> fold ->
    5 trustees (quorum 3, 2 missing) -> exact counts; 200 spoiled ballots decrypted one by one."""
    _full_pipeline_1M(group, 20, 4, nspoiled=200, say=_say(capsys))


@pytest.mark.timeout(180)
def test_config2_1M_ballots_4x5_full_pipeline(group, capsys):
    """configs[2]'s 1M ballots of 4 x (5+1) on one GPU as its 8 ranks shard them; 1,000 spoiled; and
    three tampered records in the last 125,000-ballot shard flip exactly their verdicts."""
    _full_pipeline_1M(group, 4, 2, nspoiled=1000, say=_say(capsys), tamper=True)
