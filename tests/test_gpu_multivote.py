"""GPU: contests with votesAllowed = 2 (two placeholder selections, selection limit L = 2 in the
constant proof b = K^v B^c g^(-L c)), with under-votes filled by placeholders as EG does, and
ragged batch sizes (1 and 7 ballots).  Oracle-made
ballots verify, the tally skips both placeholders, a changed limit or a flipped placeholder
vote is rejected, and the GPU encryptor reproduces the oracle's bytes."""
import random

import numpy as np
import pytest

import eg_oracle as O
from conftest import be2i
from test_gpu_ballots import _oracle_ballots

pytestmark = pytest.mark.gpu


def _votes(man_o, rng):
    """0, 1 or 2 real votes per contest; placeholders make the contest sum equal L = 2."""
    out = []
    for _ in range(man_o.n_contests):
        k = rng.randrange(0, man_o.votes_allowed + 1)
        real = [0] * man_o.n_selections
        for i in rng.sample(range(man_o.n_selections), k):
            real[i] = 1
        out += real + [1] * (man_o.votes_allowed - k) + [0] * k
    return out


@pytest.mark.parametrize("nb", [1, 7])
def test_two_placeholders_limit_two(group, nb, monkeypatch):
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier, batch_encryption
    og = O.production_group()
    rng = random.Random(100 + nb)
    gs, K = O.key_ceremony(og, 2, 2, rng)
    qbar = rng.randrange(og.q)
    man_o, man = O.Manifest(2, 3, 2), Manifest(2, 3, 2)
    monkeypatch.setattr(O, "ballot_plaintexts", _votes)
    state = rng.getstate()
    cts, rp, cp, obs = _oracle_ballots(og, K, qbar, man_o, nb, rng)
    if nb == 1:
        assert O.verify_ballot(og, K, qbar, man_o, obs[0][1])
    key = ElectionKey(group, K)
    V = Verifier(group, key, qbar, man)
    ok_s, ok_c, tally = V.verify(EncryptedBallots(cts, rp, cp))
    assert ok_s.all() and ok_c.all()
    want = O.accumulate_tally(og, man_o, [eb for _, eb in obs])
    assert tally.shape == (man.n_real, 2, 512)
    for s, ct in enumerate(want):
        assert be2i(tally[s, 0]) == ct.pad and be2i(tally[s, 1]) == ct.data
    # limit 1 instead of 2: every contest proof fails, selection proofs still pass
    from electionguard.core import native
    ok_s1 = np.zeros((nb, man.nsel), np.uint8)
    ok_c1 = np.zeros((nb, man.n_contests), np.uint8)
    native.check(group._lib, "eg_verify_ballots", group._lib.eg_verify_ballots(
        group.handle, native.buf(int(K).to_bytes(512, "big")), native.buf(int(qbar).to_bytes(32, "big")), nb,
        man.n_contests, man.spc, 2, 1, cts.ctypes.data_as(native.c_vp), rp.ctypes.data_as(native.c_vp),
        cp.ctypes.data_as(native.c_vp), None, ok_s1.ctypes.data_as(native.c_vp), ok_c1.ctypes.data_as(native.c_vp),
        None))
    assert ok_s1.all() and not ok_c1.any()
    # the GPU encryptor with the oracle's injected nonces reproduces every byte
    r2 = random.Random()
    r2.setstate(state)
    votes, sn, cn = [], [], []
    for b in range(nb):
        v = _votes(man_o, r2)
        votes.append(v)
        s4, c1 = [], []
        for c in range(man_o.n_contests):
            for s in range(man_o.sel_per_contest):
                s4.append([r2.randrange(1, og.q), r2.randrange(1, og.q), r2.randrange(og.q), r2.randrange(og.q)])
            c1.append(r2.randrange(1, og.q))
        sn.append(s4)
        cn.append(c1)
    to = lambda xs: np.frombuffer(b"".join(int(x).to_bytes(32, "big") for x in xs), np.uint8)
    SN = np.stack([to([x for s4 in b for x in s4]).reshape(-1, 4, 32) for b in sn])
    CN = np.stack([to(b).reshape(-1, 32) for b in cn])
    eb = batch_encryption(group, key, qbar, man, np.array(votes, np.uint8), SN, CN)
    assert np.array_equal(eb.cts, cts) and np.array_equal(eb.rproof, rp) and np.array_equal(eb.cproof, cp)
