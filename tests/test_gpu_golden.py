"""GPU path (through the C ABI) against the committed golden fixtures of BOTH production
groups (Mode4096 = EG 1.0, the reference's group; Mode4096_V2 = EG 2.0), and the
residue-validation forgery (alpha * (p-1) with matching proofs) rejected on the GPU."""
import numpy as np
import pytest

import eg_oracle as O
from test_oracle_golden import (MODES, _arr, ballot_wire_arrays, golden_ballot_arrays, h, load,
                                residue_forgery_case, twisted_pair_case)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=MODES)
def mode_group(request, group):
    from electionguard.core import productionGroup
    return request.param, productionGroup(0, request.param)


def test_group_golden(mode_group):
    mode, group = mode_group
    d = load("group_ops.json", mode)
    out = group.powP_batch(_arr([v["b"] for v in d["powP"]], 512), _arr([v["e"] for v in d["powP"]], 32))
    assert [x.tobytes().hex() for x in out] == [v["r"] for v in d["powP"]]
    out = group.gPowP_batch(_arr([v["e"] for v in d["gPowP"]], 32))
    assert [x.tobytes().hex() for x in out] == [v["r"] for v in d["gPowP"]]
    out = group.multP_batch(_arr([v["a"] for v in d["multP"]], 512), _arr([v["b"] for v in d["multP"]], 512))
    assert [x.tobytes().hex() for x in out] == [v["r"] for v in d["multP"]]
    out = group.multInv_batch(_arr([v["a"] for v in d["multInv"]], 512))
    assert [x.tobytes().hex() for x in out] == [v["r"] for v in d["multInv"]]
    for v in d["prodP"]:
        out = group.prodP_groups(_arr(v["xs"], 512), 1, len(v["xs"]))
        assert out[0].tobytes().hex() == v["r"]


def test_ballots_golden_verify_tally_and_reencrypt(mode_group):
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier, batch_encryption
    mode, group = mode_group
    d, (nc, ns, va, spc), cts, rp, cp = golden_ballot_arrays(mode)
    man = Manifest(nc, ns, va)
    key = ElectionKey(group, h(d["K"]))
    ok_s, ok_c, tally = Verifier(group, key, h(d["qbar"]), man).verify(EncryptedBallots(cts, rp, cp))
    assert ok_s.all() and ok_c.all()
    assert [[t[0].tobytes().hex(), t[1].tobytes().hex()] for t in tally] == d["tally"]
    nb = len(d["ballots"])
    votes = np.array([b["votes"] for b in d["ballots"]], np.uint8)
    sn = np.stack([_arr([x for n4 in b["nonces"] for x in n4], 32).reshape(-1, 4, 32) for b in d["ballots"]])
    cn = np.stack([_arr(b["contest_nonces"], 32) for b in d["ballots"]])
    eb = batch_encryption(group, key, h(d["qbar"]), man, votes, sn, cn)
    assert np.array_equal(eb.cts, cts) and np.array_equal(eb.rproof, rp) and np.array_equal(eb.cproof, cp)
    assert nb == eb.n


def test_trustee_golden(mode_group):
    from electionguard.decrypt import partial_decrypt_batch
    mode, group = mode_group
    d = load("trustee.json", mode)
    T = np.stack([_arr(t, 512) for t in d["texts"]])
    N = _arr(d["nonces"], 32)
    M, pr = partial_decrypt_batch(group, h(d["guardians"][0]["coeffs"][0]), h(d["qbar"]), T, N)
    for i, w in enumerate(d["direct"]):
        assert (M[i].tobytes().hex(), pr[i, 0].tobytes().hex(), pr[i, 1].tobytes().hex()) == (w["M"], w["c"], w["v"])
    share = O.poly_eval([h(a) for a in d["guardians"][2]["coeffs"]], 2, O.Q)
    M, pr = partial_decrypt_batch(group, share, h(d["qbar"]), T, N)
    for i, w in enumerate(d["compensated_by_x2_for_x3"]):
        assert (M[i].tobytes().hex(), pr[i, 0].tobytes().hex(), pr[i, 1].tobytes().hex()) == (w["M"], w["c"], w["v"])


def _ballot_arrays(eb):
    b = lambda x, n: np.frombuffer(int(x).to_bytes(n, "big"), np.uint8)
    cts = np.stack([np.stack([b(ct.pad, 512), b(ct.data, 512)]) for ct in eb.cts])[None]
    rp = np.stack([np.stack([b(v, 32) for v in (pr.c0, pr.v0, pr.c1, pr.v1)]) for pr in eb.proofs])[None]
    cp = np.stack([np.stack([b(pr.c, 32), b(pr.v, 32)]) for pr in eb.contest_proofs])[None]
    return cts, rp, cp


def test_gpu_rejects_non_residue_alpha_with_matching_proofs(group):
    """alpha * (p-1) with every Fiat-Shamir equation re-made to hold (c even): only the
    x^q == 1 tests catch it, for the selection (alpha) and for its contest (A = prod alpha, valid
    only when every alpha is).
    The same ciphertexts with beta negated instead, and an honest ballot alongside, too."""
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
    G, K, qbar, man_o, eb, sel = residue_forgery_case()
    cts, rp, cp = _ballot_arrays(eb)
    # second ballot: the honest re-encryption of a fresh ballot, third: beta negated in selection 4
    import random
    rng = random.Random(5)
    honest = O.encrypt_ballot(G, K, qbar, man_o, O.ballot_plaintexts(man_o, rng), rng)
    c2, r2, p2 = _ballot_arrays(honest)
    c3 = c2.copy()
    c3[0, 4, 1] = np.frombuffer(((G.p - 1) * honest.cts[4].data % G.p).to_bytes(512, "big"), np.uint8)
    man = Manifest(man_o.n_contests, man_o.n_selections, man_o.votes_allowed)
    ok_s, ok_c, _ = Verifier(group, ElectionKey(group, K), qbar, man).verify(
        EncryptedBallots(np.concatenate([cts, c2, c3]), np.concatenate([rp, r2, r2]), np.concatenate([cp, p2, p2])))
    assert ok_s[0].tolist() == [i != sel for i in range(man.nsel)]
    assert ok_c[0].tolist() == [False, True]
    assert ok_s[1].all() and ok_c[1].all()
    assert not ok_s[2, 4] and ok_s[2].sum() == man.nsel - 1          # beta residue (the hash fails too)
    assert ok_c[2].tolist() == [True, False]                          # B = prod beta is not a residue


def test_gpu_rejects_contest_whose_selections_are_invalid(group):
    """Contest 0 holds two alphas times p - 1: A = prod alpha is a valid residue and the contest
    proof verifies, but its selections are invalid, so the contest is rejected (the round-3
    contest rule, k_contest_flags), as both oracles do."""
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
    G, K, qbar, man_o, eb = twisted_pair_case()
    man = Manifest(man_o.n_contests, man_o.n_selections, man_o.votes_allowed)
    ok_s, ok_c, _ = Verifier(group, ElectionKey(group, K), qbar, man).verify(
        EncryptedBallots(*ballot_wire_arrays(eb)), with_tally=False)
    assert ok_s[0].tolist() == [i > 1 for i in range(man.nsel)]
    assert ok_c[0].tolist() == [False, True]
