"""GPU path (through the C ABI) against the committed golden fixtures."""
import json
from pathlib import Path

import numpy as np
import pytest

from test_oracle_golden import _arr, golden_ballot_arrays, h, load

pytestmark = pytest.mark.gpu


def test_group_golden(group):
    d = load("group_ops.json")
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


def test_ballots_golden_verify_tally_and_reencrypt(group):
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier, batch_encryption
    d, (nc, ns, va, spc), cts, rp, cp = golden_ballot_arrays()
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


def test_trustee_golden(group):
    from electionguard.decrypt import partial_decrypt_batch
    d = load("trustee.json")
    T = np.stack([_arr(t, 512) for t in d["texts"]])
    N = _arr(d["nonces"], 32)
    M, pr = partial_decrypt_batch(group, h(d["guardians"][0]["coeffs"][0]), h(d["qbar"]), T, N)
    for i, w in enumerate(d["direct"]):
        assert (M[i].tobytes().hex(), pr[i, 0].tobytes().hex(), pr[i, 1].tobytes().hex()) == (w["M"], w["c"], w["v"])
    import eg_oracle as O
    share = O.poly_eval([h(a) for a in d["guardians"][2]["coeffs"]], 2, O.Q)
    M, pr = partial_decrypt_batch(group, share, h(d["qbar"]), T, N)
    for i, w in enumerate(d["compensated_by_x2_for_x3"]):
        assert (M[i].tobytes().hex(), pr[i, 0].tobytes().hex(), pr[i, 1].tobytes().hex()) == (w["M"], w["c"], w["v"])
