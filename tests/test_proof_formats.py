"""CPU: the switchable proof conventions in the oracle (eg_oracle.proof_format: the response sign
and the challenge pre-image order; unpinned upstream).  The committed fixture
tests/golden/Mode4096/proof_formats.json holds the same ballots, nonces and trustee texts under
each of the 6 variants; the oracle reproduces every variant's bytes from the injected nonces, and a
variant's proofs fail under every other variant."""
import json
import random

import pytest

import eg_oracle as O
from test_oracle_golden import GOLD, h

FX = json.loads((GOLD / O.MODE4096 / "proof_formats.json").read_text())
VARIANTS = [(v["response"], v["preimage"]) for v in FX["variants"]]


def _variant(resp, pre):
    return next(v for v in FX["variants"] if (v["response"], v["preimage"]) == (resp, pre))


def _ballot(G, b):
    cts = [O.Ciphertext(h(a), h(d)) for a, d in b["cts"]]
    prs = [O.RangeProof(*[h(x) for x in p]) for p in b["rproofs"]]
    cps = [O.GenericProof(h(c), h(v)) for c, v in b["cproofs"]]
    return O.EncryptedBallot(cts, prs, cps)


def test_fixture_covers_every_variant():
    assert sorted(VARIANTS) == sorted((r, p) for r in O.RESPONSES for p in O.PREIMAGES)
    assert _variant("minus", "message_first")["ballots"][0]["cts"] == _variant("plus", "with_key")["ballots"][0]["cts"]
    assert _variant("minus", "message_first")["ballots"][0]["rproofs"] != _variant("plus", "message_first")["ballots"][0]["rproofs"]


@pytest.mark.parametrize("resp,pre", VARIANTS)
def test_oracle_reproduces_each_variant(resp, pre):
    G = O.production_group()
    K, qbar = h(FX["K"]), h(FX["qbar"])
    nc, ns, va = FX["manifest"]
    man = O.Manifest(nc, ns, va)
    v = _variant(resp, pre)
    gs = [O.Guardian(f"guardian{g['x']}", g["x"], [h(a) for a in g["coeffs"]], [h(k) for k in g["commitments"]])
          for g in FX["guardians"]]
    texts = [O.Ciphertext(h(a), h(b)) for a, b in FX["texts"]]
    nonces = [h(u) for u in FX["nonces"]]
    with O.proof_format(resp, pre):
        b = v["ballots"][0]
        # re-make the first contest's proofs from the injected nonces
        for s in range(man.sel_per_contest):
            R, u, cf, vf = (h(x) for x in b["nonces"][s])
            ct = O.encrypt(G, K, b["votes"][s], R)
            pr = O.make_range_proof(G, K, qbar, ct, b["votes"][s], R, u, cf, vf)
            assert [pr.c0, pr.v0, pr.c1, pr.v1] == [h(x) for x in b["rproofs"][s]]
        eb = _ballot(G, b)
        assert O.verify_ballot(G, K, qbar, man, eb)
        d = O.direct_decrypt(G, qbar, gs[0], texts, nonces)
        assert [(M, p.c, p.v) for M, p in d] == [(h(w["M"]), h(w["c"]), h(w["v"])) for w in v["direct"]]
        c = O.compensated_decrypt(G, qbar, gs[1], gs[2], texts, nonces)
        assert [(M, p.c, p.v, rk) for M, p, rk in c] == \
            [(h(w["M"]), h(w["c"]), h(w["v"]), h(w["recovery"])) for w in v["compensated_by_x2_for_x3"]]


@pytest.mark.parametrize("resp,pre", VARIANTS)
def test_each_variant_fails_under_the_others(resp, pre):
    G = O.production_group()
    K, qbar = h(FX["K"]), h(FX["qbar"])
    v = _variant(resp, pre)
    b = v["ballots"][0]
    ct = O.Ciphertext(h(b["cts"][0][0]), h(b["cts"][0][1]))
    pr = O.RangeProof(*[h(x) for x in b["rproofs"][0]])
    text = O.Ciphertext(*[h(x) for x in FX["texts"][0]])
    w = v["direct"][0]
    Ki = h(FX["guardians"][0]["commitments"][0])
    share = (h(w["M"]), O.GenericProof(h(w["c"]), h(w["v"])))
    for r2 in O.RESPONSES:
        for p2 in O.PREIMAGES:
            with O.proof_format(r2, p2):
                same = (r2, p2) == (resp, pre)
                assert O.verify_range_proof(G, K, qbar, ct, pr) == same, (r2, p2)
                assert O.verify_share(G, qbar, Ki, text, *share) == same, (r2, p2)
