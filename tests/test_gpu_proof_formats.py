"""The switchable proof conventions on the GPU (eg_ctx_set_proof_format: the response sign x the
challenge pre-image order, 6 variants; unpinned upstream): under each variant the encryptor
reproduces the fixture's bytes from its injected nonces, the verifier accepts that variant's
ballots and rejects every other variant's, the trustee reproduces its direct and compensated shares
and the mediator's share check accepts exactly them; tools/pin_format.py's pin_formats() names
the variant of each fixture set (and only it)."""
import json

import numpy as np
import pytest

import eg_oracle as O
from test_oracle_golden import GOLD, _arr, h

pytestmark = pytest.mark.gpu

FX = json.loads((GOLD / O.MODE4096 / "proof_formats.json").read_text())
VARIANTS = [(v["response"], v["preimage"]) for v in FX["variants"]]


def _arrays(v):
    nc, ns, va = FX["manifest"]
    nsel = nc * (ns + va)
    bs = v["ballots"]
    cts = np.stack([_arr([x for ct in b["cts"] for x in ct], 512).reshape(nsel, 2, 512) for b in bs])
    rp = np.stack([_arr([x for pr in b["rproofs"] for x in pr], 32).reshape(nsel, 4, 32) for b in bs])
    cp = np.stack([_arr([x for pr in b["cproofs"] for x in pr], 32).reshape(nc, 2, 32) for b in bs])
    votes = np.array([b["votes"] for b in bs], np.uint8)
    sn = np.stack([_arr([x for n4 in b["nonces"] for x in n4], 32).reshape(-1, 4, 32) for b in bs])
    cn = np.stack([_arr(b["contest_nonces"], 32) for b in bs])
    return cts, rp, cp, votes, sn, cn


@pytest.fixture()
def fmt_group(group):
    yield group
    group.proof_format = ("minus", "message_first")


@pytest.mark.parametrize("resp,pre", VARIANTS)
def test_variant_encrypt_verify_trustee_bit_exact(fmt_group, resp, pre):
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier, batch_encryption
    from electionguard.decrypt import partial_decrypt_batch, verify_shares
    group = fmt_group
    group.proof_format = (resp, pre)
    v = next(x for x in FX["variants"] if (x["response"], x["preimage"]) == (resp, pre))
    K, qbar = h(FX["K"]), h(FX["qbar"])
    man = Manifest(*FX["manifest"])
    key = ElectionKey(group, K)
    cts, rp, cp, votes, sn, cn = _arrays(v)
    eb = batch_encryption(group, key, qbar, man, votes, sn, cn)
    assert np.array_equal(eb.cts, cts) and np.array_equal(eb.rproof, rp) and np.array_equal(eb.cproof, cp)
    group.ct_encrypt = True  # the constant-time encryptor follows the convention too
    try:
        eb2 = batch_encryption(group, key, qbar, man, votes, sn, cn)
    finally:
        group.ct_encrypt = False
    assert np.array_equal(eb2.rproof, rp) and np.array_equal(eb2.cproof, cp)
    V = Verifier(group, key, qbar, man)
    for other in FX["variants"]:
        o_cts, o_rp, o_cp = _arrays(other)[:3]
        ok_s, ok_c, _ = V.verify(EncryptedBallots(o_cts, o_rp, o_cp), with_tally=False)
        if other is v:
            assert ok_s.all() and ok_c.all()
        else:  # every proof of another variant fails here
            assert not ok_s.any() and not ok_c.any(), (other["response"], other["preimage"])
    T = np.stack([_arr(t, 512) for t in FX["texts"]])
    N = _arr(FX["nonces"], 32)
    gs = FX["guardians"]
    M, pr = partial_decrypt_batch(group, h(gs[0]["coeffs"][0]), qbar, T, N)
    assert [(m.tobytes().hex(), p[0].tobytes().hex(), p[1].tobytes().hex()) for m, p in zip(M, pr)] == \
        [(w["M"], w["c"], w["v"]) for w in v["direct"]]
    share = O.poly_eval([h(a) for a in gs[2]["coeffs"]], 2, O.Q)
    Mc, prc = partial_decrypt_batch(group, share, qbar, T, N)
    assert [(m.tobytes().hex(), p[0].tobytes().hex(), p[1].tobytes().hex()) for m, p in zip(Mc, prc)] == \
        [(w["M"], w["c"], w["v"]) for w in v["compensated_by_x2_for_x3"]]
    Ki = h(gs[0]["commitments"][0])
    assert verify_shares(group, qbar, Ki, T, M, pr).all()
    rk = np.stack([_arr([w["recovery"]], 512)[0] for w in v["compensated_by_x2_for_x3"]])
    assert verify_shares(group, qbar, rk, T, Mc, prc).all()
    for other in FX["variants"]:
        if other is v:
            continue
        Mo = _arr([w["M"] for w in other["direct"]], 512)
        pro = np.stack([np.stack([_arr([w["c"]], 32)[0], _arr([w["v"]], 32)[0]]) for w in other["direct"]])
        assert not verify_shares(group, qbar, Ki, T, Mo, pro).any(), (other["response"], other["preimage"])


def test_pin_tool_names_each_variant(fmt_group):
    """pin_formats (tools/pin_format.py) on a record holding one variant's ballots and shares: exactly
    that (hash form, response, pre-image) combination verifies everything."""
    from electionguard.formats import pin_formats, summarize
    gs = FX["guardians"]
    for v in FX["variants"]:
        rec = {"K": FX["K"], "qbar": FX["qbar"], "manifest": FX["manifest"],
               "ballots": [{"cts": b["cts"], "rproofs": b["rproofs"], "cproofs": b["cproofs"]} for b in v["ballots"]],
               "shares": [{"text": FX["texts"][i], "key": gs[0]["commitments"][0], "M": w["M"], "c": w["c"],
                           "v": w["v"]} for i, w in enumerate(v["direct"])]}
        res = pin_formats(fmt_group, rec)
        hits = [(r["hash_format"], r["response"], r["preimage"]) for r in res if r["all_valid"]]
        # the response and the pre-image order are pinned; the hex form only when some hashed element
        # has a leading zero byte (else the fixed-width and minimal forms hash the same text)
        assert {(r, p) for _, r, p in hits} == {(v["response"], v["preimage"])}, hits
        assert ("fixed", v["response"], v["preimage"]) in hits
        assert summarize(res)["response"] == v["response"] and summarize(res)["preimage"] == v["preimage"]
    assert fmt_group.proof_format == ("minus", "message_first") and fmt_group.hash_format == "fixed"
