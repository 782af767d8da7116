"""CPU: gRPC DecryptingTrusteeService wire path (decrypting_trustee_rpc.proto:9-45) with an
oracle-backed stand-in trustee — message layout, field numbers, error-string convention
(RunRemoteDecryptingTrustee.java:200-204) and the proxy's empty-list-on-error contract
(RemoteDecryptingTrusteeProxy.java:64-66)."""
import random

import pytest

import eg_oracle as O


class OracleTrustee:
    """Stand-in DecryptingTrusteeIF computing with the CPU oracle (test only)."""

    def __init__(self, G, qbar_nonces, guardian, missing=None):
        self.G, self.g, self.missing = G, guardian, missing or {}
        self.rng = random.Random(99)

    def directDecrypt(self, group, texts, qbar, nonce=None):
        from electionguard.decrypt import DirectDecryptionAndProof, GenericChaumPedersenProof
        cts = [O.Ciphertext(a, b) for a, b in texts]
        res = O.direct_decrypt(self.G, qbar, self.g, cts, [self.rng.randrange(1, self.G.q) for _ in cts])
        return [DirectDecryptionAndProof(M, GenericChaumPedersenProof(p.c, p.v)) for M, p in res]

    def compensatedDecrypt(self, group, missing_id, texts, qbar, nonce=None):
        from electionguard.decrypt import CompensatedDecryptionAndProof, GenericChaumPedersenProof
        if missing_id not in self.missing:
            raise KeyError(f"no backup for {missing_id}")
        cts = [O.Ciphertext(a, b) for a, b in texts]
        res = O.compensated_decrypt(self.G, qbar, self.g, self.missing[missing_id], cts,
                                    [self.rng.randrange(1, self.G.q) for _ in cts])
        return [CompensatedDecryptionAndProof(M, GenericChaumPedersenProof(p.c, p.v), rk) for M, p, rk in res]


@pytest.fixture(scope="module")
def setup():
    G = O.production_group()
    rng = random.Random(31)
    gs, K = O.key_ceremony(G, 3, 2, rng)
    qbar = rng.randrange(G.q)
    texts = [O.encrypt(G, K, rng.randrange(3), rng.randrange(1, G.q)) for _ in range(4)]
    return G, gs, K, qbar, texts


def test_descriptors_match_reference_field_numbers():
    from electionguard.remote import POOL
    f = POOL.FindMessageTypeByName("GenericChaumPedersenProof").fields_by_name
    assert (f["challenge"].number, f["response"].number) == (3, 4)
    c = POOL.FindMessageTypeByName("CompensatedDecryptionRequest").fields_by_name
    assert (c["extended_base_hash"].number, c["missing_guardian_id"].number, c["text"].number) == (1, 2, 3)
    r = POOL.FindMessageTypeByName("CompensatedDecryptionResult").fields_by_name
    assert r["recoveryPublicKey"].number == 3
    svc = POOL.FindServiceByName("DecryptingTrusteeService")
    assert [m.name for m in svc.methods] == ["directDecrypt", "compensatedDecrypt", "finish"]


def test_direct_and_compensated_over_grpc(setup):
    from electionguard.remote import DecryptingTrusteeServer, RemoteDecryptingTrusteeProxy
    G, gs, K, qbar, texts = setup
    tr = OracleTrustee(G, None, gs[0], {gs[2].gid: gs[2]})
    srv = DecryptingTrusteeServer(None, tr).start()
    try:
        px = RemoteDecryptingTrusteeProxy(gs[0].gid, f"127.0.0.1:{srv.port}", gs[0].x, gs[0].K)
        res = px.directDecrypt(None, [(t.pad, t.data) for t in texts], qbar)
        assert len(res) == len(texts)
        for t, r in zip(texts, res):
            assert r.partialDecryption == pow(t.pad, gs[0].s, G.p)
            assert O.verify_share(G, qbar, gs[0].K, t, r.partialDecryption, O.GenericProof(r.proof.c, r.proof.v))
        cres = px.compensatedDecrypt(None, gs[2].gid, [(t.pad, t.data) for t in texts], qbar)
        share = O.poly_eval(gs[2].coeffs, gs[0].x, G.q)
        assert [r.partialDecryption for r in cres] == [pow(t.pad, share, G.p) for t in texts]
        assert all(r.recoveredPublicKeyShare == O.recovery_public_key(G, gs[2], gs[0].x) for r in cres)
        # error string -> empty list
        assert px.compensatedDecrypt(None, "nobody", [(t.pad, t.data) for t in texts], qbar) == []
        assert px.finish(True) == ""
        assert srv.wait(5) and srv.all_ok is True
        px.close()
    finally:
        srv.stop()


def test_proxy_transport_failure_returns_empty(setup):
    from electionguard.remote import RemoteDecryptingTrusteeProxy
    G, gs, K, qbar, texts = setup
    px = RemoteDecryptingTrusteeProxy("x", "127.0.0.1:1", 1, 1)
    assert px.directDecrypt(None, [(texts[0].pad, texts[0].data)], qbar) == []
    px.close()


class EchoTrustee:
    """Stand-in whose results are cheap functions of the texts (wire sizing test only): M = pad,
    proof (c, v) = (i, data mod q), recovery key = data.  Records the batch sizes it served."""

    def __init__(self, q):
        self.q, self.calls = q, []

    def directDecrypt(self, group, texts, qbar, nonce=None):
        from electionguard.decrypt import DirectDecryptionAndProof, GenericChaumPedersenProof
        self.calls.append(len(texts))
        return [DirectDecryptionAndProof(a, GenericChaumPedersenProof(qbar, b % self.q)) for a, b in texts]

    def compensatedDecrypt(self, group, missing_id, texts, qbar, nonce=None):
        from electionguard.decrypt import CompensatedDecryptionAndProof, GenericChaumPedersenProof
        self.calls.append(len(texts))
        return [CompensatedDecryptionAndProof(a, GenericChaumPedersenProof(qbar, b % self.q), b) for a, b in texts]


def test_ten_thousand_texts_fit_default_channel_limits():
    """A 10k-text tally through default-limit channels (4 MiB inbound on both ends, as the
    reference's RemoteDecryptingTrusteeProxy.java:202-210 and its server): the proxy splits it
    into <= 3,500-text RPCs and reassembles the results in text order."""
    from electionguard.remote import MAX_TEXTS_PER_RPC, DecryptingTrusteeServer, RemoteDecryptingTrusteeProxy
    G = O.production_group()
    rng = random.Random(4)
    n = 10_000
    texts = [(rng.randrange(G.p), rng.randrange(G.p)) for _ in range(n)]
    tr = EchoTrustee(G.q)
    srv = DecryptingTrusteeServer(None, tr).start()
    try:
        px = RemoteDecryptingTrusteeProxy("g1", f"127.0.0.1:{srv.port}", 1, 1)
        res = px.directDecrypt(None, texts, 77)
        assert len(res) == n and tr.calls == [3500, 3500, 3000] and MAX_TEXTS_PER_RPC == 3500
        assert all(r.partialDecryption == a and r.proof.v == b % G.q for r, (a, b) in zip(res, texts))
        tr.calls.clear()
        cres = px.compensatedDecrypt(None, "g2", texts, 77)
        assert len(cres) == n and tr.calls == [3500, 3500, 3000]
        assert all(r.recoveredPublicKeyShare == b for r, (a, b) in zip(cres, texts))
        # one RPC of the whole tally, as the reference sends it, exceeds the default limit
        big = RemoteDecryptingTrusteeProxy("g1", f"127.0.0.1:{srv.port}", 1, 1, max_texts_per_rpc=n)
        assert big.directDecrypt(None, texts, 77) == []
        big.close()
        px.close()
    finally:
        srv.stop()


class ShortTrustee(EchoTrustee):
    """Echo stand-in that drops the last result of its second batch without reporting an error."""

    def directDecrypt(self, group, texts, qbar, nonce=None):
        res = super().directDecrypt(group, texts, qbar, nonce)
        return res[:-1] if len(self.calls) == 2 else res


def test_short_batch_without_error_fails_the_whole_call():
    """A trustee answering one of the proxy's RPCs with fewer results than texts (and no error
    string) must not shift the later results onto the wrong texts: the proxy returns the
    reference's failure value, an empty list (RemoteDecryptingTrusteeProxy.java:64-66)."""
    from electionguard.remote import DecryptingTrusteeServer, RemoteDecryptingTrusteeProxy
    G = O.production_group()
    rng = random.Random(5)
    texts = [(rng.randrange(G.p), rng.randrange(G.p)) for _ in range(9)]
    tr = ShortTrustee(G.q)
    srv = DecryptingTrusteeServer(None, tr).start()
    try:
        px = RemoteDecryptingTrusteeProxy("g1", f"127.0.0.1:{srv.port}", 1, 1, max_texts_per_rpc=4)
        assert px.directDecrypt(None, texts, 7) == []
        assert tr.calls == [4, 4]  # the third RPC is never sent
        px.close()
    finally:
        srv.stop()
