"""CPU: gRPC DecryptingTrusteeService wire path (decrypting_trustee_rpc.proto:9-45) with an
oracle-backed stand-in trustee — message layout, field numbers, error-string convention
(RunRemoteDecryptingTrustee.java:200-204) and the proxy's empty-list-on-error contract
(RemoteDecryptingTrusteeProxy.java:64-66)."""
import copy
import json
import random
import sys
from pathlib import Path

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


REF_FIELDS = Path(__file__).resolve().parent / "golden" / "reference_proto_fields.json"


def _pool_files(pool):
    """The FileDescriptorProtos behind electionguard.remote.POOL (what the server and proxy speak)."""
    from google.protobuf import descriptor_pb2
    out = {}
    for name in ("common.proto", "common_rpc.proto", "decrypting_trustee_rpc.proto"):
        fdp = descriptor_pb2.FileDescriptorProto()
        pool.FindFileByName(name).CopyToProto(fdp)
        out[name] = fdp
    return out


def wire_mismatches(files, ref) -> list:
    """Compare FileDescriptorProtos with the reference's extracted .proto table (both directions):
    every message and service the files define must exist in the reference's same-named file with
    the same fields (name, number, type, label, type name) and reserved ranges, and every message
    the reference's DecryptingTrusteeService reaches (requests, responses and the messages their
    fields name, transitively) must be defined here.  -> list of differences (empty = identical)."""
    from google.protobuf import descriptor_pb2
    F = descriptor_pb2.FieldDescriptorProto
    bad, have = [], {}
    for fn, fdp in files.items():
        rfile = ref["files"].get(fn)
        if rfile is None:
            bad.append(f"{fn}: no such reference file")
            continue
        if list(fdp.dependency) != rfile["imports"]:
            bad.append(f"{fn}: imports {list(fdp.dependency)} != {rfile['imports']}")
        if (fdp.package or None) != rfile["package"]:
            bad.append(f"{fn}: package {fdp.package!r} != {rfile['package']!r}")
        for m in fdp.message_type:
            have["." + m.name] = m
            rm = rfile["messages"].get(m.name)
            if rm is None:
                bad.append(f"{fn}: message {m.name} not in the reference")
                continue
            mine = sorted((f.name, f.number, F.Type.Name(f.type), F.Label.Name(f.label), f.type_name or None)
                          for f in m.field)
            theirs = sorted((f["name"], f["number"], f["type"], f["label"], f["type_name"]) for f in rm["fields"])
            if mine != theirs:
                bad.append(f"{fn}: {m.name} fields {mine} != reference {theirs}")
            rr = sorted([r.start, r.end] for r in m.reserved_range) + sorted(m.reserved_name)
            if rr != sorted(x for x in rm["reserved"] if isinstance(x, list)) + sorted(
                    x for x in rm["reserved"] if isinstance(x, str)):
                bad.append(f"{fn}: {m.name} reserved {rr} != reference {rm['reserved']}")
        for s in fdp.service:
            rs = rfile["services"].get(s.name)
            mine = [(x.name, x.input_type, x.output_type) for x in s.method]
            theirs = None if rs is None else [(x["name"], x["input"], x["output"]) for x in rs]
            if mine != theirs:
                bad.append(f"{fn}: service {s.name} methods {mine} != reference {theirs}")
    # reference -> here: everything the trustee service reaches
    rmsgs = {"." + n: m for f in ref["files"].values() for n, m in f["messages"].items()}
    todo = [t for x in ref["files"]["decrypting_trustee_rpc.proto"]["services"]["DecryptingTrusteeService"]
            for t in (x["input"], x["output"])]
    seen = set()
    while todo:
        t = todo.pop()
        if t in seen:
            continue
        seen.add(t)
        if t not in have:
            bad.append(f"reference message {t} (reached from DecryptingTrusteeService) is not defined here")
        todo.extend(f["type_name"] for f in rmsgs[t]["fields"] if f["type_name"])
    return bad


def test_wire_descriptors_match_the_reference_protos():
    """electionguard.remote.POOL == the reference's own .proto files (decrypting_trustee_rpc.proto:9-45,
    common.proto:8-28, common_rpc.proto:6-12), via the table tools/extract_proto_fields.py extracted."""
    from electionguard.remote import POOL
    ref = json.loads(REF_FIELDS.read_text())
    assert wire_mismatches(_pool_files(POOL), ref) == []


def test_wire_check_catches_one_field_edits():
    """A one-field edit of either side -- the reference table or the hand-built descriptors -- fails."""
    from electionguard.remote import POOL
    ref = json.loads(REF_FIELDS.read_text())
    # reference side: renumber, rename, retype, relabel one field; drop a reserved range; rename a method
    edits = [("challenge", "number", 5), ("challenge", "name", "c"), ("response", "type_name", ".ElementModP"),
             ("response", "label", "LABEL_REPEATED")]
    for fname, key, val in edits:
        r = copy.deepcopy(ref)
        f = next(x for x in r["files"]["common.proto"]["messages"]["GenericChaumPedersenProof"]["fields"]
                 if x["name"] == fname)
        f[key] = val
        assert wire_mismatches(_pool_files(POOL), r), (fname, key, val)
    r = copy.deepcopy(ref)
    r["files"]["common.proto"]["messages"]["GenericChaumPedersenProof"]["reserved"].pop()
    assert wire_mismatches(_pool_files(POOL), r)
    r = copy.deepcopy(ref)
    r["files"]["decrypting_trustee_rpc.proto"]["services"]["DecryptingTrusteeService"][2]["output"] = ".FinishRequest"
    assert wire_mismatches(_pool_files(POOL), r)
    # our side: one field of one request, a missing message, one method
    files = _pool_files(POOL)
    next(f for m in files["decrypting_trustee_rpc.proto"].message_type if m.name == "CompensatedDecryptionRequest"
         for f in m.field if f.name == "text").number = 4
    assert wire_mismatches(files, ref)
    files = _pool_files(POOL)
    del files["common.proto"].message_type[[m.name for m in files["common.proto"].message_type].index("ElementModQ")]
    assert wire_mismatches(files, ref)
    files = _pool_files(POOL)
    files["decrypting_trustee_rpc.proto"].service[0].method[0].input_type = ".CompensatedDecryptionRequest"
    assert wire_mismatches(files, ref)


@pytest.mark.skipif(not Path("/root/reference/src/main/proto").is_dir(), reason="the reference is not on this host")
def test_committed_table_is_the_reference_extraction():
    """Where the reference is present, re-extracting its .proto files gives the committed table."""
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
    import extract_proto_fields
    assert extract_proto_fields.extract() == json.loads(REF_FIELDS.read_text())


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
