"""Remote DecryptingTrustee over gRPC — wire-compatible with the reference.

Reference: ``service DecryptingTrusteeService`` (src/main/proto/decrypting_trustee_rpc.proto:9-45)
over the messages of src/main/proto/common.proto:8-28 and common_rpc.proto:8-14 (no
``package`` statement, so the method paths are ``/DecryptingTrusteeService/<method>``).
``protoc`` / ``grpc_tools`` are not in the image, so the descriptors are built here
programmatically with the reference's message names and field numbers.  They are pinned to the
reference's own IDL: tools/extract_proto_fields.py parses its .proto files into
tests/golden/reference_proto_fields.json, and tests/test_remote_wire.py requires POOL to equal
that table in both directions (every field's name, number, type, label and type name, reserved
ranges, the service's methods).

* :class:`DecryptingTrusteeServer` — the trustee process (``RunRemoteDecryptingTrustee``,
  RunRemoteDecryptingTrustee.java:58-120, handlers :180-247): each RPC is ONE GPU batch;
  exceptions become the response ``error`` string (:200-204), never a gRPC status.
* :class:`RemoteDecryptingTrusteeProxy` — the mediator-side ``DecryptingTrusteeIF``
  (RemoteDecryptingTrusteeProxy.java:30-122): on an error string or a transport failure it
  returns an EMPTY list (:64-66, :103-105), as the reference does.
"""
from __future__ import annotations

import logging
import threading
from concurrent import futures
from typing import List, Optional, Sequence

import numpy as np
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

log = logging.getLogger(__name__)

_F = descriptor_pb2.FieldDescriptorProto


def _msg(fd, name, fields):
    m = fd.message_type.add()
    m.name = name
    for fname, num, ftype, label, tname in fields:
        f = m.field.add()
        f.name, f.number, f.type, f.label = fname, num, ftype, label
        if tname:
            f.type_name = tname
    return m


def _build_pool():
    pool = descriptor_pool.DescriptorPool()
    opt, rep = _F.LABEL_OPTIONAL, _F.LABEL_REPEATED
    B, S, M, BOOL, U32 = _F.TYPE_BYTES, _F.TYPE_STRING, _F.TYPE_MESSAGE, _F.TYPE_BOOL, _F.TYPE_UINT32
    common = descriptor_pb2.FileDescriptorProto(name="common.proto", syntax="proto3")
    _msg(common, "ElementModP", [("value", 1, B, opt, None)])
    _msg(common, "ElementModQ", [("value", 1, B, opt, None)])
    _msg(common, "ElGamalCiphertext", [("pad", 1, M, opt, ".ElementModP"), ("data", 2, M, opt, ".ElementModP")])
    gp = _msg(common, "GenericChaumPedersenProof", [("challenge", 3, M, opt, ".ElementModQ"),
                                                    ("response", 4, M, opt, ".ElementModQ")])
    for lo in (1, 2):  # reserved 1; reserved 2;  (common.proto:24-25)
        r = gp.reserved_range.add()
        r.start, r.end = lo, lo + 1
    _msg(common, "UInt256", [("value", 1, B, opt, None)])
    pool.Add(common)
    crpc = descriptor_pb2.FileDescriptorProto(name="common_rpc.proto", syntax="proto3")
    _msg(crpc, "FinishRequest", [("all_ok", 1, BOOL, opt, None)])
    _msg(crpc, "ErrorResponse", [("error", 1, S, opt, None)])
    pool.Add(crpc)
    dt = descriptor_pb2.FileDescriptorProto(name="decrypting_trustee_rpc.proto", syntax="proto3",
                                            dependency=["common.proto", "common_rpc.proto"])
    _msg(dt, "DirectDecryptionRequest", [("extended_base_hash", 1, M, opt, ".ElementModQ"),
                                         ("text", 2, M, rep, ".ElGamalCiphertext")])
    _msg(dt, "DirectDecryptionResponse", [("error", 1, S, opt, None),
                                          ("results", 2, M, rep, ".DirectDecryptionResult")])
    _msg(dt, "DirectDecryptionResult", [("decryption", 1, M, opt, ".ElementModP"),
                                        ("proof", 2, M, opt, ".GenericChaumPedersenProof")])
    _msg(dt, "CompensatedDecryptionRequest", [("extended_base_hash", 1, M, opt, ".ElementModQ"),
                                              ("missing_guardian_id", 2, S, opt, None),
                                              ("text", 3, M, rep, ".ElGamalCiphertext")])
    _msg(dt, "CompensatedDecryptionResponse", [("error", 1, S, opt, None),
                                               ("results", 2, M, rep, ".CompensatedDecryptionResult")])
    _msg(dt, "CompensatedDecryptionResult", [("decryption", 1, M, opt, ".ElementModP"),
                                             ("proof", 2, M, opt, ".GenericChaumPedersenProof"),
                                             ("recoveryPublicKey", 3, M, opt, ".ElementModP")])
    svc = dt.service.add()
    svc.name = "DecryptingTrusteeService"
    for name, req, resp in [("directDecrypt", ".DirectDecryptionRequest", ".DirectDecryptionResponse"),
                            ("compensatedDecrypt", ".CompensatedDecryptionRequest", ".CompensatedDecryptionResponse"),
                            ("finish", ".FinishRequest", ".ErrorResponse")]:
        m = svc.method.add()
        m.name, m.input_type, m.output_type = name, req, resp
    pool.Add(dt)
    return pool


POOL = _build_pool()
MSG = {name: message_factory.GetMessageClass(POOL.FindMessageTypeByName(name)) for name in [
    "ElementModP", "ElementModQ", "ElGamalCiphertext", "GenericChaumPedersenProof", "UInt256", "FinishRequest",
    "ErrorResponse", "DirectDecryptionRequest", "DirectDecryptionResponse", "DirectDecryptionResult",
    "CompensatedDecryptionRequest", "CompensatedDecryptionResponse", "CompensatedDecryptionResult"]}
SERVICE = "DecryptingTrusteeService"


# ---- ConvertCommonProto (ConvertCommonProto.java:41-144) ----
def publish_p(x: int):
    return MSG["ElementModP"](value=int(x).to_bytes(512, "big"))


def publish_q(x: int):
    return MSG["ElementModQ"](value=int(x).to_bytes(32, "big"))


def import_int(m) -> Optional[int]:
    """new BigInteger(1, bytes); empty -> None (ConvertCommonProto.java:42-44, 51-53)."""
    if m is None or len(m.value) == 0:
        return None
    return int.from_bytes(m.value, "big")


def publish_ct(pad: int, data: int):
    return MSG["ElGamalCiphertext"](pad=publish_p(pad), data=publish_p(data))


def _p_wire(m) -> bytes:
    """An ElementModP's value as 512 big-endian bytes (new BigInteger(1, bytes), any length)."""
    b = m.value
    return b if len(b) == 512 else int.from_bytes(b, "big").to_bytes(512, "big")


def _q_wire(m) -> bytes:
    b = m.value
    return b if len(b) == 32 else int.from_bytes(b, "big").to_bytes(32, "big")


def _share_wire(results, recovery: bool = False):
    """(M (n, 512), proofs (n, 2, 32)[, recovery keys (n, 512)]) from response results; an empty
    element (importElementModP's null) raises ValueError."""
    def need(m, conv):
        if len(m.value) == 0:
            raise ValueError("result with an empty element")
        return conv(m)

    n = len(results)
    M = np.frombuffer(bytearray().join(need(r.decryption, _p_wire) for r in results), dtype=np.uint8).reshape(n, 512)
    pr = np.frombuffer(bytearray().join(need(r.proof.challenge, _q_wire) + need(r.proof.response, _q_wire)
                                        for r in results), dtype=np.uint8).reshape(n, 2, 32)
    if not recovery:
        return M, pr
    rk = np.frombuffer(bytearray().join(need(r.recoveryPublicKey, _p_wire) for r in results),
                       dtype=np.uint8).reshape(n, 512)
    return M, pr, rk


def _texts_from(req) -> np.ndarray:
    """The request's ciphertexts as an (n, 2, 512) array, straight from the wire bytes."""
    def ct(t) -> bytes:
        if not t.HasField("pad"):
            raise ValueError("ciphertext without pad")  # importCiphertext returns null (:60-62)
        return _p_wire(t.pad) + _p_wire(t.data)

    raw = bytearray().join(ct(t) for t in req.text)
    return np.frombuffer(raw, dtype=np.uint8).reshape(-1, 2, 512)


class DecryptingTrusteeServer:
    """gRPC DecryptingTrusteeService backed by a GPU DecryptingTrustee (one GPU per process)."""

    def __init__(self, group, trustee, port: int = 0, host: str = "127.0.0.1", max_workers: int = 4):
        import grpc

        self.group, self.trustee = group, trustee
        self._done = threading.Event()
        self.all_ok: Optional[bool] = None
        handlers = {
            "directDecrypt": grpc.unary_unary_rpc_method_handler(
                self._direct, request_deserializer=MSG["DirectDecryptionRequest"].FromString,
                response_serializer=MSG["DirectDecryptionResponse"].SerializeToString),
            "compensatedDecrypt": grpc.unary_unary_rpc_method_handler(
                self._compensated, request_deserializer=MSG["CompensatedDecryptionRequest"].FromString,
                response_serializer=MSG["CompensatedDecryptionResponse"].SerializeToString),
            "finish": grpc.unary_unary_rpc_method_handler(
                self._finish, request_deserializer=MSG["FinishRequest"].FromString,
                response_serializer=MSG["ErrorResponse"].SerializeToString),
        }
        # gRPC's default limits, as the reference's server (RunRemoteDecryptingTrustee.java:111-112):
        # 4 MiB inbound; RemoteDecryptingTrusteeProxy keeps every request and response below it
        self.server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
        self.server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
        self.port = self.server.add_insecure_port(f"{host}:{port}")

    def start(self) -> "DecryptingTrusteeServer":
        self.server.start()
        return self

    def wait(self, timeout: Optional[float] = None) -> bool:
        return self._done.wait(timeout)

    def stop(self) -> None:
        self.server.stop(grace=1).wait()

    def _texts(self, req):
        """(n, 2, 512) array for trustees that take one (DecryptingTrustee.accepts_arrays), else
        (pad, data) int pairs as the reference's importCiphertext gives them."""
        T = _texts_from(req)
        if getattr(self.trustee, "accepts_arrays", False):
            return T
        return [(int.from_bytes(t[0].tobytes(), "big"), int.from_bytes(t[1].tobytes(), "big")) for t in T]

    # RunRemoteDecryptingTrustee.directDecrypt (:180-208)
    def _direct(self, req, ctx):
        resp = MSG["DirectDecryptionResponse"]()
        try:
            texts = self._texts(req)
            qbar = import_int(req.extended_base_hash)
            if hasattr(self.trustee, "directDecryptArrays"):  # shares straight from the GPU's bytes
                M, pr = self.trustee.directDecryptArrays(self.group, texts, qbar, None)
                for i in range(len(M)):
                    x = resp.results.add()
                    x.decryption.value = M[i].tobytes()
                    x.proof.challenge.value = pr[i, 0].tobytes()
                    x.proof.response.value = pr[i, 1].tobytes()
                return resp
            res = self.trustee.directDecrypt(self.group, texts, qbar, None)
            for r in res:  # field by field: a third of the cost of nested message constructors
                x = resp.results.add()
                x.decryption.value = int(r.partialDecryption).to_bytes(512, "big")
                x.proof.challenge.value = int(r.proof.c).to_bytes(32, "big")
                x.proof.response.value = int(r.proof.v).to_bytes(32, "big")
        except Exception as e:  # error string, not a gRPC status (:200-204)
            log.exception("directDecrypt failed")
            del resp.results[:]
            resp.error = str(e) or "Unknown"
        return resp

    # RunRemoteDecryptingTrustee.compensatedDecrypt (:217-247)
    def _compensated(self, req, ctx):
        resp = MSG["CompensatedDecryptionResponse"]()
        try:
            texts = self._texts(req)
            qbar = import_int(req.extended_base_hash)
            if hasattr(self.trustee, "compensatedDecryptArrays"):
                M, pr, rk = self.trustee.compensatedDecryptArrays(self.group, req.missing_guardian_id, texts, qbar,
                                                                  None)
                rkb = rk.tobytes()
                for i in range(len(M)):
                    x = resp.results.add()
                    x.decryption.value = M[i].tobytes()
                    x.proof.challenge.value = pr[i, 0].tobytes()
                    x.proof.response.value = pr[i, 1].tobytes()
                    x.recoveryPublicKey.value = rkb
                return resp
            res = self.trustee.compensatedDecrypt(self.group, req.missing_guardian_id, texts, qbar, None)
            for r in res:
                x = resp.results.add()
                x.decryption.value = int(r.partialDecryption).to_bytes(512, "big")
                x.proof.challenge.value = int(r.proof.c).to_bytes(32, "big")
                x.proof.response.value = int(r.proof.v).to_bytes(32, "big")
                x.recoveryPublicKey.value = int(r.recoveredPublicKeyShare).to_bytes(512, "big")
        except Exception as e:
            log.exception("compensatedDecrypt failed")
            del resp.results[:]
            resp.error = str(e) or "Unknown"
        return resp

    def _finish(self, req, ctx):
        self.all_ok = bool(req.all_ok)
        self._done.set()
        return MSG["ErrorResponse"]()


# Texts per RPC so that every message stays under gRPC's default 4 MiB inbound limit on both
# ends: a request text is ~1,039 B on the wire, a compensated result ~1,112 B (M, proof, recovery
# key), so 3,500 texts are ~3.9 MB.  The reference sends the whole tally in one RPC
# (RemoteDecryptingTrusteeProxy.java:55-63), which its default channels reject above ~3.8k texts.
MAX_TEXTS_PER_RPC = 3500


class RemoteDecryptingTrusteeProxy:
    """Mediator-side DecryptingTrusteeIF over gRPC (RemoteDecryptingTrusteeProxy.java).  A call
    over more than ``max_texts_per_rpc`` texts is split into consecutive RPCs whose results are
    concatenated in text order; if any of them fails the call returns [] (:64-66, :103-105)."""

    def __init__(self, trustee_id: str, url: str, x: int, public_key: int,
                 max_texts_per_rpc: int = MAX_TEXTS_PER_RPC):
        import grpc

        self._id, self._x, self._K = trustee_id, x, public_key
        self.max_texts = max_texts_per_rpc
        # default message limits (4 MiB inbound) and the reference's 1-minute keepalive
        # (RemoteDecryptingTrusteeProxy.java:202-210)
        self.channel = grpc.insecure_channel(url, options=[("grpc.keepalive_time_ms", 60000)])
        mk = lambda m, req, resp: self.channel.unary_unary(f"/{SERVICE}/{m}", request_serializer=req.SerializeToString,
                                                           response_deserializer=resp.FromString)
        self._direct = mk("directDecrypt", MSG["DirectDecryptionRequest"], MSG["DirectDecryptionResponse"])
        self._comp = mk("compensatedDecrypt", MSG["CompensatedDecryptionRequest"], MSG["CompensatedDecryptionResponse"])
        self._finish = mk("finish", MSG["FinishRequest"], MSG["ErrorResponse"])

    def id(self) -> str:
        return self._id

    def xCoordinate(self) -> int:
        return self._x

    def electionPublicKey(self) -> int:
        return self._K

    def _requests(self, make, texts):
        """Consecutive requests of at most max_texts ciphertexts each, filled from the texts'
        512-byte wire form (the bytes publish_ct writes)."""
        from .decrypt import _texts_array

        T = _texts_array(texts)
        for a in range(0, len(T), self.max_texts):
            req = make()
            for t in T[a:a + self.max_texts]:
                x = req.text.add()
                x.pad.value = t[0].tobytes()
                x.data.value = t[1].tobytes()
            yield req

    def _call(self, name, stub, requests):
        import grpc

        results = []
        for req in requests:
            try:
                resp = stub(req)
            except grpc.RpcError as e:
                log.error("%s failed: %s", name, e)
                return None
            if resp.error:
                log.error("%s failed: %s", name, resp.error)
                return None
            if len(resp.results) != len(req.text):
                # a short (or long) batch would pair every later result with the wrong text
                log.error("%s: %d results for %d texts", name, len(resp.results), len(req.text))
                return None
            results.extend(resp.results)
        return results

    def directDecrypt(self, group, texts, extendedBaseHash: int, nonce=None):
        reqs = self._requests(lambda: MSG["DirectDecryptionRequest"](extended_base_hash=publish_q(extendedBaseHash)),
                              texts)
        res = self._call("directDecrypt", self._direct, reqs)
        if res is None:
            return []
        from .decrypt import ShareBatch

        try:
            return ShareBatch(*_share_wire(res))
        except (ValueError, OverflowError) as e:  # an empty (null) or oversized element
            log.error("directDecrypt: %s", e)
            return []

    def compensatedDecrypt(self, group, missingGuardianId: str, texts, extendedBaseHash: int, nonce=None):
        reqs = self._requests(lambda: MSG["CompensatedDecryptionRequest"](
            extended_base_hash=publish_q(extendedBaseHash), missing_guardian_id=missingGuardianId), texts)
        res = self._call("compensatedDecrypt", self._comp, reqs)
        if res is None:
            return []
        from .decrypt import ShareBatch

        try:
            return ShareBatch(*_share_wire(res, recovery=True))
        except (ValueError, OverflowError) as e:
            log.error("compensatedDecrypt: %s", e)
            return []

    def finish(self, all_ok: bool) -> str:
        import grpc

        try:
            return self._finish(MSG["FinishRequest"](all_ok=all_ok)).error
        except grpc.RpcError as e:
            return str(e)

    def close(self) -> None:
        self.channel.close()
