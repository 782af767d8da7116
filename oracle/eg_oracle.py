"""CPU oracle for the batched 4096-bit modexp path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker.  The product path
(``electionguard-remote_amd/``) never imports it.

PARITY STATUS: parity unpinned.  The reference (JohnLCaron/electionguard-remote)
holds no arithmetic: every group / ElGamal / proof / tally / decryption operation
lives in the third-party module
``electionguard-kotlin-multiplatform:electionguard-kotlin-multiplatform-jvm:1.0-SNAPSHOT``
(build.gradle.kts:55), fetched from an authenticated Maven repo
(build.gradle.kts:25-31) and absent here; there is no JDK either.  The
reference's own tests pin nothing on this path
(src/test/java/electionguard/keyceremony/RemoteKeyCeremonyTrusteeTest.java:10-14
only asserts a protobuf builder is non-null).  What IS pinned:

* group-level ops (powP, multP, multInv, products) are uniquely defined integers
  mod p, so equality with ``java.math.BigInteger.modPow`` is a mathematical fact;
  this module computes them with CPython ``int`` and is cross-checked against an
  independent OpenSSL-BN restatement (``oracle/eg_oracle_c.c``);
* the group: upstream 1.0-SNAPSHOT (2022) implements ElectionGuard 1.0, whose
  ``Mode4096`` group is built from Euler's gamma.  :func:`derive_group` re-derives it
  from gamma and the published delta, and the result is pinned twice: q | p - 1 (2^-256
  chance for a wrong delta) and g = 2^r mod p reproducing the published EG 1.0
  generator's leading digits.  The EG 2.0 (ln 2) group is a named second option
  (``Mode4096_V2``); every golden fixture exists for both;
* protocol-level restatements (ElGamal, Chaum-Pedersen, tally, threshold
  decryption) follow the ElectionGuard 1.0 spec (cited by the reference at
  src/main/proto/keyceremony_trustee_rpc.proto:40) and the reference's wire
  formats (src/main/proto/common.proto:6-48, decrypting_trustee_rpc.proto:15-45).
  The Fiat-Shamir hash pre-image format and nonce derivation are upstream and
  unpinned; this oracle defines them (``hash_elems``) and the HIP path must match
  this oracle bit-for-bit.

Reference call sites into the restated upstream code:
KUtils.java:11 (group), ConvertCommonProto.java:41-68 (element import, unchecked),
RunRemoteWorkflowTest.java:140-141 (batchEncryption), :151 (runAccumulateBallots),
:179-182 (Verifier), RunRemoteDecryptingTrustee.java:189-193 (directDecrypt),
:227-232 (compensatedDecrypt), RunRemoteDecryptor.java:261-262 (Decryption.decrypt).
"""
from __future__ import annotations

import hashlib
import random
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

# --------------------------------------------------------------------------------------
# Group constants (EG 1.0, ProductionMode.Mode4096 — KUtils.java:10-12)
# --------------------------------------------------------------------------------------

Q = 2**256 - 189
# The two 4096-bit groups (electionguard-remote_amd/electionguard/core/constants.py):
#   Mode4096    -- ElectionGuard 1.0, the group of the reference's upstream 1.0-SNAPSHOT
#                  (build.gradle.kts:26,55; 2022):
#                  p = 2^4096 - 2^3840 + 2^256 (floor(2^3584 gamma) + DELTA) - 1
#   Mode4096_V2 -- ElectionGuard 2.0 (ln 2 in place of Euler's gamma), a named option:
#                  p = 2^4096 - 2^3840 + 2^256 (floor(2^3584 ln 2) + DELTA') + 2^256 - 1
# In both, r = (p-1)/q and g = 2^r mod p.  DELTA is the published EG 1.0 correction term;
# q | p - 1 pins it (a wrong value passes with probability 2^-256), and the derived g must
# reproduce the published EG 1.0 generator's leading digits 037DE384F98F6E03...
# DELTA' is the first delta of its residue class with p and (p-1)/(2q) both prime (checked
# by a sieve run when this restatement was written: k = 2,487,002 classes above the base).
MODE4096, MODE4096_V2 = "Mode4096", "Mode4096_V2"
_DELTAS = {
    MODE4096: 495448529856135475846147600290107731951815687842437876083937612367400355133042233301,
    MODE4096_V2: int("25f2da6646e943db028bd17d654a5fe9dc13e777f86b494195b2a55ba0d6d33e6d9d4f", 16),
}
EG1_G_PREFIX = "037DE384F98F6E038D2A3141825B33D5"  # published EG 1.0 generator, leading digits


def derive_group(mode: str = MODE4096) -> Tuple[int, int, int, int]:
    """Re-derive (p, q, g, r) of a 4096-bit group from its constant (gamma or ln 2)."""
    import mpmath

    with mpmath.workprec(3700):
        c = mpmath.euler if mode == MODE4096 else mpmath.log(2)
        x = int(mpmath.floor(c * mpmath.mpf(2) ** 3584))
    d = _DELTAS[mode]
    if mode == MODE4096:
        p = 2**4096 - 2**3840 + 2**256 * (x + d) - 1
    else:
        p = 2**4096 - 2**3840 + 2**256 * (x + d) + 2**256 - 1
    assert (p - 1) % Q == 0, "q does not divide p-1: constants mis-derived"
    r = (p - 1) // Q
    g = pow(2, r, p)
    assert g != 1 and pow(g, Q, p) == 1
    if mode == MODE4096:
        assert f"{g:01024X}".startswith(EG1_G_PREFIX), "EG 1.0 generator prefix mismatch"
    return p, Q, g, r


def derive_production_group() -> Tuple[int, int, int, int]:
    """KUtils.productionGroup() (KUtils.java:10-12): Mode4096, the EG 1.0 group."""
    return derive_group(MODE4096)


_GROUP_CACHE: Dict[str, Tuple[int, int, int, int]] = {}


def production_group(mode: str = MODE4096) -> "Group":
    if mode not in _GROUP_CACHE:
        _GROUP_CACHE[mode] = derive_group(mode)
    p, q, g, r = _GROUP_CACHE[mode]
    return Group(p, q, g)


@dataclass(frozen=True)
class Group:
    p: int
    q: int
    g: int

    # ---- group-level ops (upstream ElementModP / GroupContext) ----
    def powP(self, b: int, e: int) -> int:
        """ElementModP.powP: BigInteger.modPow semantics (base reduced mod p)."""
        return pow(b % self.p, e, self.p)

    def gPowP(self, e: int) -> int:
        return pow(self.g, e, self.p)

    def multP(self, a: int, b: int) -> int:
        return (a * b) % self.p

    def multInv(self, a: int) -> int:
        return pow(a % self.p, -1, self.p)

    def prodP(self, xs: Sequence[int]) -> int:
        acc = 1
        for x in xs:
            acc = (acc * x) % self.p
        return acc

    def dlogG(self, y: int, max_result: int) -> Optional[int]:
        """Discrete log base g by incremental table, as upstream dLogG (§8a a14)."""
        acc = 1
        for t in range(max_result + 1):
            if acc == y:
                return t
            acc = (acc * self.g) % self.p
        return None


# --------------------------------------------------------------------------------------
# Hashing (Fiat-Shamir).  Pre-image format: EG 1.0-style hash_elems with fixed-width
# upper-case hex: "|" + "|".join(hex(e)) + "|", SHA-256, big-endian int mod q.
# ElementModP -> 1024 hex chars (512 B BE, common.proto:6-10);
# ElementModQ -> 64 hex chars (32 B BE, common.proto:12-16).  Unpinned upstream.
# --------------------------------------------------------------------------------------

# The hex form is switchable because upstream's is unpinned: "fixed" (the default above) or
# "minimal" (the integer's even-length hex, leading zero bytes dropped, 0 -> "00": the
# electionguard-python 1.x to_hex form).  Tests switch it with `with hash_format("minimal"):`.
HASH_FORMAT = "fixed"


class hash_format:
    def __init__(self, fmt: str):
        assert fmt in ("fixed", "minimal")
        self.fmt = fmt

    def __enter__(self):
        global HASH_FORMAT
        self.prev, HASH_FORMAT = HASH_FORMAT, self.fmt

    def __exit__(self, *exc):
        global HASH_FORMAT
        HASH_FORMAT = self.prev


def _hexb(b: bytes) -> str:
    if HASH_FORMAT == "minimal":
        b = b.lstrip(b"\0") or b"\0"
    return b.hex().upper()


def hexP(x: int) -> str:
    return _hexb(x.to_bytes(512, "big"))


def hexQ(x: int) -> str:
    return _hexb(x.to_bytes(32, "big"))


def hash_elems(q: int, *elems: Tuple[str, int]) -> int:
    """elems: sequence of ("P"|"Q", value)."""
    parts = [hexP(v) if kind == "P" else hexQ(v) for kind, v in elems]
    msg = ("|" + "|".join(parts) + "|").encode("ascii")
    return int.from_bytes(hashlib.sha256(msg).digest(), "big") % q


# The two other unpinned proof conventions, switchable like the hex form (eg_ctx_set_proof_format):
#   RESPONSE "minus" (default): v = u - c x, checked as a = g^v X^c;
#            "plus": v = u + c x, checked as g^v = a X^c (a = g^v X^-c) -- ElectionGuard 1.0's spec form;
#   PREIMAGE (the hashed elements after Q-bar):
#            "message_first" (default): message, commitments, extra -- (alpha, beta, a0, b0, a1, b1),
#                                       (A, B, a, b), (pad, data, a, b, M);
#            "commitments_first": commitments, message, extra;
#            "with_key": the public key (K; the guardian's K_i = g^s for a share), message, commitments,
#                        extra.
# Tests switch them with `with proof_format("plus", "with_key"):`.
RESPONSES = ("minus", "plus")
PREIMAGES = ("message_first", "commitments_first", "with_key")
RESPONSE, PREIMAGE = "minus", "message_first"


class proof_format:
    def __init__(self, response: str = "minus", preimage: str = "message_first"):
        assert response in RESPONSES and preimage in PREIMAGES
        self.fmt = (response, preimage)

    def __enter__(self):
        global RESPONSE, PREIMAGE
        self.prev, (RESPONSE, PREIMAGE) = (RESPONSE, PREIMAGE), self.fmt

    def __exit__(self, *exc):
        global RESPONSE, PREIMAGE
        RESPONSE, PREIMAGE = self.prev


def _resp_exp(q: int, c: int) -> int:
    """The exponent the public base is raised to when recomputing a commitment: c (minus: a = g^v X^c)
    or -c (plus: a = g^v X^-c)."""
    return c % q if RESPONSE == "minus" else (-c) % q


def _response(q: int, u: int, c: int, x: int) -> int:
    return (u - c * x) % q if RESPONSE == "minus" else (u + c * x) % q


def challenge(q: int, qbar: int, key: int, msg: Sequence[int], comm: Sequence[int], extra: Sequence[int] = ()) -> int:
    """H(Q-bar, elements in the PREIMAGE order) mod q; every element an ElementModP."""
    if PREIMAGE == "message_first":
        els = [*msg, *comm, *extra]
    elif PREIMAGE == "commitments_first":
        els = [*comm, *msg, *extra]
    else:
        els = [key, *msg, *comm, *extra]
    return hash_elems(q, ("Q", qbar), *(("P", e) for e in els))


# --------------------------------------------------------------------------------------
# ElGamal + Chaum-Pedersen (compact (c, v) proofs: common.proto:23-28)
# --------------------------------------------------------------------------------------

@dataclass
class Ciphertext:
    pad: int   # alpha = g^R
    data: int  # beta  = K^R g^m


@dataclass
class RangeProof:
    """Disjunctive 0/1 Chaum-Pedersen proof, compact: (c0, v0), (c1, v1)."""
    c0: int
    v0: int
    c1: int
    v1: int


@dataclass
class GenericProof:
    """GenericChaumPedersenProof(c, v) — common.proto:23-28."""
    c: int
    v: int


def encrypt(G: Group, K: int, m: int, R: int) -> Ciphertext:
    return Ciphertext(G.gPowP(R), G.multP(G.powP(K, R), G.gPowP(m)))


def range_commitments(G: Group, K: int, ct: Ciphertext, pr: RangeProof) -> Tuple[int, int, int, int]:
    """Verifier recompute: a_j = g^{v_j} alpha^{e_j}, b_j = K^{v_j} (beta g^-j)^{e_j}, e_j = c_j
    (RESPONSE minus) or -c_j (plus)."""
    q = G.q
    e0, e1 = _resp_exp(q, pr.c0), _resp_exp(q, pr.c1)
    a0 = G.multP(G.gPowP(pr.v0), G.powP(ct.pad, e0))
    b0 = G.multP(G.powP(K, pr.v0), G.powP(ct.data, e0))
    a1 = G.multP(G.gPowP(pr.v1), G.powP(ct.pad, e1))
    b1 = G.prodP([G.powP(K, pr.v1), G.powP(ct.data, e1), G.gPowP((q - e1) % q)])
    return a0, b0, a1, b1


def range_challenge(G: Group, qbar: int, ct: Ciphertext, a0: int, b0: int, a1: int, b1: int, K: int = 0) -> int:
    return challenge(G.q, qbar, K, (ct.pad, ct.data), (a0, b0, a1, b1))


def make_range_proof(G: Group, K: int, qbar: int, ct: Ciphertext, m: int, R: int,
                     u: int, c_fake: int, v_fake: int) -> RangeProof:
    """Prover with known nonce R and injected proof nonces (u, c_fake, v_fake)."""
    q = G.q
    f = 1 - m
    a_real, b_real = G.gPowP(u), G.powP(K, u)
    # fake branch f: a_f = g^{v_f} alpha^{e_f}, b_f = K^{v_f} (beta g^{-f})^{e_f}, e_f = +-c_f
    ef = _resp_exp(q, c_fake)
    a_fake = G.multP(G.gPowP(v_fake), G.powP(ct.pad, ef))
    b_fake = G.prodP([G.powP(K, v_fake), G.powP(ct.data, ef), G.gPowP((q - f * ef) % q)])
    if m == 0:
        a0, b0, a1, b1 = a_real, b_real, a_fake, b_fake
    else:
        a0, b0, a1, b1 = a_fake, b_fake, a_real, b_real
    c = range_challenge(G, qbar, ct, a0, b0, a1, b1, K)
    c_real = (c - c_fake) % q
    v_real = _response(q, u, c_real, R)
    if m == 0:
        return RangeProof(c_real, v_real, c_fake, v_fake)
    return RangeProof(c_fake, v_fake, c_real, v_real)


def is_valid_residue(G: Group, x: int) -> bool:
    """ElementModP.isValidResidue (EG 1.0 verifier): 0 <= x < p and x^q == 1 mod p, i.e. x is
    in the order-q subgroup.  The reference imports elements unchecked
    (ConvertCommonProto.java:50-57) and leaves this to Verifier (RunRemoteWorkflowTest.java:179-182)."""
    return 0 < x < G.p and pow(x, G.q, G.p) == 1


def verify_range_proof(G: Group, K: int, qbar: int, ct: Ciphertext, pr: RangeProof) -> bool:
    q, p = G.q, G.p
    if not (is_valid_residue(G, ct.pad) and is_valid_residue(G, ct.data)):
        return False
    if not all(0 <= x < q for x in (pr.c0, pr.v0, pr.c1, pr.v1)):
        return False
    a0, b0, a1, b1 = range_commitments(G, K, ct, pr)
    return (pr.c0 + pr.c1) % q == range_challenge(G, qbar, ct, a0, b0, a1, b1, K)


def constant_commitments(G: Group, K: int, A: int, B: int, limit: int, pr: GenericProof) -> Tuple[int, int]:
    q = G.q
    e = _resp_exp(q, pr.c)
    a = G.multP(G.gPowP(pr.v), G.powP(A, e))
    b = G.prodP([G.powP(K, pr.v), G.powP(B, e), G.gPowP((q - (limit * e) % q) % q)])
    return a, b


def constant_challenge(G: Group, qbar: int, A: int, B: int, a: int, b: int, K: int = 0) -> int:
    return challenge(G.q, qbar, K, (A, B), (a, b))


def make_constant_proof(G: Group, K: int, qbar: int, A: int, B: int, R_sum: int, u: int) -> GenericProof:
    q = G.q
    a, b = G.gPowP(u), G.powP(K, u)
    c = constant_challenge(G, qbar, A, B, a, b, K)
    return GenericProof(c, _response(q, u, c, R_sum))


def verify_constant_proof(G: Group, K: int, qbar: int, A: int, B: int, limit: int, pr: GenericProof) -> bool:
    """Contest selection-limit proof over the aggregate message (A, B) = (prod alpha, prod beta).
    The message's validity is checked by the caller on its factors (verify_ballot): the order-q
    subgroup is closed under products, so (A, B) are valid residues when every selection is."""
    if not (0 <= pr.c < G.q and 0 <= pr.v < G.q):
        return False
    a, b = constant_commitments(G, K, A, B, limit, pr)
    return pr.c == constant_challenge(G, qbar, A, B, a, b, K)


# --------------------------------------------------------------------------------------
# Ballots (synthetic, seeded — restates RandomBallotProvider usage at
# RunRemoteWorkflowTest.java:133-134; votesAllowed = 1, one placeholder per contest)
# --------------------------------------------------------------------------------------

@dataclass
class Manifest:
    n_contests: int = 4
    n_selections: int = 5   # real selections per contest
    votes_allowed: int = 1  # one placeholder selection per contest

    @property
    def sel_per_contest(self) -> int:
        return self.n_selections + self.votes_allowed

    @property
    def sel_per_ballot(self) -> int:
        return self.n_contests * self.sel_per_contest


@dataclass
class EncryptedBallot:
    cts: List[Ciphertext]          # n_contests * sel_per_contest, placeholder last in each contest
    proofs: List[RangeProof]
    contest_proofs: List[GenericProof]


def ballot_plaintexts(man: Manifest, rng: random.Random) -> List[int]:
    votes = []
    for _ in range(man.n_contests):
        sel = [0] * man.sel_per_contest
        sel[rng.randrange(man.n_selections)] = 1   # one-hot over real selections
        votes.extend(sel)
    return votes


def encrypt_ballot(G: Group, K: int, qbar: int, man: Manifest, votes: List[int],
                   rng: random.Random) -> EncryptedBallot:
    q = G.q
    cts, proofs, cproofs = [], [], []
    spc = man.sel_per_contest
    for c in range(man.n_contests):
        R_sum = 0
        for s in range(spc):
            m = votes[c * spc + s]
            R = rng.randrange(1, q)
            u, cf, vf = rng.randrange(1, q), rng.randrange(q), rng.randrange(q)
            ct = encrypt(G, K, m, R)
            cts.append(ct)
            proofs.append(make_range_proof(G, K, qbar, ct, m, R, u, cf, vf))
            R_sum = (R_sum + R) % q
        A = G.prodP([ct.pad for ct in cts[c * spc:(c + 1) * spc]])
        B = G.prodP([ct.data for ct in cts[c * spc:(c + 1) * spc]])
        cproofs.append(make_constant_proof(G, K, qbar, A, B, R_sum, rng.randrange(1, q)))
    return EncryptedBallot(cts, proofs, cproofs)


def verify_ballot(G: Group, K: int, qbar: int, man: Manifest, eb: EncryptedBallot) -> bool:
    spc = man.sel_per_contest
    ok = True
    for c in range(man.n_contests):
        for s in range(spc):
            i = c * spc + s
            ok &= verify_range_proof(G, K, qbar, eb.cts[i], eb.proofs[i])
        sel = eb.cts[c * spc:(c + 1) * spc]
        A = G.prodP([ct.pad for ct in sel])
        B = G.prodP([ct.data for ct in sel])
        msg_ok = all(is_valid_residue(G, ct.pad) and is_valid_residue(G, ct.data) for ct in sel)
        ok &= msg_ok and verify_constant_proof(G, K, qbar, A, B, man.votes_allowed, eb.contest_proofs[c])
    return ok


def accumulate_tally(G: Group, man: Manifest, ballots: Sequence[EncryptedBallot],
                     cast: Optional[Sequence[bool]] = None) -> List[Ciphertext]:
    """runAccumulateBallots (RunRemoteWorkflowTest.java:151): per real selection,
    componentwise product of ciphertexts over CAST ballots (cast[i] false = spoiled, left to
    decryptBallot, RunRemoteDecryptor.java:264-269); placeholders excluded."""
    spc = man.sel_per_contest
    if cast is not None:
        ballots = [b for b, c in zip(ballots, cast) if c]
    out = []
    for c in range(man.n_contests):
        for s in range(man.n_selections):
            i = c * spc + s
            out.append(Ciphertext(G.prodP([b.cts[i].pad for b in ballots]),
                                  G.prodP([b.cts[i].data for b in ballots])))
    return out


# --------------------------------------------------------------------------------------
# Threshold decryption (DecryptingTrusteeIF — RunRemoteDecryptingTrustee.java:180-247;
# Decryption.decrypt — RunRemoteDecryptor.java:261-262)
# --------------------------------------------------------------------------------------

@dataclass
class Guardian:
    gid: str
    x: int                 # x-coordinate 1..n (RunRemoteKeyCeremony.java:268)
    coeffs: List[int]      # polynomial a_{i,j}, a_{i,0} = s_i
    commitments: List[int] # g^{a_{i,j}}

    @property
    def s(self) -> int:
        return self.coeffs[0]

    @property
    def K(self) -> int:
        return self.commitments[0]


def poly_eval(coeffs: List[int], x: int, q: int) -> int:
    acc = 0
    for a in reversed(coeffs):
        acc = (acc * x + a) % q
    return acc


def key_ceremony(G: Group, n: int, quorum: int, rng: random.Random) -> Tuple[List[Guardian], int]:
    gs = []
    for i in range(n):
        co = [rng.randrange(1, G.q) for _ in range(quorum)]
        gs.append(Guardian(f"guardian{i + 1}", i + 1, co, [G.gPowP(a) for a in co]))
    K = G.prodP([g.K for g in gs])
    return gs, K


# --------------------------------------------------------------------------------------
# Key-ceremony share backups (HashedElGamalCiphertext) — SURVEY §8a row a12: a trustee's
# compensatedDecrypt first decrypts guardian l's backup of P_l(x_i) with its own secret
# (1 variable-base powP + SHA/HMAC), RunRemoteDecryptingTrustee.java:227-232 via upstream.
# The upstream KDF / MAC layout is not in the container (unpinned); this restatement
# defines it and the GPU-backed trustee must match it:
#   c0 = g^r,  k = K_i^r = c0^{s_i}  (512 B BE),  kk = SHA256(c0 || k)
#   stream = HMAC-SHA256(kk, 0x01 || "share" || l || i),  mac_key = HMAC-SHA256(kk, 0x02 || ...)
#   c1 = P_l(x_i) (32 B BE) XOR stream,  c2 = HMAC-SHA256(mac_key, c0 || c1)
# --------------------------------------------------------------------------------------

def _backup_keys(c0: int, k: int, label: bytes) -> Tuple[bytes, bytes]:
    import hmac
    kk = hashlib.sha256(c0.to_bytes(512, "big") + k.to_bytes(512, "big")).digest()
    stream = hmac.new(kk, b"\x01share" + label, hashlib.sha256).digest()
    mac_key = hmac.new(kk, b"\x02share" + label, hashlib.sha256).digest()
    return stream, mac_key


def backup_label(from_gid: str, to_gid: str) -> bytes:
    return from_gid.encode() + b"|" + to_gid.encode()


def backup_encrypt(G: Group, K_to: int, share: int, r: int, label: bytes) -> Tuple[int, bytes, bytes]:
    import hmac
    c0 = G.gPowP(r)
    stream, mac_key = _backup_keys(c0, G.powP(K_to, r), label)
    c1 = bytes(a ^ b for a, b in zip(share.to_bytes(32, "big"), stream))
    return c0, c1, hmac.new(mac_key, c0.to_bytes(512, "big") + c1, hashlib.sha256).digest()


def backup_decrypt(G: Group, s_to: int, backup: Tuple[int, bytes, bytes], label: bytes) -> Optional[int]:
    """-> P_l(x_i), or None when the MAC does not verify."""
    import hmac
    c0, c1, c2 = backup
    stream, mac_key = _backup_keys(c0, G.powP(c0, s_to), label)
    if not hmac.compare_digest(c2, hmac.new(mac_key, c0.to_bytes(512, "big") + c1, hashlib.sha256).digest()):
        return None
    return int.from_bytes(bytes(a ^ b for a, b in zip(c1, stream)), "big")


# --------------------------------------------------------------------------------------
# Key-ceremony proofs (RunRemoteKeyCeremony.java:200-233 and
# RunRemoteTrustee.java:184 reach them through upstream KeyCeremonyTrustee):
#  * Schnorr proof of knowledge of each coefficient a_ij behind K_ij = g^{a_ij}, compact
#    (c, v) like the other proofs: h = g^u, c = H(K_ij, h), v = u - c*a_ij mod q;
#    verify: K_ij^q == 1 (valid residue), h = g^v K_ij^c, c == H(K_ij, h);
#  * a recipient checks a decrypted backup share against the sender's commitments:
#    g^{P_l(x_i)} == prod_j K_lj^{x_i^j} (= recovery_public_key).
# The upstream pre-image (domain labels) is not in the container: unpinned, and defined
# identically here and in electionguard/keyceremony.py.
# --------------------------------------------------------------------------------------

def schnorr_prove(G: Group, a: int, K: int, u: int) -> GenericProof:
    h = G.gPowP(u)
    c = hash_elems(G.q, ("P", K), ("P", h))
    return GenericProof(c, (u - c * a) % G.q)


def schnorr_verify(G: Group, K: int, pr: GenericProof) -> bool:
    if not (0 < K < G.p) or G.powP(K, G.q) != 1 or not (0 <= pr.c < G.q and 0 <= pr.v < G.q):
        return False
    h = G.multP(G.gPowP(pr.v), G.powP(K, pr.c))
    return pr.c == hash_elems(G.q, ("P", K), ("P", h))


def verify_backup_share(G: Group, share: int, sender: Guardian, x: int) -> bool:
    return G.gPowP(share) == recovery_public_key(G, sender, x)


def direct_decrypt(G: Group, qbar: int, gd: Guardian, texts: Sequence[Ciphertext],
                   nonces: Sequence[int]) -> List[Tuple[int, GenericProof]]:
    """DirectDecryptionAndProof per text: M_i = A^{s_i} + generic CP proof
    (decrypting_trustee_rpc.proto:25-28)."""
    return [(M, pr) for M, pr in share_proofs(G, qbar, gd.s, texts, nonces)]


def share_proofs(G: Group, qbar: int, secret: int, texts: Sequence[Ciphertext],
                 nonces: Sequence[int]) -> List[Tuple[int, GenericProof]]:
    """M = pad^secret and its generic CP proof per text: a = g^u, b = pad^u,
    c = H(qbar, [K_i = g^secret,] pad, data, a, b, M) (PREIMAGE order), v = u -+ c secret (RESPONSE)."""
    Ki = G.gPowP(secret) if PREIMAGE == "with_key" else 0
    out = []
    for ct, u in zip(texts, nonces):
        M = G.powP(ct.pad, secret)
        a, b = G.gPowP(u), G.powP(ct.pad, u)
        c = challenge(G.q, qbar, Ki, (ct.pad, ct.data), (a, b), (M,))
        out.append((M, GenericProof(c, _response(G.q, u, c, secret))))
    return out


def recovery_public_key(G: Group, missing: Guardian, x: int) -> int:
    """g^{P_l(x)} = prod_j K_{l,j}^{x^j}."""
    return G.prodP([G.powP(Kj, pow(x, j, G.q)) for j, Kj in enumerate(missing.commitments)])


def compensated_decrypt(G: Group, qbar: int, gd: Guardian, missing: Guardian,
                        texts: Sequence[Ciphertext], nonces: Sequence[int]) -> List[Tuple[int, GenericProof, int]]:
    """CompensatedDecryptionAndProof (decrypting_trustee_rpc.proto:41-45)."""
    share = poly_eval(missing.coeffs, gd.x, G.q)
    rk = recovery_public_key(G, missing, gd.x)
    return [(M, pr, rk) for M, pr in share_proofs(G, qbar, share, texts, nonces)]


def verify_share(G: Group, qbar: int, Ki: int, ct: Ciphertext, M: int, pr: GenericProof) -> bool:
    e = _resp_exp(G.q, pr.c)
    a = G.multP(G.gPowP(pr.v), G.powP(Ki, e))
    b = G.multP(G.powP(ct.pad, pr.v), G.powP(M, e))
    return pr.c == challenge(G.q, qbar, Ki, (ct.pad, ct.data), (a, b), (M,))


def lagrange(xs: Sequence[int], xi: int, q: int) -> int:
    num, den = 1, 1
    for xj in xs:
        if xj != xi:
            num = num * xj % q
            den = den * (xj - xi) % q
    return num * pow(den, -1, q) % q


def combine(G: Group, ct: Ciphertext, direct: Dict[str, int], comp: Dict[str, Dict[str, int]],
            avail_x: Dict[str, int], max_t: int) -> Optional[int]:
    """M = prod direct M_i * prod_l prod_i M_{l,i}^{w_i}; T = B M^-1; t = dlog_g T."""
    xs = list(avail_x.values())
    M = G.prodP(list(direct.values()))
    for _, shares in comp.items():
        for gid, Mli in shares.items():
            M = G.multP(M, G.powP(Mli, lagrange(xs, avail_x[gid], G.q)))
    T = G.multP(ct.data, G.multInv(M))
    return G.dlogG(T, max_t)


def decrypt_ballot(G: Group, qbar: int, man: Manifest, eb: EncryptedBallot, avail: Sequence[Guardian],
                   missing: Sequence[Guardian], nonces: Sequence[int]) -> Tuple[List[Optional[int]], dict]:
    """decryptBallot of one spoiled ballot (RunRemoteDecryptor.java:264-269): each real
    selection (placeholders are not part of the plaintext ballot) is decrypted like a tally
    text -- every available guardian's direct share, every (missing, available) pair's
    compensated share, Lagrange combine, dLog_g up to votesAllowed.  nonces: the proof nonces,
    one per (share kind, text) in the order direct(avail...) then compensated(missing x avail),
    each list len(texts) long.  -> (plaintexts, shares by kind)."""
    spc = man.sel_per_contest
    texts = [eb.cts[c * spc + s] for c in range(man.n_contests) for s in range(man.n_selections)]
    n = len(texts)
    it = iter(nonces)
    take = lambda: [next(it) for _ in range(n)]  # noqa: E731
    direct = {g.gid: direct_decrypt(G, qbar, g, texts, take()) for g in avail}
    comp = {l.gid: {g.gid: compensated_decrypt(G, qbar, g, l, texts, take()) for g in avail} for l in missing}
    avail_x = {g.gid: g.x for g in avail}
    out = []
    for i, ct in enumerate(texts):
        out.append(combine(G, ct, {gid: d[i][0] for gid, d in direct.items()},
                           {l: {gid: c[i][0] for gid, c in by.items()} for l, by in comp.items()},
                           avail_x, man.votes_allowed))
    return out, {"direct": direct, "compensated": comp}
