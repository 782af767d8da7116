"""GPU: per-element calls coalesced behind the C ABI (eg_powp_one / eg_multp_one / eg_gpowp_one and
eg_powp_submit + eg_ticket_wait).  The reference drives the group one element per call from 11
threads (RunRemoteWorkflowTest.java:140,180) on the context KUtils.productionGroup() makes
(KUtils.java:10-12); concurrent calls must join GPU batches and stay bit-exact.

* the C++ driver (tests/cpp/coalesce_bench.cpp, built in-tree by __graft_entry__.build()) runs 11
  threads of per-element calls on vectors whose expected results come from CPython pow (the
  oracle) and reports their rates beside one eg_powp_batch call;
* 11 Python threads through ElementModP.powP / times and GroupContext.gPowP (the ctypes mirror),
  checked against CPython pow."""
import json
import random
import struct
import subprocess
import threading
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "electionguard-remote_amd" / "host" / "_build" / "coalesce_bench"


def test_cpp_eleven_threads_per_element_bitexact(group, tmp_path):
    import eg_oracle as O
    og = O.production_group()
    rng = random.Random(17)
    n = 1500
    recs = []
    for i in range(n):
        b = rng.randrange(og.p) if i % 7 else rng.choice([0, 1, og.p - 1, og.p, 2**4096 - 1])
        e = rng.randrange(og.q) if i % 11 else rng.choice([0, 1, og.q - 1, 2**256 - 1])
        b2 = rng.randrange(2**4096)
        recs.append(b.to_bytes(512, "big") + e.to_bytes(32, "big") + pow(b, e, og.p).to_bytes(512, "big") +
                    b2.to_bytes(512, "big") + (b * b2 % og.p).to_bytes(512, "big") +
                    pow(og.g, e, og.p).to_bytes(512, "big"))
    vec = tmp_path / "vectors.bin"
    vec.write_bytes(struct.pack("<I", n) + b"".join(recs))
    assert BIN.exists(), "run __graft_entry__.build() first"
    r = subprocess.run([str(BIN), str(vec), "11"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["mismatches"] == 0 and res["threads"] == 11
    # (rates are recorded by tools/coalesce_shapes.py under profiles/; this suite gates on bit-exactness)


def test_latency_shape_for_blocking_callers(group, tmp_path):
    """The coalescer's small powP batches run on the latency-shaped layouts (eg_pow16.hip): one element
    per wave up to one per SIMD, 16-lane groups up to one resident round (EG_LATENCY_POW=16 skips the
    per-wave one, =0 keeps every batch on the 8-lane layout; EG_POWWAVE_D2=0 runs the per-wave kernel's
    per-step-quotient multiply instead of the delayed-quotient one).  Every layout is bit-exact on the edge
    cases (bases 0, 1, p-1, p, p+1, 2^4096-1; exponents 0, 1, 2, q-1, q, 2^256-1), from 1 and from 11
    blocking threads."""
    import os
    import eg_oracle as O
    og = O.production_group()
    rng = random.Random(41)
    n = 660
    recs = []
    for i in range(n):
        b = rng.randrange(og.p) if i % 5 else rng.choice([0, 1, og.p - 1, og.p, og.p + 1, 2**4096 - 1])
        e = rng.randrange(og.q) if i % 9 else rng.choice([0, 1, 2, og.q - 1, og.q, 2**256 - 1])
        recs.append(b.to_bytes(512, "big") + e.to_bytes(32, "big") + pow(b, e, og.p).to_bytes(512, "big") +
                    bytes(512) + bytes(512) + pow(og.g, e, og.p).to_bytes(512, "big"))
    vec = tmp_path / "vectors.bin"
    vec.write_bytes(struct.pack("<I", n) + b"".join(recs))
    res = {}
    for shape, env in (("per-wave", {}), ("per-wave-cios", {"EG_POWWAVE_D2": "0"}), ("16-lane", {"EG_LATENCY_POW": "16"}),
                       ("8-lane", {"EG_LATENCY_POW": "0"})):
        for threads in (11, 1):
            r = subprocess.run([str(BIN), str(vec), str(threads)], capture_output=True, text=True, timeout=600,
                               env=dict(os.environ, **env))
            assert r.returncode == 0, (shape, threads, r.stdout + r.stderr)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            res[(shape, threads)] = d
    print({k: (v["powp_one_blocking_per_s"], v["mismatches"]) for k, v in res.items()})
    for (shape, threads), d in res.items():
        assert d["mismatches"] == 0, (shape, threads, d)  # (the multP vectors are a x 0 = 0)
    # The rates of the layouts (per-wave against 16- and 8-lane, the delayed-quotient multiply against the
    # per-step one) are measurements, recorded by tools/coalesce_shapes.py under profiles/, not gates: a
    # fresh lease's clock and neighbours move them.


def test_python_threads_per_element_bitexact(group):
    from electionguard.core.group import ElementModP, ElementModQ
    rng = random.Random(23)
    p, q, g = group.p, group.q, group.g
    work = [(rng.randrange(p), rng.randrange(q), rng.randrange(p)) for _ in range(11 * 12)]
    bad = []

    def run(k):
        for i in range(k, len(work), 11):
            b, e, c = work[i]
            x = ElementModP(b, group)
            if x.powP(ElementModQ(e, group)).value != pow(b, e, p):
                bad.append(("powP", i))
            if x.times(ElementModP(c, group)).value != b * c % p:
                bad.append(("times", i))
            if group.gPowP(e).value != pow(g, e, p):
                bad.append(("gPowP", i))

    ths = [threading.Thread(target=run, args=(k,)) for k in range(11)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not bad, bad[:5]


def test_coalescing_window_and_errors(group):
    from electionguard.core import native
    group.set_coalescing(4, 50)
    out = group.powP_one(3, 5)
    assert int.from_bytes(out, "big") == 243
    group.set_coalescing(16384, 0)  # the adaptive default
    with pytest.raises(native.EgError):
        group.set_coalescing(0, 100)


def test_constant_time_mode_recorded_per_job(group, oracle_group):
    """eg_ctx_set_ct_pow is read when a job is SUBMITTED: jobs queued with the switch on stay in a
    constant-time batch even when the switch goes off before their batch runs, and the jobs submitted
    after it form a separate batch (a batch never mixes modes).  A fixed 30 ms window
    keeps the first jobs queued while the switch changes; every result equals CPython's."""
    import random
    og = oracle_group
    rng = random.Random(5150)
    subs = []
    group.set_coalescing(16384, 30000)  # the next batch waits for 16384 jobs or the fixed 30 ms window
    try:
        group.ct_pow = True
        for i in range(6):  # secret-exponent jobs: g^x and b^x
            x = rng.randrange(og.q)
            b = rng.randrange(og.p)
            subs.append((group.mexp_submit([], None, [(None, x)]), pow(og.g, x, og.p)))
            subs.append((group.mexp_submit([b], x), pow(b, x, og.p)))
        group.ct_pow = False  # returns at once: no batch is running, the queued ones keep their mode
        for i in range(6):
            x = rng.randrange(og.q)
            subs.append((group.mexp_submit([], None, [(None, x)]), pow(og.g, x, og.p)))
        group.ct_pow = True
        subs.append((group.mexp_submit([7], 11), pow(7, 11, og.p)))
        got = [int.from_bytes(t.wait(), "big") for t, _ in subs]
    finally:
        group.ct_pow = False
        group.set_coalescing(16384, 0)
    assert got == [w for _, w in subs]


def test_ticket_outlives_context(group):
    """A ticket submitted before eg_ctx_destroy stays waitable after it: destroy drains the open
    batches, and the ticket keeps the dispatcher's state alive."""
    import ctypes
    from electionguard.core import native
    lib = native.load()
    h = ctypes.c_void_p()
    native.check(lib, "eg_ctx_create", lib.eg_ctx_create(native.buf(group._p_be), native.buf(group._q_be),
                                                         native.buf(group._g_be), group.device, ctypes.byref(h)))
    native.check(lib, "eg_ctx_set_coalescing", lib.eg_ctx_set_coalescing(h, 16384, 200000))  # 0.2 s window
    base, e = 0x1234567, 0xABCDEF
    out = bytearray(512)
    t = ctypes.c_void_p()
    native.check(lib, "eg_powp_submit", lib.eg_powp_submit(h, native.buf(base.to_bytes(512, "big")),
                                                           native.buf(e.to_bytes(32, "big")), native.buf(out),
                                                           ctypes.byref(t)))
    native.check(lib, "eg_ctx_destroy", lib.eg_ctx_destroy(h))  # drains the batch before returning
    native.check(lib, "eg_ticket_wait", lib.eg_ticket_wait(t))
    assert int.from_bytes(out, "big") == pow(base, e, group.p)
