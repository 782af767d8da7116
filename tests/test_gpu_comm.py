"""libeg_hip's own device memory, verdict reduction and multi-GPU tally exchange,
on one MI355X: eg_dev_alloc / eg_memcpy_* / eg_all_nonzero_dev, the RCCL communicator at world
size 1 (eg_comm_init / eg_comm_all_valid) and eg_tally_allgather_fold bit-exact against the
oracle's fold, every collective's completion polled under the deadline (a stalled one aborted, the
failure sticky); the job-table cache's failure path and two election keys alternating
on one context."""
import random

import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


def _rand_elems(rng, n, p):
    return np.stack([np.frombuffer(rng.randrange(p).to_bytes(512, "big"), np.uint8) for _ in range(n)])


def test_device_buffer_roundtrip_views_and_flags(group):
    a = np.arange(7 * 33, dtype=np.uint32).reshape(7, 33)
    d = group.to_device(a)
    assert np.array_equal(d.download(), a)
    assert np.array_equal(d[2:5].download(), a[2:5])
    z = group.device_zeros((5, 3))
    assert not z.download().any() and not group.all_nonzero(z)
    f = np.ones(100_003, np.uint8)
    df = group.to_device(f)
    assert group.all_nonzero(df)
    for pos in (0, 63, 64, 99_999, 100_002):
        g = f.copy()
        g[pos] = 0
        df.upload(g)
        assert not group.all_nonzero(df), pos
        assert group.all_nonzero(df, pos) == bool(g[:pos].all())  # the first pos flags only
    assert group.all_nonzero(df, 0)  # no flags: vacuously all valid


@pytest.mark.parametrize("nparts", [1, 3])
def test_tally_fold_local_parts_equals_oracle(group, oracle_group, nparts):
    """eg_tally_allgather_fold without a communicator folds the local parts: out[k] = prod_j part j's
    element k mod p, bit-exact with CPython (including 0, 1 and p - 1 rows)."""
    rng = random.Random(17 + nparts)
    p = oracle_group.p
    n = 40
    parts = _rand_elems(rng, nparts * n, p).reshape(nparts, n, 512)
    parts[0, 0] = np.frombuffer((0).to_bytes(512, "big"), np.uint8)
    parts[0, 1] = np.frombuffer((1).to_bytes(512, "big"), np.uint8)
    parts[-1, 2] = np.frombuffer((p - 1).to_bytes(512, "big"), np.uint8)
    out = group.tally_allgather_fold(group.to_device(parts), nparts, n)
    for k in range(n):
        want = oracle_group.prodP([int.from_bytes(parts[j, k].tobytes(), "big") for j in range(nparts)])
        assert int.from_bytes(out[k].tobytes(), "big") == want, k


def test_rccl_world_one_exchange(group, oracle_group):
    """The RCCL communicator inside libeg_hip at world size 1: unique id, init (non-blocking, with a
    deadline), what it reports about itself (eg_comm_info), the verdict
    all-reduce (min) and the all-gather + fold of 2 partial tallies on the ctx stream, through the
    TallyExchange bench.py uses."""
    from electionguard.distributed import TallyExchange
    rng = random.Random(29)
    p = oracle_group.p
    uid = group.comm_unique_id()
    assert len(uid) == 128
    assert group.comm_info() == (0, 0)  # no communicator yet
    group.comm_init(uid, 1, 0)
    try:
        assert group.comm_info() == (1, 0)  # what RCCL reports (ncclCommCount / ncclCommUserRank)
        assert group.comm_all_valid(True) is True and group.comm_all_valid(False) is False
        n = 24
        parts = _rand_elems(rng, 2 * n, p).reshape(2, n, 512)
        out = group.tally_allgather_fold(group.to_device(parts), 2, n)
        for k in range(n):
            want = oracle_group.prodP([int.from_bytes(parts[j, k].tobytes(), "big") for j in range(2)])
            assert int.from_bytes(out[k].tobytes(), "big") == want, k
    finally:
        group.comm_destroy()
    assert group.comm_info() == (0, 0)
    x = TallyExchange(group, None, 1, 0)
    # world 1 never creates a communicator, and the bench line says so
    assert x.collective == "no communicator (world 1: local fold)" and x.rccl_ranks == 0
    one = _rand_elems(rng, 6, p).reshape(3, 2, 512)
    assert np.array_equal(x.fold(group.to_device(one), 3), one)  # world 1: the local tally itself
    assert x.all_valid(True) and not x.all_valid(False)


@pytest.mark.parametrize("where", ["all_valid", "fold"])
def test_rccl_collective_deadline_and_sticky_failure(group, oracle_group, monkeypatch, where):
    """A collective whose completion never arrives (EG_TEST_COMM_STALL=1: libeg's wait never sees the
    event, as with a peer that died after the enqueue) fails within the deadline (EG_COMM_TIMEOUT_S)
    instead of hanging in hipStreamSynchronize; the communicator is aborted and the failure is
    STICKY: every later collective AND the fold fail with EG_ERR_STATE (no silent local-parts fold
    that would be a partial tally), until eg_comm_destroy resets the context."""
    import time

    from electionguard.core.native import EgError
    rng = random.Random(41)
    p = oracle_group.p
    n = 8
    parts = _rand_elems(rng, n, p).reshape(1, n, 512)
    d = group.to_device(parts)
    monkeypatch.setenv("EG_COMM_TIMEOUT_S", "1.5")
    group.comm_init(group.comm_unique_id(), 1, 0)
    try:
        monkeypatch.setenv("EG_TEST_COMM_STALL", "1")
        t = time.monotonic()
        with pytest.raises(EgError) as e:
            if where == "all_valid":
                group.comm_all_valid(True)
            else:
                group.tally_allgather_fold(d, 1, n)
        took = time.monotonic() - t
        assert e.value.code == 2 and "not complete after" in str(e.value), str(e.value)
        assert 1.4 <= took < 10, took
        monkeypatch.delenv("EG_TEST_COMM_STALL")
        assert group.comm_info() == (0, 0)  # aborted
        for call in (lambda: group.comm_all_valid(True), lambda: group.tally_allgather_fold(d, 1, n)):
            with pytest.raises(EgError) as e:
                call()
            assert e.value.code == 5 and "aborted" in str(e.value), str(e.value)
    finally:
        monkeypatch.delenv("EG_TEST_COMM_STALL", raising=False)
        group.comm_destroy()  # resets the sticky failure
    out = group.tally_allgather_fold(d, 1, n)  # a clean context folds its local parts again
    assert np.array_equal(out, parts[0])
    group.comm_init(group.comm_unique_id(), 1, 0)  # and a new communicator works through the polled wait
    try:
        assert group.comm_all_valid(True) is True
        assert np.array_equal(group.tally_allgather_fold(d, 1, n), parts[0])
    finally:
        group.comm_destroy()


def test_job_cache_survives_a_failed_upload(oracle_group):
    """A job-table upload that fails part-way through a shape's set (EG_TEST_FAIL_JOBS=3: the third
    of the verifier's four tables, as an out-of-memory hipMalloc would) fails that call with
    EG_ERR_NOMEM and leaves no partial set: the next call on the same context rebuilds every table
    and verifies (before the fix it took the first table as a hit and read a null one)."""
    import os

    from electionguard.ballot import EncryptedBallots, Manifest, Verifier, ElectionKey
    from electionguard.core.group import GroupContext
    from electionguard.core.native import EgError
    from test_gpu_golden import _ballot_arrays
    G = oracle_group
    rng = random.Random(31)
    gs, K = O.key_ceremony(G, 2, 2, rng)
    qbar = rng.randrange(G.q)
    man_o, man = O.Manifest(2, 2, 1), Manifest(2, 2, 1)
    arrs = [_ballot_arrays(O.encrypt_ballot(G, K, qbar, man_o, O.ballot_plaintexts(man_o, rng), rng))
            for _ in range(3)]
    eb = EncryptedBallots(*(np.concatenate([a[i] for a in arrs]) for i in range(3)))
    os.environ["EG_TEST_FAIL_JOBS"] = "3"
    try:
        ctx = GroupContext(G.p, G.q, G.g, device=0)
    finally:
        del os.environ["EG_TEST_FAIL_JOBS"]
    try:
        V = Verifier(ctx, ElectionKey(ctx, K), qbar, man)
        with pytest.raises(EgError) as e:
            V.verify(eb)
        assert e.value.code == 3 and "EG_TEST_FAIL_JOBS" in str(e.value)
        for _ in range(2):  # rebuilt, then a cache hit
            ok_s, ok_c, tally = V.verify(eb)
            assert ok_s.all() and ok_c.all()
    finally:
        ctx.close()


def test_two_keys_alternating_on_one_context(group, oracle_group):
    """Two election keys of different table widths alternate on one context (each call
    used to rebuild the other key's table at the current width): every call verifies its own
    ballots and rejects the other key's."""
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
    from test_gpu_golden import _ballot_arrays
    G = oracle_group
    rng = random.Random(37)
    man_o, man = O.Manifest(1, 2, 1), Manifest(1, 2, 1)
    sets = []
    for wb in (8, 12):
        _, K = O.key_ceremony(G, 2, 2, rng)
        qbar = rng.randrange(G.q)
        eb = EncryptedBallots(*_ballot_arrays(O.encrypt_ballot(G, K, qbar, man_o, O.ballot_plaintexts(man_o, rng), rng)))
        sets.append((Verifier(group, ElectionKey(group, K, window_bits=wb), qbar, man), eb))
    for _ in range(3):
        for i, (V, eb) in enumerate(sets):
            ok_s, ok_c, _ = V.verify(eb)
            assert ok_s.all() and ok_c.all()
            other = sets[1 - i][1]
            ok_s, _, _ = V.verify(other, with_tally=False)
            assert not ok_s.all()
