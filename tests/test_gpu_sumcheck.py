"""GPU parity for the GF(2^128) sumcheck prover (Sumcheck<N, d, T>, src/ulvt/sumcheck/sumcheck.cuh)
against the oracle transcript (every round's sum and points), the reference test's protocol
checks (test.cu:41,49,77,100), and sharded provers on one GPU against the unsharded transcript."""
import numpy as np
import pytest

import _oracle as O
import binius_ntt_amd as B

pytestmark = pytest.mark.gpu


def _rand(n, seed):
    return np.random.default_rng(seed).integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)


def _case(n, d, seed):
    ev = _rand(4 * (1 << n) * d, seed)  # compact columns, column-major
    ch = _rand(4 * n, seed + 1).reshape(n, 4)
    return ev, ch


def _transcript(sc, n, ch):
    sums, pts = [], []
    for r in range(n + 1):
        s, p = sc.this_round_messages()
        sums.append(s)
        pts.append(p)
        if r < n:
            sc.move_to_next_round(ch[r])
    return np.stack(sums), np.stack(pts)


@pytest.mark.parametrize("n,d", [(1, 2), (3, 3), (5, 1), (5, 2), (6, 3), (8, 4), (10, 2), (9, 5)])
@pytest.mark.parametrize("transposed", [0, 1])
def test_sumcheck_transcript_matches_oracle(n, d, transposed, dev):
    if transposed and n < 5:
        pytest.skip("bitsliced input needs whole 32-element batches")
    ev, ch = _case(n, d, 1000 * n + 10 * d + transposed)
    inp = O.bitslice128(ev) if transposed else ev
    want_s, want_p = O.sumcheck_run(inp, n, d, transposed, ch)
    sc = B.Sumcheck(n, d, transposed, inp)
    got_s, got_p = _transcript(sc, n, ch)
    for r in range(n + 1):
        assert np.array_equal(got_s[r], want_s[r]), "round %d sum" % r
        assert np.array_equal(got_p[r], want_p[r]), "round %d points" % r
    sc.close()


@pytest.mark.parametrize("n,d", [(18, 3), (17, 6)])
def test_sumcheck_transcript_quad_path(n, d, dev):
    # the first rounds are big enough for the throughput kernels (quad products, the coalesced
    # fold, the separate post kernel); the smaller cases above run the 16-lane ones. d = 6 takes
    # the general GF(2^4) k-multiples (mul_small: points up to 6) on the quad path
    ev, ch = _case(n, d, 1818 if (n, d) == (18, 3) else 1700 + d)
    bs = O.bitslice128(ev)
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    sc = B.Sumcheck(n, d, True, bs)
    got_s, got_p = _transcript(sc, n, ch)
    for r in range(n + 1):
        assert np.array_equal(got_s[r], want_s[r]), "round %d sum" % r
        assert np.array_equal(got_p[r], want_p[r]), "round %d points" % r
    sc.close()


@pytest.mark.parametrize("n,d,full_points", [(19, 3, False), (19, 2, False), (19, 2, True)])
def test_sumcheck_transcript_fused_fold_messages(n, d, full_points, dev, monkeypatch):
    # N = 19 transcripts against the oracle, every round's sum and points. Round 1 (2^18
    # evaluations per column left, with and without the claim-derived point 1) is the first round
    # whose fold the -DBN_SC_FUSED experiment build runs inside the messages launch (sc_fold_msgs;
    # this test was green on that build too).
    if full_points:
        monkeypatch.setenv("BN_SUMCHECK_FULL_POINTS", "1")
    ev, ch = _case(n, d, 1900 + 10 * d + full_points)
    bs = O.bitslice128(ev)
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    sc = B.Sumcheck(n, d, True, bs)
    got_s, got_p = _transcript(sc, n, ch)
    sc.close()
    for r in range(n + 1):
        assert np.array_equal(got_s[r], want_s[r]), "round %d sum" % r
        assert np.array_equal(got_p[r], want_p[r]), "round %d points" % r


@pytest.mark.parametrize("full_points", [False, True])
@pytest.mark.parametrize("n,d", [(16, 3), (14, 4), (15, 2)])
def test_sumcheck_protocol_checks(n, d, full_points, dev, monkeypatch):
    # the reference test's verifier loop (test.cu:31-100) on a bitsliced input. With
    # BN_SUMCHECK_FULL_POINTS=1 every p(1) and sum comes from the data (no claim-derived point 1),
    # so p(0) + p(1) == previous p(r) checks the folds as the reference's loop does.
    if full_points:
        monkeypatch.setenv("BN_SUMCHECK_FULL_POINTS", "1")
    ev, ch = _case(n, d, 77 + n)
    bs = O.bitslice128(ev)
    sc = B.Sumcheck(n, d, True, bs)
    claim = None
    for r in range(n):
        s, p = sc.this_round_messages()
        if r > 0:
            assert np.array_equal(s, claim)
        assert np.array_equal(s, p[0] ^ p[1])
        claim = O.interpolate(p, ch[r])
        sc.move_to_next_round(ch[r])
    s, _ = sc.this_round_messages()
    assert np.array_equal(s, claim)
    assert np.array_equal(O.multilinear_composition(ev, n, d, ch), claim)
    sc.close()


@pytest.mark.parametrize("world,n,d", [(2, 8, 3), (4, 9, 2), (8, 10, 3)])
def test_sharded_provers_match_unsharded(world, n, d, dev):
    # `world` shard provers on one GPU, combined exactly as binius_ntt_amd.distributed does
    ev, ch = _case(n, d, 500 + world)
    want_s, want_p = O.sumcheck_run(ev, n, d, 0, ch)
    ps = []
    for r in range(world):
        p = B.Sumcheck(n, d, False, ev, shard=(r, world))
        ps.append(p)
    replicated = False
    for rnd in range(n + 1):
        if not replicated and ps[0].needs_gather():
            allw = np.concatenate([p.export_shard() for p in ps])
            for p in ps:
                p.import_gathered(allw, world)
            replicated = True
        msgs = [p.this_round_messages() for p in ps]
        if replicated:
            s, pts = msgs[0]
            for s2, p2 in msgs[1:]:
                assert np.array_equal(s2, s) and np.array_equal(p2, pts)
        else:
            s = np.bitwise_xor.reduce(np.stack([m[0] for m in msgs]), axis=0)
            pts = np.bitwise_xor.reduce(np.stack([m[1] for m in msgs]), axis=0)
        assert np.array_equal(s, want_s[rnd]), "round %d sum" % rnd
        assert np.array_equal(pts, want_p[rnd]), "round %d points" % rnd
        if rnd < n:
            for p in ps:
                p.move_to_next_round(ch[rnd])
    assert replicated
    for p in ps:
        p.close()


def _sharded_transcript(ps, world, n, ch):
    """Run `world` shard provers in lockstep, combined exactly as binius_ntt_amd.distributed does
    (XOR of the partial messages while sharded; the endgame gather once every shard is down to one
    batch); returns the combined transcript and whether the gather happened."""
    sums, pts, replicated = [], [], False
    for rnd in range(n + 1):
        if not replicated and ps[0].needs_gather():
            allw = np.concatenate([p.export_shard() for p in ps])
            for p in ps:
                p.import_gathered(allw, world)
            replicated = True
        msgs = [p.this_round_messages() for p in ps]
        if replicated:
            s, pt = msgs[0]
            for s2, p2 in msgs[1:]:
                assert np.array_equal(s2, s) and np.array_equal(p2, pt), "round %d: replicas differ" % rnd
        else:
            s = np.bitwise_xor.reduce(np.stack([m[0] for m in msgs]), axis=0)
            pt = np.bitwise_xor.reduce(np.stack([m[1] for m in msgs]), axis=0)
        sums.append(s)
        pts.append(pt)
        if rnd < n:
            for p in ps:
                p.move_to_next_round(ch[rnd])
    return np.stack(sums), np.stack(pts), replicated


@pytest.mark.parametrize("world,n,d,full_points", [(2, 20, 3, False), (8, 22, 3, False), (4, 20, 3, True)])
def test_sharded_provers_at_throughput_sizes(world, n, d, full_points, dev, monkeypatch):
    # shards large enough that each one runs the quad big-round kernels (and the
    # separate post kernel) before the endgame gather. The XOR-combined transcript must equal an
    # unsharded HIP run word for word, satisfy the reference verifier's per-round checks
    # (test.cu:41-63) and end on the oracle's multilinear composition (test.cu:95-100). With
    # BN_SUMCHECK_FULL_POINTS=1 every p(1) and sum comes from the data, so the sum check also tests
    # every fold (default: p(1) is derived from each shard's partial claim).
    if full_points:
        monkeypatch.setenv("BN_SUMCHECK_FULL_POINTS", "1")
    ev, ch = _case(n, d, 9000 + 10 * world + n)
    ref = B.Sumcheck(n, d, False, ev)
    want_s, want_p = _transcript(ref, n, ch)
    ref.close()
    ps = [B.Sumcheck(n, d, False, ev, shard=(r, world)) for r in range(world)]
    got_s, got_p, replicated = _sharded_transcript(ps, world, n, ch)
    for p in ps:
        p.close()
    assert replicated
    for r in range(n + 1):
        assert np.array_equal(got_s[r], want_s[r]), "round %d sum" % r
        assert np.array_equal(got_p[r], want_p[r]), "round %d points" % r
    for r in range(n):
        assert np.array_equal(got_s[r], got_p[r][0] ^ got_p[r][1]), "round %d: sum != p(0) + p(1)" % r
        assert np.array_equal(O.interpolate(got_p[r], ch[r]), got_s[r + 1]), "round %d: p(r) != next sum" % r
    assert np.array_equal(got_s[n], O.multilinear_composition_fold(ev, n, d, False, ch))


@pytest.mark.parametrize("n,d,transposed", [(12, 3, 0), (18, 2, 0), (13, 4, 1)])
def test_staged_create_then_prepare_matches_create(n, d, transposed, dev):
    # bn_sumcheck_create_staged + bn_sumcheck_prepare (the reference constructor's Memcpy and
    # Transpose phases, timed separately by tools/cpp/benchmark_sumcheck.cpp) = bn_sumcheck_create;
    # a staged prover used without prepare() transposes on its first round
    ev, ch = _case(n, d, 777 + n)
    inp = O.bitslice128(ev) if transposed else ev
    ref = B.Sumcheck(n, d, transposed, inp)
    want_s, want_p = _transcript(ref, n, ch)
    ref.close()
    for explicit in (True, False):
        sc = B.Sumcheck(n, d, transposed, inp, staged=True)
        if explicit:
            sc.prepare()
            sc.prepare()  # idempotent
        got_s, got_p = _transcript(sc, n, ch)
        sc.close()
        assert np.array_equal(got_s, want_s) and np.array_equal(got_p, want_p), "explicit prepare: %s" % explicit


def test_sumcheck_from_device_buffer(dev):
    import torch
    n, d = 11, 3
    ev, ch = _case(n, d, 4242)
    bs = O.bitslice128(ev)
    t = torch.from_numpy(bs.view(np.int32)).to(dev)
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    sc = B.Sumcheck(n, d, True, t)
    got_s, got_p = _transcript(sc, n, ch)
    assert np.array_equal(got_s, want_s) and np.array_equal(got_p, want_p)
    # the prover copied the buffer: the caller's tensor is untouched
    assert np.array_equal(t.cpu().numpy().view(np.uint32), bs)
    sc.close()


def test_sumcheck_errors(dev):
    n, d = 6, 2
    ev, ch = _case(n, d, 9)
    sc = B.Sumcheck(n, d, False, ev)
    for r in range(n):
        sc.this_round_messages()
        sc.move_to_next_round(ch[r])
    with pytest.raises(B.BnError):
        sc.move_to_next_round(ch[0])  # no variables left
    with pytest.raises(B.BnError):
        B._check(B.lib().bn_sumcheck_set_shard(sc._sc, 0, 2))  # too late to shard
    sc.close()
    with pytest.raises(B.BnError):
        B.Sumcheck(4, 2, True, _rand(4 * 16 * 2, 1))  # bitsliced input below one batch
    with pytest.raises(B.BnError):
        B.Sumcheck(6, 9, False, _rand(4 * 64 * 9, 1))  # composition size above 8


@pytest.mark.parametrize("n,d,transposed", [(1, 1, 0), (4, 3, 0), (5, 2, 1), (9, 3, 0), (12, 4, 1), (13, 1, 1)])
def test_multilinear_composition_eval_matches_oracle(n, d, transposed, dev):
    # evaluate_multilinear_composition (verifier.cu:88-107) on the GPU vs the oracle
    ev, ch = _case(n, d, 900 + 10 * n + d)
    inp = O.bitslice128(ev) if transposed else ev
    want = O.multilinear_composition(ev, n, d, ch)
    assert np.array_equal(B.evaluate_multilinear_composition(inp, n, d, transposed, ch), want)
    import torch
    t = torch.from_numpy(inp.view(np.int32)).to(dev)
    assert np.array_equal(B.evaluate_multilinear_composition(t, n, d, transposed, ch), want)
    assert np.array_equal(t.cpu().numpy().view(np.uint32), inp)  # device input untouched


def test_full_protocol_with_gpu_verifier(dev):
    # test.cu:13-101 with every verifier step on this library: interpolation on the host,
    # the final brute-force claim on the GPU
    n, d = 18, 3
    ev, ch = _case(n, d, 31337)
    bs = O.bitslice128(ev)
    sc = B.Sumcheck(n, d, True, bs)
    claim = None
    for r in range(n):
        s, p = sc.this_round_messages()
        if r > 0:
            assert np.array_equal(s, claim)
        assert np.array_equal(s, p[0] ^ p[1])
        claim = B.evaluate_univariate_given_points(ch[r], p)
        sc.move_to_next_round(ch[r])
    s, _ = sc.this_round_messages()
    assert np.array_equal(s, claim)
    assert np.array_equal(B.evaluate_multilinear_composition(bs, n, d, True, ch), claim)
    sc.close()


@pytest.mark.parametrize("n,d", [(9, 3), (7, 2), (8, 4)])
def test_point1_from_claim_irregular_call_patterns(n, d, dev):
    """Rounds after a messages call skip point 1 (p(1) = claim + p(0), sumcheck.hip round claims).
    A round whose messages were never asked for, and a second messages call in one round, must
    fall back to computing every point: the transcript of the rounds that are asked still matches
    the oracle's word for word."""
    ev, ch = _case(n, d, 4242 + n + d)
    bs = O.bitslice128(ev)
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    sc = B.Sumcheck(n, d, True, bs)
    for r in range(n + 1):
        if r % 3 != 1:  # rounds 1, 4, 7, ... are folded without their messages
            s, p = sc.this_round_messages()
            assert np.array_equal(s, want_s[r]), "round %d sum" % r
            assert np.array_equal(p, want_p[r]), "round %d points" % r
            if r % 3 == 2:  # and some rounds are asked twice
                s2, p2 = sc.this_round_messages()
                assert np.array_equal(s2, want_s[r]) and np.array_equal(p2, want_p[r]), "round %d repeat" % r
        if r < n:
            sc.move_to_next_round(ch[r])
    sc.close()


def test_prover_from_asynchronous_ntt_output(dev):
    # the prover is built from a device tensor an NTT is still writing on torch's
    # current stream (no synchronisation by the caller). The columns are the two transforms of a
    # batched 2^18-point GF(2^128) NTT (compact, column-major, as DATA_IS_TRANSPOSED = false
    # wants); the transcript must equal the one of a prover built from the host copy afterwards.
    import torch
    n, d = 18, 2
    x = torch.from_numpy(_rand(4 * (1 << n) * d, 4242).view(np.int32)).to(dev)
    torch.cuda.synchronize()
    cols = torch.empty_like(x)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(n, 0, B.FanPaarTowerField(7), device=dev.index or 0))
    for _ in range(4):  # queue several transforms so the last one is surely still running
        ntt.forward_device(x, cols, batch=d)
    sc = B.Sumcheck(n, d, False, cols)
    ch = _rand(4 * n, 4243).reshape(n, 4)
    got_s, got_p = _transcript(sc, n, ch)
    sc.close()
    host = cols.cpu().numpy().view(np.uint32).copy()
    ref = B.Sumcheck(n, d, False, host)
    want_s, want_p = _transcript(ref, n, ch)
    ref.close()
    assert np.array_equal(got_s, want_s)
    assert np.array_equal(got_p, want_p)
    exp = O.antt128(_rand(4 * (1 << n) * d, 4242).reshape(d, 1 << n, 4)[1], n, 0)
    assert np.array_equal(host.reshape(d, 1 << n, 4)[1], exp)


@pytest.mark.parametrize("n,d,pattern", [(12, 3, "busy"), (11, 2, "slow"), (13, 4, "busy+slow")])
def test_round_server_with_other_work_and_slow_host(n, d, pattern, dev):
    """The last rounds (<= 512 evaluations per column) run on the resident round server
    (sumcheck.hip sc_server). Unrelated kernels queued on the prover's own stream while the server
    waits for a challenge ("busy", the host then waits for them), and a host slower than the server's
    bounded wait ("slow": the server ends and is relaunched for the next challenge) must neither
    deadlock nor change the transcript, which is checked word for word against the oracle."""
    import time

    import torch
    ev, ch = _case(n, d, 6060 + n + d)
    bs = O.bitslice128(ev)
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    sc = B.Sumcheck(n, d, True, bs)
    ps = torch.cuda.ExternalStream(sc.stream_handle(), device=dev)
    junk = torch.ones(1 << 20, device=dev)
    for r in range(n + 1):
        s, p = sc.this_round_messages()
        assert np.array_equal(s, want_s[r]), "round %d sum" % r
        assert np.array_equal(p, want_p[r]), "round %d points" % r
        if "busy" in pattern:
            with torch.cuda.stream(ps):
                junk.mul_(1.5).add_(-0.5)
            ps.synchronize()
        if "slow" in pattern and r % 2:
            time.sleep(0.002)  # 2 ms: ten times the server's wait
        if r < n:
            sc.move_to_next_round(ch[r])
    sc.close()


def test_round_server_challenge_at_the_timeout(dev):
    """The host posts each challenge about when the round server's bounded wait (200 us) ends, so
    some posts land just before and some just after it times out, and some while its exit races the
    host's poll (wait_posted must relaunch such a server, not report an unposted round).
    Busy-waits swept over 120-320 us around the timeout; every transcript word against the oracle."""
    import time

    n, d = 12, 3
    ev, ch = _case(n, d, 8181)
    bs = O.bitslice128(ev)
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    delays = [120e-6 + 10e-6 * k for k in range(21)]
    for rep in range(4):
        sc = B.Sumcheck(n, d, True, bs)
        for r in range(n + 1):
            s, p = sc.this_round_messages()
            assert np.array_equal(s, want_s[r]), "rep %d round %d sum" % (rep, r)
            assert np.array_equal(p, want_p[r]), "rep %d round %d points" % (rep, r)
            if r < n:
                t_end = time.perf_counter() + delays[(rep * 7 + r) % len(delays)]
                while time.perf_counter() < t_end:
                    pass
                sc.move_to_next_round(ch[r])
        sc.close()


def test_round_server_abandoned_prover(dev):
    """A prover destroyed while its round server waits for the next challenge releases it: the
    stream drains and a new prover on the same device runs a correct transcript afterwards."""
    import torch
    n, d = 10, 3
    ev, ch = _case(n, d, 7070)
    bs = O.bitslice128(ev)
    sc = B.Sumcheck(n, d, True, bs)
    for r in range(n - 2):  # deep enough that the server is running
        sc.this_round_messages()
        sc.move_to_next_round(ch[r])
    sc.close()
    torch.cuda.synchronize()
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    sc = B.Sumcheck(n, d, True, bs)
    got_s, got_p = _transcript(sc, n, ch)
    sc.close()
    assert np.array_equal(got_s, want_s) and np.array_equal(got_p, want_p)


@pytest.mark.parametrize("n,d,pattern", [(15, 3, "plain"), (14, 2, "slow"), (15, 4, "busy"), (14, 3, "skip"),
                                         (14, 3, "reread"), (16, 3, "slow+skip")])
def test_big_rounds_host_patterns(n, d, pattern, dev):
    """The launched (big) rounds under the host behaviours a caller may show: a host slower than the
    GPU between reading a round and sending its challenge ("slow"), unrelated kernels queued on the
    prover's stream between rounds ("busy"), rounds whose messages are never read ("skip": the next
    round then computes p(1) from the data) and rounds read twice ("reread"). The transcript must be
    the oracle's word for word. (Round 5 ran these against pre-enqueued folds that wait on the GPU
    for their challenge; that design was measured slower and removed)"""
    import time

    import torch
    ev, ch = _case(n, d, 8080 + n + d)
    bs = O.bitslice128(ev)
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    sc = B.Sumcheck(n, d, True, bs)
    ps = torch.cuda.ExternalStream(sc.stream_handle(), device=dev)
    junk = torch.ones(1 << 20, device=dev)
    for r in range(n + 1):
        if not ("skip" in pattern and r % 3 == 1 and r < n):
            s, p = sc.this_round_messages()
            assert np.array_equal(s, want_s[r]), "round %d sum" % r
            assert np.array_equal(p, want_p[r]), "round %d points" % r
            if pattern == "reread":
                s2, p2 = sc.this_round_messages()
                assert np.array_equal(s2, s) and np.array_equal(p2, p), "round %d re-read" % r
        if pattern == "busy":
            with torch.cuda.stream(ps):
                junk.mul_(1.5).add_(-0.5)
            ps.synchronize()
        if "slow" in pattern and r % 2 == 0:
            time.sleep(0.002)  # 2 ms: longer than the GPU work of any of these rounds
        if r < n:
            sc.move_to_next_round(ch[r])
    sc.close()


def test_big_round_abandoned_prover(dev):
    """A prover destroyed in the middle of its big rounds (messages read, no challenge sent) drains
    its stream at once, and the next prover's transcript is the oracle's."""
    import time

    import torch
    n, d = 16, 3
    ev, ch = _case(n, d, 9090)
    bs = O.bitslice128(ev)
    sc = B.Sumcheck(n, d, True, bs)
    for r in range(3):
        sc.this_round_messages()
        sc.move_to_next_round(ch[r])
    sc.this_round_messages()  # round 3 read, its challenge never sent
    t0 = time.perf_counter()
    sc.close()
    torch.cuda.synchronize()
    assert time.perf_counter() - t0 < 5.0
    want_s, want_p = O.sumcheck_run(bs, n, d, 1, ch)
    sc = B.Sumcheck(n, d, True, bs)
    got_s, got_p = _transcript(sc, n, ch)
    sc.close()
    assert np.array_equal(got_s, want_s) and np.array_equal(got_p, want_p)


@pytest.mark.parametrize("n,d", [(4, 2), (5, 3), (6, 2), (10, 4), (16, 3)])
def test_device_compact_input_matches_host_input(n, d, dev):
    """A prover built from compact device columns transposes them straight into its storage
    (bn_sumcheck_create_device: one bitslice pass from the caller's buffer; below one whole block,
    n < 5, a padded copy and an in-place transpose); its transcript equals the host-built prover's,
    and the caller's buffer is left untouched."""
    import torch
    host = _rand(4 * (1 << n) * d, 5150 + n)
    ev = torch.from_numpy(host.view(np.int32)).to(dev)
    ch = _rand(4 * n, 5151 + n).reshape(n, 4)
    sc = B.Sumcheck(n, d, False, ev)
    got_s, got_p = _transcript(sc, n, ch)
    sc.close()
    ref = B.Sumcheck(n, d, False, host)
    want_s, want_p = _transcript(ref, n, ch)
    ref.close()
    assert np.array_equal(got_s, want_s) and np.array_equal(got_p, want_p)
    torch.cuda.synchronize()
    assert np.array_equal(ev.cpu().numpy().view(np.uint32), host)
