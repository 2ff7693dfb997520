#!/usr/bin/env python3
"""Secondary benchmark lines for BASELINE.json configs 2-5 (bench.py keeps the headline NTT).

  python tools/bench_configs.py [--only c2,c3,c4,c5,bb,qm] [--sc-vars 24] [--out FILE]

c2  GF(2^128) multiply microbench, register-resident repeat loops (bitsliced_repeat style):
    compact (one element per lane) and bitsliced (32 products per lane-block), products/s.
c3  2^20-point GF(2^128) additive NTT, device-resident, elements/s.
c4  Sumcheck over GF(2^128), 2^N evals, bitsliced input (DATA_IS_TRANSPOSED = true),
    d in {2,3,4}: all N rounds (messages + fold) plus the final messages, device-resident
    columns; evals/s = 2^N / t.  Synthetic evals (numpy PCG64, fixed seed) and challenges.
c5  one GPU's share of the 256 x 2^20 batched NTT (32 transforms), elements/s; and one GPU's
    shard (rank 0 of 8) of the 2^28-eval d=3 sumcheck: the sharded rounds up to the endgame
    gather (the per-round all-gather of (d+2)x16 B partials is not included).
bb  BabyBear radix-2 NTT (prime-field sibling): 2^24 single transform and
    16 x 2^20 batched, device-resident, elements/s and algorithmic GB/s (4 B read + 4 B written
    per element).
qm  QM31 sumcheck (prime-field sibling), two columns of 2^N QM31, product
    composition: all N rounds (round messages + fold, one host round trip per round as in
    sumcheck.cuh:46-96) on device-resident columns; evals/s = 2^N / t (wall clock, setup upload
    excluded as the reference's benchmarking timer does).
Every line is one JSON object.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "binius-ntt_amd", "python"))

import numpy as np  # noqa: E402


def ev_time(fn, reps, stream):
    import torch
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    a.record(stream)
    for _ in range(reps):
        fn()
    b.record(stream)
    b.synchronize()
    return a.elapsed_time(b) / reps


def c2(dev, out):
    import torch
    import binius_ntt_amd as B
    st = torch.cuda.current_stream(dev)
    g = np.random.default_rng(2)
    # kind 2 is the product behind the boundary's multiply_unrolled<7> (bn_multiply_unrolled_device(7),
    # bn_gf128_mul_bitsliced_device); kind 1 keeps the reference's structure (one 32-product block
    # per lane, binary_tower_unrolled7.cu) for comparison only
    for kind, name, words, per in ((0, "compact", 4, 1),
                                   (2, "bitsliced multiply_unrolled<7>, quad-lane product (the boundary's path)", 128, 32),
                                   (1, "bitsliced, one 9712-gate multiply_unrolled<7> circuit per lane (reference "
                                       "structure, not the boundary's path)", 128, 32)):
        threads = 256 * 2048 if kind == 0 else 256 * 1024
        iters = 2000 if kind == 0 else 20 if kind == 1 else 200
        state = torch.from_numpy(g.integers(0, 2**32, size=threads * words, dtype=np.uint64).astype(np.uint32)
                                 .view(np.int32)).to(dev)
        opnd = torch.from_numpy(g.integers(0, 2**32, size=threads * words, dtype=np.uint64).astype(np.uint32)
                                .view(np.int32)).to(dev)  # one multiplier per lane, same shape as state
        ms = ev_time(lambda: B.gf128_mul_repeat(kind, state, opnd, threads, iters, stream=st), 3, st)
        prods = threads * iters * per
        out({"config": "c2", "workload": "GF(2^128) multiply repeat loop, %s" % name, "value": prods / (ms * 1e-3),
             "unit": "products/s", "ms": ms, "threads": threads, "iters": iters,
             "kernel": ("bn::k_repeat_compact", "bn::k_repeat_bitsliced", "bn::k_repeat_quad")[kind]})
    # the boundary entry itself on HBM-resident operands: dst = a * b over 2^20 blocks (32 Mi products;
    # 48 B of HBM traffic per product: two operands read, one product written)
    nblk = 1 << 20
    a = torch.from_numpy(g.integers(0, 2**32, size=128 * nblk, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    b = torch.from_numpy(g.integers(0, 2**32, size=128 * nblk, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    o = torch.empty_like(a)
    ms = ev_time(lambda: B.multiply_unrolled_device(7, a, b, o, stream=st), 5, st)
    prods = 32 * nblk
    out({"config": "c2", "workload": "GF(2^128) bitsliced products through bn_multiply_unrolled_device(7), 2^20 "
                                     "HBM-resident 128-word blocks", "value": prods / (ms * 1e-3), "unit": "products/s",
         "ms": ms, "hbm_gbps_algorithmic": 3 * 512.0 * nblk / (ms * 1e-3) / 1e9, "kernel": "bn::k_gf128_mul_bs"})
    del a, b, o
    # the compact entry on HBM-resident operands: dst = a * b over 2^25 compact elements
    # (tower_height_7_mul semantics; 48 B of HBM traffic per product)
    n = 1 << 25
    a = torch.randint(-2**31, 2**31, (4 * n,), dtype=torch.int32, device=dev)
    b = torch.randint(-2**31, 2**31, (4 * n,), dtype=torch.int32, device=dev)
    o = torch.empty_like(a)
    ms = ev_time(lambda: B.gf128_mul(a, b, o, stream=st), 5, st)
    out({"config": "c2", "workload": "GF(2^128) compact products through bn_gf128_mul_device, 2^25 HBM-resident "
                                     "elements", "value": n / (ms * 1e-3), "unit": "products/s", "ms": ms,
         "hbm_gbps_algorithmic": 48.0 * n / (ms * 1e-3) / 1e9, "kernel": "bn::k_gf128_mul"})
    del a, b, o


def ntt_line(dev, out, cfg, log_h, batch):
    import torch
    import binius_ntt_amd as B
    n = 1 << log_h
    g = np.random.default_rng(3)
    x = torch.from_numpy(g.integers(0, 2**32, size=4 * n * batch, dtype=np.uint64).astype(np.uint32)
                         .view(np.int32)).to(dev)
    y = torch.empty_like(x)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7), device=dev.index or 0))
    st = torch.cuda.current_stream(dev)
    ms = ev_time(lambda: ntt.forward_device(x, y, batch=batch, stream=st), 10, st)
    elems = n * batch
    out({"config": cfg, "workload": "%d x 2^%d-point GF(2^128) additive NTT (r=0)" % (batch, log_h),
         "value": elems / (ms * 1e-3), "unit": "elements/s", "ms": ms,
         "hbm_gbps_algorithmic": 32.0 * elems / (ms * 1e-3) / 1e9})


def c4(dev, out, nvars, ds):
    import torch
    import binius_ntt_amd as B
    for d in ds:
        g = np.random.default_rng(0x5C00 + d)
        words = 4 * (1 << nvars) * d
        ev = torch.from_numpy(g.integers(0, 2**32, size=words, dtype=np.uint64).astype(np.uint32)
                              .view(np.int32)).to(dev)
        ch = g.integers(0, 2**32, size=(nvars, 4), dtype=np.uint64).astype(np.uint32)
        torch.cuda.synchronize()
        runs = []
        for _ in range(3):  # median of 3 whole protocol runs (the first also warms the kernels)
            sc = B.Sumcheck(nvars, d, True, ev)  # copies the columns (device to device)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for r in range(nvars):
                sc.this_round_messages()
                sc.move_to_next_round(ch[r])
            sc.this_round_messages()
            runs.append(time.perf_counter() - t0)
            sc.close()
        dt = sorted(runs)[1]
        del ev
        torch.cuda.empty_cache()
        out({"config": "c4", "workload": "sumcheck GF(2^128), 2^%d evals, d=%d, bitsliced input" % (nvars, d),
             "value": (1 << nvars) / dt, "unit": "evals/s", "ms": dt * 1e3,
             "hbm_gbps_algorithmic": 3.0 * d * 16 * (1 << nvars) / dt / 1e9})


def c4_phases(dev, out, nvars, d, runs=3):
    """The reference's sumcheck benchmark shape (src/ulvt/sumcheck/bench/benchmark.cu:12-46, main at
    :71-85 runs N in {20, 24, 28} x d in {2, 3, 4}): DATA_IS_TRANSPOSED = false, timed as memcpy
    (compact host evals -> HBM; the reference copies from a pageable std::vector, reported as
    memcpy_ms, with the pinned-staging copy beside it), transpose (prover construction from the
    compact device columns: copy + bitslice transpose on the device) and raw (all rounds + the final
    messages); medians of `runs` after one warm-up. Inputs above 1 GiB repeat a random 64 MiB pattern
    (the reference feeds zeros; the kernels have no data-dependent control flow)."""
    import torch
    import binius_ntt_amd as B
    g = np.random.default_rng(0x5CF0 + d)
    words = 4 * (1 << nvars) * d
    if words <= (1 << 28):
        host = g.integers(0, 2**32, size=words, dtype=np.uint64).astype(np.uint32).view(np.int32)
    else:
        pat = g.integers(0, 2**32, size=1 << 24, dtype=np.uint64).astype(np.uint32).view(np.int32)
        host = np.tile(pat, words // pat.size)
    pinned = torch.from_numpy(host).pin_memory()
    ch = g.integers(0, 2**32, size=(nvars, 4), dtype=np.uint64).astype(np.uint32)
    res = []
    for it in range(runs + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev = torch.from_numpy(host).to(dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        sc = B.Sumcheck(nvars, d, False, ev)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for r in range(nvars):
            sc.this_round_messages()
            sc.move_to_next_round(ch[r])
        sc.this_round_messages()
        t3 = time.perf_counter()
        sc.close()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        ev.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        del ev
        if it:
            res.append((t1 - t0, t2 - t1, t3 - t2, t5 - t4))
    del pinned
    torch.cuda.empty_cache()
    med = [sorted(x)[len(x) // 2] * 1e3 for x in zip(*res)]
    out({"config": "c4", "workload": "sumcheck GF(2^128), 2^%d evals, d=%d, compact input "
                                     "(DATA_IS_TRANSPOSED=false): memcpy / transpose / raw" % (nvars, d),
         "memcpy_ms": med[0], "memcpy_pinned_ms": med[3], "transpose_ms": med[1], "raw_ms": med[2],
         "total_ms": med[0] + med[1] + med[2],
         "value": (1 << nvars) / (med[2] * 1e-3), "unit": "evals/s (raw)", "runs": runs,
         "memcpy_note": "memcpy_ms: pageable numpy -> HBM (the reference's std::vector source); "
                        "memcpy_pinned_ms: the same bytes from a pinned staging tensor"})


def c5_sumcheck_single(dev, out, nvars=28, d=3):
    """The whole 2^28-eval d=3 sumcheck on ONE GPU (12.9 GB of columns, fits in 288 GB)."""
    import torch
    import binius_ntt_amd as B
    g = torch.Generator(device=dev)
    g.manual_seed(0x5C00 + d)
    ev = torch.randint(-2**31, 2**31 - 1, (4 * (1 << nvars) * d,), dtype=torch.int32, device=dev, generator=g)
    ch = np.random.default_rng(1).integers(0, 2**32, size=(nvars, 4), dtype=np.uint64).astype(np.uint32)
    sc = B.Sumcheck(nvars, d, True, ev)
    del ev
    torch.cuda.empty_cache()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for r in range(nvars):
        sc.this_round_messages()
        sc.move_to_next_round(ch[r])
    sc.this_round_messages()
    dt = time.perf_counter() - t0
    sc.close()
    out({"config": "c5 (1 GPU, whole problem)", "workload": "sumcheck GF(2^128), 2^%d evals, d=%d, bitsliced input"
         % (nvars, d), "value": (1 << nvars) / dt, "unit": "evals/s", "ms": dt * 1e3})


def c5_sumcheck_shard(dev, out, nvars=28, d=3, world=8):
    import torch
    import binius_ntt_amd as B
    g = torch.Generator(device=dev)
    g.manual_seed(0x5C00 + d)
    ev = torch.randint(-2**31, 2**31 - 1, (4 * (1 << nvars) * d,), dtype=torch.int32, device=dev, generator=g)
    sc = B.Sumcheck(nvars, d, True, ev, shard=(0, world))  # keeps batches b % 8 == 0
    del ev
    torch.cuda.empty_cache()
    ch = np.random.default_rng(1).integers(0, 2**32, size=(nvars, 4), dtype=np.uint64).astype(np.uint32)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = 0
    while not sc.needs_gather():
        sc.this_round_messages()
        sc.move_to_next_round(ch[r])
        r += 1
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    sc.close()
    out({"config": "c5 (per-GPU share)", "workload": "sumcheck GF(2^128), 2^%d evals, d=%d, shard 0 of %d: %d local rounds"
         % (nvars, d, world, r), "value": (1 << nvars) / world / dt, "unit": "evals/s (this shard)", "ms": dt * 1e3})


def bb_line(dev, out, log_n, batch):
    import torch
    import binius_ntt_amd as B
    st = torch.cuda.current_stream(dev)
    n = 1 << log_n
    x = torch.from_numpy(np.random.default_rng(9).integers(0, 2**32, size=n * batch, dtype=np.uint64)
                         .astype(np.uint32).view(np.int32)).to(dev)
    y = torch.empty_like(x)
    ntt = B.NTT(B.NTTConfRad2(B.BB31(137), 27, log_n))
    ms = ev_time(lambda: ntt.forward_device(x, y, batch=batch, stream=st), 20, st)
    out({"config": "bb", "workload": "BabyBear NTT 2^%d x %d (natural order in/out)" % (log_n, batch),
         "value": n * batch / (ms * 1e-3), "unit": "elements/s", "ms": ms,
         "hbm_gbps_algorithmic": 8 * n * batch / (ms * 1e-3) / 1e9})


def qm_line(dev, out, nvars, reps=3):
    import torch
    import binius_ntt_amd.prime_field as PF
    ev = np.random.default_rng(11).integers(0, 2**31 - 1, size=(2 << nvars, 4), dtype=np.uint64).astype(np.uint32)
    r = PF.QM31([32482843, 85864538, 8348234, 9544334])
    best = None
    for _ in range(reps):
        sc = PF.Sumcheck(nvars, ev, device=dev.index or 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(nvars):
            sc.this_round_messages()
            sc.fold(r)
        sc.final_values()
        dt = time.perf_counter() - t0
        sc.close()
        best = dt if best is None else min(best, dt)
    out({"config": "qm", "workload": "QM31 sumcheck 2 x 2^%d, d=2, all rounds" % nvars,
         "value": (1 << nvars) / best, "unit": "evals/s", "ms": best * 1e3,
         # per round over cur evals: the fused fold+messages pass reads 2 x 16 B x cur and writes
         # half of that; sum of cur over rounds ~ 2 x 2^N  ->  96 B per eval
         "hbm_gbps_algorithmic": 96 * (1 << nvars) / best / 1e9})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="c2,c3,c4,c5,bb,qm")
    ap.add_argument("--sc-vars", type=int, default=24)
    ap.add_argument("--sc-d", default="2,3,4")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    lines = []

    def out(d):
        lines.append(d)
        print(json.dumps(d), flush=True)

    only = set(a.only.split(","))
    if "c2" in only:
        c2(dev, out)
    if "c3" in only:
        ntt_line(dev, out, "c3", 20, 1)
    if "c4" in only:
        c4(dev, out, a.sc_vars, [int(x) for x in a.sc_d.split(",")])
        for d in [int(x) for x in a.sc_d.split(",")]:
            c4_phases(dev, out, a.sc_vars, d)
    if "c5" in only:
        ntt_line(dev, out, "c5 (per-GPU share)", 20, 32)
        c5_sumcheck_shard(dev, out)
        c5_sumcheck_single(dev, out)
    if "bb" in only:
        bb_line(dev, out, 24, 1)
        bb_line(dev, out, 20, 16)
    if "qm" in only:
        qm_line(dev, out, 24)
    if a.out:
        with open(a.out, "w") as f:
            for d in lines:
                f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
