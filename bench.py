#!/usr/bin/env python3
"""Headline benchmark: 2^24-point GF(2^128) additive NTT (BASELINE.json configs[...], north star).

One "step" = one full forward transform (log_h = 24, log_rate = 0) of a device-resident,
synthetic GF(2^128) vector (numpy PCG64, seed 0xdeadbeef + 24 + rank) into a separate device
output buffer. The oracle (test infrastructure) is used only by the cpu_baseline leg.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--log-h 24] [--no-cpu]

N > 1 is launched by torch.distributed.run: every rank transforms its own 2^24 vector
(independent transforms = batched sharding, weak scaling, no data-path collective); the timed
region is bracketed by barriers + synchronize and the max over ranks is reported. Rank 0
prints one JSON line.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "binius-ntt_amd", "python"))

HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-h", type=int, default=24)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-log-h", type=int, default=24)
    return ap.parse_args()


def cpu_baseline(log_h):
    """Oracle (C restatement of the reference algorithm) on one transform: 1 thread (the
    reported value), and the 4 limb-plane GF(2^32) transforms on 4 threads (`parallel`)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from concurrent.futures import ThreadPoolExecutor
    import numpy as np
    import _oracle as O
    x = O.fill128(0xDEADBEEF + log_h, 0x5EED0000, 1 << log_h)
    t0 = time.perf_counter()
    O.antt128(x, log_h, 0)
    dt = time.perf_counter() - t0
    planes = [np.ascontiguousarray(x.reshape(-1, 4)[:, j]) for j in range(4)]
    t1 = time.perf_counter()
    with ThreadPoolExecutor(4) as ex:  # ctypes releases the GIL inside the oracle
        list(ex.map(lambda p: O.antt32(p, log_h, 0), planes))
    dt4 = time.perf_counter() - t1
    return {"value": (1 << log_h) / dt, "unit": "elements/s", "cores": 1, "kind": "port",
            "sample": "one 2^%d-point GF(2^128) additive NTT (r=0), oracle/ C port of the reference "
                      "algorithm, 1 thread, %.2f s" % (log_h, dt),
            "parallel": {"value": (1 << log_h) / dt4, "cores": 4,
                         "sample": "same transform as 4 limb-plane GF(2^32) transforms on 4 threads, %.2f s"
                                   % dt4}}


def load_valu_insts():
    """SQ_INSTS_VALU per launch of each pass kernel from the committed PMC summary (rocprofv3)."""
    try:
        with open(os.path.join(ROOT, "profiles", "r01", "pmc_summary.json")) as f:
            d = json.load(f)
        return [v.get("SQ_INSTS_VALU") for k, v in sorted(d.items(), key=lambda kv: kv[0])]
    except (OSError, ValueError):
        return None


def load_pmc(log_h):
    """HBM traffic per launch from the committed rocprofv3 PMC summary, if present."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(str(log_h))
    except (OSError, ValueError):
        return None


VALU_PEAK_WAVE_INSTS = 256 * 4 * 0.5 * 2.4e9


def valu_block(dom, dom_ms):
    insts = load_valu_insts()
    if not insts or dom is None or dom >= len(insts) or not insts[dom]:
        return None
    rate = insts[dom] / (dom_ms * 1e-3)
    return {"insts_per_launch": insts[dom], "achieved": rate, "peak": VALU_PEAK_WAVE_INSTS,
            "unit": "wave64 instructions/s", "frac": rate / VALU_PEAK_WAVE_INSTS}


def apply_e2e(B, ntt, d_in, n, reps=3):
    """Reference-semantics AdditiveNTT::apply (host buffers: H2D + transform + D2H, synchronous);
    reported beside `value`, never as it."""
    import numpy as np
    host = d_in.cpu().numpy().view(np.uint32).reshape(n, 4)
    inp = B.NTTData(n, B.DataOrder.IN_ORDER, 128, host)
    out = B.NTTData(n, B.DataOrder.INVALID, 128)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        if not ntt.apply(inp, out):
            return None
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    return {"ms": t * 1e3, "elements_per_s": n / t, "reps": reps,
            "note": "AdditiveNTT.apply on pageable host buffers (PCIe-inclusive), median"}


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    import binius_ntt_amd as B

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; BENCH_DIST_BACKEND=gloo rehearses the multi-rank path on fewer GPUs
    # (ranks then share devices round-robin; the timing all-reduce runs on CPU tensors)
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local = local % max(1, ndev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    log_h = a.log_h
    n = 1 << log_h

    # synthetic input generated on the host, resident in HBM before timing
    x = np.random.default_rng(0xDEADBEEF + log_h + rank).integers(0, 2**32, size=4 * n, dtype=np.uint64)
    d_in = torch.from_numpy(x.astype(np.uint32).view(np.int32)).to(dev)
    del x
    d_out = torch.empty_like(d_in)
    ntt = B.AdditiveNTT(B.AdditiveNTTConf(log_h, 0, B.FanPaarTowerField(7), device=local))
    stream = torch.cuda.current_stream(dev)

    for _ in range(a.warmup):
        ntt.forward_device(d_in, d_out, stream=stream)
    torch.cuda.synchronize(dev)

    # per-kernel timing with hipEvents on the launch stream (separate, untimed pass)
    ntt.set_event_timing(True)
    for _ in range(max(3, min(a.steps, 10))):
        ntt.forward_device(d_in, d_out, stream=stream)
    kind_ms = ntt.event_timing()
    ntt.set_event_timing(False)
    torch.cuda.synchronize(dev)

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        ntt.forward_device(d_in, d_out, stream=stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    ms_step = dt / a.steps * 1e3
    elems_per_s = world * n / (dt / a.steps)
    alg_bytes = 2 * 16 * n  # read input once + write output once
    transform_gbps = alg_bytes / (ms_step * 1e-3) / 1e9

    if rank == 0:
        # dominant kernel = the pass with the largest mean hipEvent duration; each pass reads and
        # writes the whole vector once, so its algorithmic bytes are the same 32 B/element.
        dom = max(range(len(kind_ms)), key=lambda i: kind_ms[i]) if kind_ms else None
        dom_ms = kind_ms[dom] if dom is not None else ms_step
        achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
        pmc = load_pmc(log_h)
        res = {
            "metric": "GF(2^128) additive-NTT elements/sec (2^24 pts)",
            "value": elems_per_s,
            "unit": "elements/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "gf2_128 (u32 limbs, bitwise)",
            "data": "synthetic (numpy PCG64 seeded limbs)",
            "config": {"workload": "additive NTT over GF(2^128), log_h=%d, log_rate=0, one transform per GPU"
                                   % log_h, "log_h": log_h, "log_rate": 0, "field": "GF(2^128)",
                       "kernel_variant": ntt.variant(), "parallelism": "independent transform per rank"},
            "hbm_gbps_transform": transform_gbps,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": pmc,
                "kernel": "pass %s of %d" % (dom, len(kind_ms)),
                "kernel_ms": dom_ms,
                "pass_ms": kind_ms,
                "transform_frac": transform_gbps / HBM_PEAK_GBPS,
            },
            # the pass kernels are VALU-issue bound: wave-instructions per launch
            # (SQ_INSTS_VALU, committed PMC run) / the live hipEvent duration vs the issue peak of
            # 256 CU x 4 SIMD x 0.5 wave64 instructions/cycle x 2.4 GHz
            "valu": valu_block(dom, dom_ms),
        }
        if world == 1:
            res["apply_e2e"] = apply_e2e(B, ntt, d_in, n)
        if not a.no_cpu and world == 1:
            res["cpu_baseline"] = cpu_baseline(a.cpu_log_h)
        else:
            res["cpu_baseline"] = None
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
