# Dev measurement (not part of the library): bitsliced GF(2^128) quad-product rate (k_repeat_quad)
# against the number of dependent products per quad, at a fixed total of products; the short cases
# include the state/operand traffic (1.5 KiB per quad). Result: DESIGN.md section 5.4.
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "binius-ntt_amd", "python"))
import binius_ntt_amd as B
dev = torch.device("cuda:0"); st = torch.cuda.current_stream(dev)
g = np.random.default_rng(1)
total = 256 * 1024 * 200  # quad-products
for iters in (1, 2, 4, 8, 16, 50, 200):
    threads = total // iters
    state = torch.from_numpy(g.integers(0, 2**32, size=threads * 128, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    opnd = torch.from_numpy(g.integers(0, 2**32, size=threads * 128, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    B.gf128_mul_repeat(2, state, opnd, threads, iters, stream=st); torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(3): B.gf128_mul_repeat(2, state, opnd, threads, iters, stream=st)
    b.record(st); b.synchronize()
    ms = a.elapsed_time(b) / 3
    print("iters %4d threads %9d: %.3f ms, %.3e products/s" % (iters, threads, ms, threads * iters * 32 / (ms * 1e-3)), flush=True)
    del state, opnd; torch.cuda.empty_cache()
