"""Host side of a sumcheck round (c4: 2^24 evals, d=3, bitsliced), through the Python mirror:
per round, the wall time inside this_round_messages (the claim, the poll for the posted points)
and inside move_to_next_round (fold + next messages launches), medians over 3 protocol runs.
  python tools/sc_host_timing.py [nvars] [d]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "binius-ntt_amd", "python"))


def main():
    import torch
    import binius_ntt_amd as B
    nvars = int(sys.argv[1]) if len(sys.argv) > 1 else 24
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    g = np.random.default_rng(5)
    ev = torch.from_numpy(g.integers(0, 2**32, size=4 * (1 << nvars) * d, dtype=np.uint64).astype(np.uint32).view(np.int32)).to(dev)
    ch = g.integers(0, 2**32, size=(nvars, 4), dtype=np.uint64).astype(np.uint32)
    runs = []
    for _ in range(4):
        sc = B.Sumcheck(nvars, d, True, ev)
        torch.cuda.synchronize()
        tm, tv = [], []
        t0 = time.perf_counter()
        for r in range(nvars):
            a = time.perf_counter()
            sc.this_round_messages()
            b = time.perf_counter()
            sc.move_to_next_round(ch[r])
            c = time.perf_counter()
            tm.append(b - a)
            tv.append(c - b)
        a = time.perf_counter()
        sc.this_round_messages()
        tm.append(time.perf_counter() - a)
        runs.append((time.perf_counter() - t0, tm, tv))
        sc.close()
    runs = runs[1:]
    runs.sort(key=lambda x: x[0])
    total, tm, tv = runs[1]
    print("total %.3f ms" % (total * 1e3))
    for r in range(nvars + 1):
        print("round %2d  messages call %7.1f us  move call %6.1f us" % (r, tm[r] * 1e6, tv[r] * 1e6 if r < nvars else 0.0))
    print("sum messages %.1f us, sum move %.1f us" % (sum(tm) * 1e6, sum(tv) * 1e6))


if __name__ == "__main__":
    main()
