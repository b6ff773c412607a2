"""Debug helper: one small write log, report which pages' bytes / CRCs differ."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from curve_amd import crc as C
from oracle import oracle as O
dev = torch.device("cuda", 0)
for delta in (False, True):
    for case in ("one_whole_aligned", "one_unaligned", "tiny", "random", "random_big"):
        rng = np.random.default_rng(5)
        pb, pool_bytes = 4096, 1 << 20
        host = rng.integers(0, 256, pool_bytes, dtype=np.uint8)
        d_pool = torch.from_numpy(host.copy()).to(dev)
        crcs = C.page_crc(d_pool, pb)
        src = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
        if case == "one_whole_aligned":
            dst, so, ln = np.array([8192 + 256]), np.array([512]), np.array([1024])
        elif case == "one_unaligned":
            dst, so, ln = np.array([8192 + 257]), np.array([513]), np.array([1030])
        elif case == "tiny":
            dst, so, ln = np.array([8192 + 261, 3 * 4096 + 17, 5 * 4096 + 30]), np.array([5, 100, 7]), np.array([2, 16, 21])
        elif case == "random_big":
            n = 3000
            ln = rng.integers(1, 4097, n); dst = rng.integers(0, pool_bytes - 4096, n); so = rng.integers(0, (1 << 16) - 4096, n)
        else:
            n = 50
            ln = rng.integers(1, 4097, n); dst = rng.integers(0, pool_bytes - 4096, n); so = rng.integers(0, (1 << 16) - 4096, n)
        C.apply_updates(d_pool, crcs, torch.from_numpy(src).to(dev), dst, so, ln, pb, delta=delta)
        want = host.copy()
        for i in range(len(dst)):
            want[dst[i]:dst[i] + ln[i]] = src[so[i]:so[i] + ln[i]]
        got = d_pool.cpu().numpy()
        badb = np.flatnonzero(got != want)
        wc = O.page_crcs(want, pb)
        gc = crcs.cpu().numpy().view(np.uint32)
        badc = np.flatnonzero(wc != gc)
        print(f"delta={delta} {case}: bad bytes {badb.size} first {badb[:8].tolist()} pages {sorted(set((badb // pb).tolist()))[:8]}; bad crcs {badc[:8].tolist()}")
        if badb.size:
            b = badb[0]
            print("   got", got[b - 4:b + 8].tolist(), "want", want[b - 4:b + 8].tolist(), "old", host[b - 4:b + 8].tolist())
