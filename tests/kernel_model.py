"""CPU replay of the page kernel's arithmetic (curve_amd/csrc/kernels.hip).

Uses the exact LDS image the library uploads (cc_lds_image), forms every LDS
address the way the kernel does (v_perm_b32 byte splice, immediate offsets),
runs the per-lane Horner chain, the lane-specific nibble final map and the
wave XOR-reduce.  Lets the CPU suite pin the table math and the address
layout; only instruction semantics remain for the GPU tests.
"""
from __future__ import annotations

import ctypes

import numpy as np

K_LDS_BYTES = 163840
K_FIN_BASE = 131072


def lds_image() -> np.ndarray:
    from curve_amd import _lib
    img = np.zeros(K_LDS_BYTES // 4, dtype=np.uint32)
    rc = _lib.lib().cc_lds_image(ctypes.c_void_p(img.ctypes.data), K_LDS_BYTES)
    assert rc == 0
    return img


def v_perm_b32(s0: np.ndarray, s1: np.ndarray, sel: int) -> np.ndarray:
    """V_PERM_B32: D.byte[i] = byte sel.byte[i] of the 64-bit {S0:S1}
    (0-3 -> S1 bytes, 4-7 -> S0 bytes, 12 -> 0x00); only selectors the kernel uses."""
    s0 = s0.astype(np.uint64)
    s1 = s1.astype(np.uint64)
    out = np.zeros(np.broadcast(s0, s1).shape, dtype=np.uint64)
    for i in range(4):
        b = (sel >> (8 * i)) & 0xFF
        if b < 4:
            v = (s1 >> np.uint64(8 * b)) & np.uint64(0xFF)
        elif b < 8:
            v = (s0 >> np.uint64(8 * (b - 4))) & np.uint64(0xFF)
        elif b == 12:
            v = np.zeros_like(out)
        else:
            raise NotImplementedError(hex(b))
        out |= v << np.uint64(8 * i)
    return out.astype(np.uint32)


def lds_read(img: np.ndarray, byte_addr: np.ndarray) -> np.ndarray:
    a = byte_addr.astype(np.int64)
    assert (a % 4 == 0).all() and (a >= 0).all() and (a < K_LDS_BYTES).all()
    return img[a // 4]


def page_crcs_model(pages: np.ndarray, page_bytes: int, img: np.ndarray | None = None) -> np.ndarray:
    """Replay the kernel over `pages` (uint8, n*page_bytes) -> uint32 CRCs."""
    from curve_amd import crc as C
    if img is None:
        img = lds_image()
    M = page_bytes // 256
    words = np.ascontiguousarray(pages).view(np.uint32).reshape(-1, M, 64)  # [page, j, lane]
    lane = np.arange(64, dtype=np.uint32)
    c0 = (lane << 2) & np.uint32(0x7C)
    c1 = c0 | np.uint32(0x10000)
    cf = np.uint32(K_FIN_BASE) + (lane << 2)
    s = words[:, 0, :].copy()
    for j in range(1, M):
        t0 = lds_read(img, v_perm_b32(c0, s, 0x0C060004))
        t1 = lds_read(img, v_perm_b32(c0, s, 0x0C060104) + 128)
        t2 = lds_read(img, v_perm_b32(c1, s, 0x0C060204))
        t3 = lds_read(img, v_perm_b32(c1, s, 0x0C060304) + 128)
        s = t0 ^ t1 ^ t2 ^ t3 ^ words[:, j, :]
    r = np.zeros_like(s)
    for n in range(8):
        v = (s >> np.uint32(4 * n)) & np.uint32(15)
        r ^= lds_read(img, ((v << np.uint32(8)) | cf) + np.uint32(4096 * n))
    red = np.bitwise_xor.reduce(r, axis=1)
    return red ^ np.uint32(C.zeros(page_bytes))


def bank_conflicts(byte_addrs: np.ndarray) -> int:
    """Extra LDS cycles of one ds_read_b32 wave instruction (64 lane addresses),
    per the gfx950 rule: lane groups {0-31},{32-63}, bank = (a/4) mod 32,
    identical addresses broadcast."""
    extra = 0
    for g in (byte_addrs[:32], byte_addrs[32:]):
        banks = {}
        for a in g.tolist():
            banks.setdefault((a // 4) % 32, set()).add(a)
        extra += max(len(v) for v in banks.values()) - 1
    return extra


def geometry(n_pages: int, cus: int = 256, waves_per_block: int = 16):
    """engine.hip geometry_for(): (blocks, tile_shift)."""
    waves = cus * waves_per_block
    ts = 6
    while ts > 0 and (n_pages >> ts) < waves:
        ts -= 1
    tiles = (n_pages + (1 << ts) - 1) >> ts
    need = (tiles + waves_per_block - 1) // waves_per_block
    blocks = need if need < cus else cus
    return max(blocks, 1), ts


def tile_walk(n_pages: int, blocks: int, ts: int, waves_per_block: int = 16):
    """Replay page_crc_kernel's per-wave page sequence and flushes.
    Returns (pages hashed in order, [(tile_first, cnt)] flushes)."""
    hashed, flushes = [], []
    tmask = (1 << ts) - 1
    wstride = (blocks * waves_per_block) << ts
    for w in range(blocks * waves_per_block):
        wfirst = w << ts
        if wfirst >= n_pages:
            continue
        k, page = 0, wfirst
        while True:
            hashed.append(page)
            k1 = k + 1
            p1 = wfirst + (k1 >> ts) * wstride + (k1 & tmask)
            if (k & tmask) == tmask or p1 >= n_pages:
                flushes.append((page - (k & tmask), (k & tmask) + 1))
            if p1 >= n_pages:
                break
            k, page = k1, p1
    return hashed, flushes


POLY = 0x82F63B78


def mulmod(a: int, b: int) -> int:
    prod = 0
    for i in range(32):
        if a & (0x80000000 >> i):
            prod ^= b
        b = (b >> 1) ^ (POLY if b & 1 else 0)
    return prod


def div_x(b: int) -> int:
    return (((b ^ POLY) << 1) | 1) & 0xFFFFFFFF if b & 0x80000000 else (b << 1) & 0xFFFFFFFF


def xinv_bytes(t: int) -> int:
    r = 0x80000000
    for _ in range(8 * t):
        r = div_x(r)
    return r


def range_crc_model(buf: np.ndarray, off: int, length: int, img: np.ndarray) -> int:
    """Replay range_crc_kernel for one range of a uint8 buffer."""
    from curve_amd import crc as C
    if length == 0:
        return 0
    a, end = off & ~3, off + length
    rows = (length + (off - a) + 255) >> 8
    t = (rows << 8) - (off - a) - length
    lane = np.arange(64, dtype=np.uint64)
    padded = np.zeros(a + rows * 256 + 8, dtype=np.uint8)
    padded[:buf.size] = buf[:padded.size] if buf.size > padded.size else buf
    words = []
    for j in range(rows):
        addr = a + (j << 8) + 4 * lane
        w = np.zeros(64, dtype=np.uint32)
        for l in range(64):
            ad = int(addr[l])
            if ad >= end:
                continue
            v = int.from_bytes(bytes(padded[ad:ad + 4]), "little")
            if ad < off:
                v &= (0xFFFFFFFF << (8 * (off - ad))) & 0xFFFFFFFF
            if ad + 4 > end:
                v &= 0xFFFFFFFF >> (8 * (ad + 4 - end))
            w[l] = v
        words.append(w)
    lanes = np.arange(64, dtype=np.uint32)
    c0 = (lanes << 2) & np.uint32(0x7C)
    c1 = c0 | np.uint32(0x10000)
    cf = np.uint32(K_FIN_BASE) + (lanes << 2)
    s = words[0].copy()
    for j in range(1, rows):
        t0 = lds_read(img, v_perm_b32(c0, s, 0x0C060004))
        t1 = lds_read(img, v_perm_b32(c0, s, 0x0C060104) + 128)
        t2 = lds_read(img, v_perm_b32(c1, s, 0x0C060204))
        t3 = lds_read(img, v_perm_b32(c1, s, 0x0C060304) + 128)
        s = t0 ^ t1 ^ t2 ^ t3 ^ words[j]
    r = np.zeros_like(s)
    for n in range(8):
        v = (s >> np.uint32(4 * n)) & np.uint32(15)
        r ^= lds_read(img, ((v << np.uint32(8)) | cf) + np.uint32(4096 * n))
    raw_pad = int(np.bitwise_xor.reduce(r))
    return mulmod(xinv_bytes(t), raw_pad) ^ C.zeros(length)


def range_flat_items(B: int, waves: int, rounds: int = 1, dyn_div: int = 32, dyn_blocks: int = 16):
    """Work items of range_flat_kernel over a stream of B blocks: `rounds`
    static pieces per wave ([Bs c / RW, Bs (c+1) / RW), c < rounds * waves,
    empty ones skipped), then the dynamic tail's chunks of dyn_blocks blocks."""
    Bs = B - B // dyn_div if dyn_div else B
    RW = rounds * waves
    items = [(Bs * c // RW, Bs * (c + 1) // RW) for c in range(RW)]
    items = [it for it in items if it[0] < it[1]]
    n_dyn = (B - Bs + dyn_blocks - 1) // dyn_blocks
    items += [(Bs + c * dyn_blocks, min(Bs + (c + 1) * dyn_blocks, B)) for c in range(n_dyn)]
    return items


def range_flat_segments(nbs, waves: int, **kw):
    """Segments (range, first block, blocks) the kernel hashes for ranges of
    nbs[r] blocks: each item cut at the range boundaries it crosses."""
    starts = np.concatenate([[0], np.cumsum(nbs)]).astype(np.int64)
    segs = []
    for b0, b1 in range_flat_items(int(starts[-1]), waves, **kw):
        r = int(np.searchsorted(starts, b0, side="right")) - 1
        b = b0
        while b < b1:
            while nbs[r] == 0 or starts[r + 1] <= b:
                r += 1
            e = min(b1, int(starts[r + 1]))
            segs.append((r, b - int(starts[r]), e - b))
            b = e
    return segs


def range_accumulate(segs, nbs, contrib, rng):
    """The split-range meeting point, in a random arrival order: a segment that
    is its range whole stores; any other XORs into the range's pair, adds its
    blocks, and the one whose add completes nb takes the XOR, stores and clears
    the pair.  Returns (out, pairs left non-zero, stores per range)."""
    out, stores = {}, {}
    acc = {}
    for i in rng.permutation(len(segs)):
        r, kb, cnt = segs[i]
        v = contrib[i]
        if kb == 0 and cnt == nbs[r]:
            out[r] = v
            stores[r] = stores.get(r, 0) + 1
            continue
        x, c = acc.get(r, (0, 0))
        x ^= v
        if c + cnt == nbs[r]:
            out[r] = x
            stores[r] = stores.get(r, 0) + 1
            acc[r] = (0, 0)
        else:
            acc[r] = (x, c + cnt)
    left = [r for r, p in acc.items() if p != (0, 0)]
    return out, left, stores


def verify_flat_pages(counts, waves: int, tiles: int = 512, dyn_div: int = 16, dyn_slots: int = 32,
                      min_slots: int = 8):
    """The page slots read_verify_kernel hashes, as (read, page-of-read) pairs in
    the order each share visits them: its static shares [Ts w / W, Ts (w+1) / W)
    and the dynamic chunks, each started at the tile holding its first slot (tile
    counts of reads [n t / tiles, n (t+1) / tiles)) and walked 64 reads a group
    from the tile's first read, the group's first slot being the running sum of
    the groups before it -- exactly the kernel's arithmetic."""
    n = len(counts)
    counts = np.asarray(counts, dtype=np.int64)
    tb = np.array([counts[n * t // tiles:n * (t + 1) // tiles].sum() for t in range(tiles)], dtype=np.int64)
    cum_t = np.cumsum(tb)
    T = int(cum_t[-1]) if tiles else 0
    Wt = (T + min_slots - 1) // min_slots
    W = min(Wt if Wt else 1, waves)
    Ts = T - T // dyn_div
    out = []

    def share(lo, hi):
        if lo >= hi:
            return
        t = int(np.searchsorted(cum_t, lo, side="right"))  # first tile whose running count passes lo
        base = n * t // tiles
        S = int(cum_t[t - 1]) if t else 0
        while True:  # the tile's reads 64 at a time, to the group whose pages pass lo
            tot = int(counts[base:base + 64].sum())
            if S + tot > lo or base + 64 >= n:
                break
            S += tot
            base += 64
        while base < n and S < hi:
            grp = counts[base:base + 64]
            cum = np.cumsum(grp)
            P = int(cum[-1])
            ks = lo - S if lo > S else 0
            ke = min(hi - S, P)
            for k in range(ks, ke):
                owner = int(np.searchsorted(cum, k, side="right"))
                before = int(cum[owner - 1]) if owner else 0
                out.append((base + owner, k - before))
            S += P
            base += 64

    for w in range(W):
        share(Ts * w // W, Ts * (w + 1) // W)
    n_dyn = (T - Ts + dyn_slots - 1) // dyn_slots
    for c in range(n_dyn):
        lo = Ts + c * dyn_slots
        share(lo, min(lo + dyn_slots, T))
    return out


# ---------------------------------------------------------------------------
# Write-log page kernel: age-weighted static shares + tail stealing
# (kernels.hip log_pages_body, round 4).  An event simulation over per-wave
# speeds: every wave rehashes its share [first, H); the last 1/tail_div of it
# (the tail, from ts) is claimed by one atomic max -- the owner as it starts the
# page before the tail (read when that page is done), a finished wave after a scan of 64
# candidates (the 4 youngest waves of the next 16 workgroups).  The table slot
# of a head is cleared by the wave that won it, after that wave read it.
# ---------------------------------------------------------------------------
SKEW = (33, 27, 22, 18)


def log_share(Hall: int, grid: int, wv: int, b: int, w: int):
    pre = lambda t: sum(SKEW[(u // 4) & 3] for u in range(t))  # noqa: E731
    h0, h1 = Hall * b // grid, Hall * (b + 1) // grid
    Hb, ws = h1 - h0, pre(wv)
    return h0 + Hb * pre(w) // ws, h0 + Hb * pre(w + 1) // ws


def log_steal_schedule(Hall: int, grid: int, wv: int, speed, tail_div: int = 4, max_steals: int = 4, start=None):
    """-> (owner[h]: the wave that rehashed head h, cleared_by[h], read_ok,
    end[w]: when each wave finished).  speed[w]: time per page of wave w;
    start[w]: when it starts (a workgroup not yet resident starts late)."""
    import heapq
    W = grid * wv
    start = start if start is not None else [0.0] * W
    claim = [None] * W  # who won wave w's tail
    owner = [-1] * Hall
    cleared = [False] * Hall
    read_ok = True
    end = [0.0] * W
    shares = [log_share(Hall, grid, wv, w // wv, w % wv) for w in range(W)]
    tails = [(h - (h - f) // tail_div, h) for f, h in shares]
    # a wave's life as a generator of (time, action) steps; actions run in time order
    def life(w):
        nonlocal read_ok
        t = start[w]
        f, H = shares[w]
        ts, _ = tails[w]
        segs = [(f, H, True)]
        steals = 0
        while segs:
            s0, s1, own = segs.pop()
            if own and ts < H:
                # own part; the claim goes out as the page before the tail starts
                issue = max(ts - 1, s0)
                for h in range(s0, s1):
                    if h == issue:
                        yield t, ("claim", w, w)
                    if h == ts:
                        if claim[w] != w:
                            break
                        for k in range(ts, s1):
                            if cleared[k]:
                                read_ok = False
                            cleared[k] = True  # cleared once won (read at load time, before)
                    if h < ts:
                        if cleared[h]:
                            read_ok = False
                        cleared[h] = True
                    t += speed[w]
                    yield t, ("page", w, h)
            else:
                for h in range(s0, s1):
                    if own or True:
                        if cleared[h]:
                            read_ok = False
                        cleared[h] = True
                for h in range(s0, s1):
                    t += speed[w]
                    yield t, ("page", w, h)
            if steals >= max_steals:
                break
            # scan: the 4 youngest waves of the next 16 workgroups
            b = w // wv
            got = None
            for l in range(64):
                vb, vw = (b + 1 + l // 4) % grid, wv - 1 - l % 4
                v = vb * wv + vw
                if v != w and tails[v][0] < tails[v][1] and claim[v] is None:
                    yield t, ("claim", w, v)
                    if claim[v] == w:
                        got = v
                        break
            if got is None:
                break
            steals += 1
            segs.append((tails[got][0], tails[got][1], False))
        end[w] = t
    gens = {w: life(w) for w in range(W)}
    heap = []
    for w, g in gens.items():
        try:
            tt, act = next(g)
            heapq.heappush(heap, (tt, w, act))
        except StopIteration:
            end[w] = start[w]
    while heap:
        tt, w, act = heapq.heappop(heap)
        kind, who, v = act
        if kind == "claim" and claim[v] is None:
            claim[v] = who
        elif kind == "page":
            owner[v] = who if owner[v] == -1 else -2  # -2: rehashed twice
        try:
            tt, act = next(gens[w])
            heapq.heappush(heap, (tt, w, act))
        except StopIteration:
            pass
    return owner, cleared, read_ok, end


def log_head_segments(counts, base: int, H: int, kspl: int = 4):
    """The write-log page kernel's head addressing (round 4): insert block b
    leaves counts[b] head records in its own segment; a batch of heads
    [base, min(base + 64, H)) in segment order finds, per lane, (segment,
    record) -- the segment holding `base` by a register search, then a walk
    over the segments the batch spans.  Returns [(segment, record)] per head."""
    counts = list(counts) + [0] * (64 * kspl - len(counts))
    n_segs = len(counts)
    # lane l holds segments kspl*l .. kspl*l + kspl-1; scum = inclusive prefix of the lane sums
    lane_sum = [sum(counts[kspl * l:kspl * l + kspl]) for l in range(64)]
    scum = np.cumsum(lane_sum)
    tl = int(np.argmax(scum > base))
    st = int(scum[tl - 1]) if tl else 0
    s = kspl * tl
    for j in range(kspl):
        v = counts[kspl * tl + j]
        if st + v > base:
            s = kspl * tl + j
            break
        st += v
    seg = [s] * 64
    sbefore = [st] * 64
    his = [base + l if base + l < H else base for l in range(64)]
    last = min(base + 63, H - 1)
    while True:
        cnt = counts[s]
        if st + cnt > last or s + 1 >= n_segs:
            break
        st += cnt
        s += 1
        for l in range(64):
            if his[l] >= st:
                seg[l], sbefore[l] = s, st
    return [(seg[l], his[l] - sbefore[l]) for l in range(64) if base + l < H]
