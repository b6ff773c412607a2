#!/usr/bin/env python3
"""A/B build of the write log (NOT the shipped kernel): patches a COPY of
kernels.hip with log_group_kernel<G, WV> -- G pages per wave, 64/G lanes per
page, each lane holding a 4G-byte chunk of every 256-byte row (G = 4: the round-4
"quad" layout, dwordx4; G = 2: dwordx2, 32 lanes a page) and G Horner chains
per lane -- and routes 4 KiB full-mode logs to it.  Pages with several pieces are
finished one per wave after the batch (log_page_multi, from the round-4 quad
kernel).  usage: log_group.py KERNELS_HIP G WAVES"""
import sys

p, G, WV = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
assert G in (2, 4)
s = open(p).read()
# log_page_multi (the quad kernel's multi-piece pages) from the round-4 tree that still had it
import subprocess
src = subprocess.run(["git", "show", "8166fb9:curve_amd/csrc/kernels.hip"], capture_output=True, text=True,
                     check=True, cwd=__import__("os").path.dirname(__import__("os").path.abspath(__file__))).stdout
multi = src[src.index("// A page with several pieces, by one wave, not pipelined"):
            src.index("// byte mask of chunk dword k (chunk bytes 4k .. 4k+3) inside [pa, pb), 0 <= pa < pb <= 16")]

KERNEL = r'''
// ---------------------------------------------------------------------------
// Write log, 4 KiB pages, full rehash: G pages per wave (A/B build).
// Lane L = LP g + i (LP = 64 / G lanes a page) holds page g's CB-byte chunk i
// (CB = 4 G) of every 256-byte row j in X[j]; its G chains k run over dwords
// G i + k + 64 j = the chains of lanes v = G i + k of the one-page layout; the
// page's LP lanes XOR their shares.
// ---------------------------------------------------------------------------
constexpr int kGrpG = @G@;
constexpr int kGrpWaves = @WV@;
constexpr int kGrpLP = 64 / kGrpG;        // lanes a page
constexpr uint32_t kGrpCB = 4u * kGrpG;   // chunk bytes a lane
typedef uint32_t gvec __attribute__((ext_vector_type(kGrpG)));
typedef __attribute__((address_space(1))) gvec ggvec;
typedef __attribute__((address_space(1))) uint32_t gu32;

@MULTI@

// byte mask of chunk dword k (chunk bytes 4k .. 4k+3) inside [pa, pb), 0 <= pa < pb <= CB
__device__ __forceinline__ uint32_t grp_dword_mask(uint32_t pa, uint32_t pb, int k) {
    const int32_t lo = min(max((int32_t)pa - 4 * k, 0), 4), hi = min(max((int32_t)pb - 4 * k, 0), 4);
    return (uint32_t)(((1ull << (8 * hi)) - 1ull) & ~((1ull << (8 * lo)) - 1ull));
}
struct GrpGeo {
    uint32_t rlo, rhi;
    uint32_t ce[2];
    bool ex[2];
    uint32_t pa[2], pz[2];
};
__device__ __forceinline__ GrpGeo grp_geo(uint32_t rr) {
    GrpGeo q;
    q.rlo = rr & 0xFFFFu;
    q.rhi = rr >> 16;
    q.ce[0] = q.rlo & ~(kGrpCB - 1u);
    q.ex[0] = (q.rlo & (kGrpCB - 1u)) || q.rhi < q.ce[0] + kGrpCB;
    q.ce[1] = (q.rhi - 1u) & ~(kGrpCB - 1u);
    q.ex[1] = q.ce[1] != q.ce[0] && (q.rhi & (kGrpCB - 1u));
    q.pa[0] = q.rlo - q.ce[0];
    q.pz[0] = (q.rhi < q.ce[0] + kGrpCB ? q.rhi : q.ce[0] + kGrpCB) - q.ce[0];
    q.pa[1] = 0;
    q.pz[1] = q.rhi - q.ce[1];
    return q;
}
struct GrpSet {
    gvec X[16];
    gvec D[2][2];  // edge chunks: the two CB-aligned source blocks around their bytes
    uint64_t sp;
    uint32_t pg, rr;
    bool valid;
};
template <int OFF>
__device__ __forceinline__ void grp_store_if(bool c, gvec v, uint64_t addr) {
    const uint64_t m = __ballot(c);
    uint64_t sv;
    if constexpr (kGrpG == 4) {
        asm volatile("s_and_saveexec_b64 %0, %1\n\tglobal_store_dwordx4 %2, %3, off offset:%4 nt\n\ts_mov_b64 exec, %0"
                     : "=&s"(sv) : "s"(m), "v"(addr), "v"(v), "i"(OFF) : "memory");
    } else {
        asm volatile("s_and_saveexec_b64 %0, %1\n\tglobal_store_dwordx2 %2, %3, off offset:%4 nt\n\ts_mov_b64 exec, %0"
                     : "=&s"(sv) : "s"(m), "v"(addr), "v"(v), "i"(OFF) : "memory");
    }
}
template <int J>
__device__ __forceinline__ void grp_store_rows(const gvec (&X)[16], bool valid, uint32_t y0, uint32_t lim, uint64_t P) {
    if constexpr (J < 16) {
        grp_store_if<256 * J>(valid && y0 + 256u * J < lim, X[J], P);
        grp_store_rows<J + 1>(X, valid, y0, lim, P);
    }
}
__device__ __forceinline__ void grp_store1_if(bool c, uint32_t v, uint64_t addr) {
    const uint64_t m = __ballot(c);
    uint64_t sv;
    asm volatile("s_and_saveexec_b64 %0, %1\n\tglobal_store_dword %2, %3, off\n\ts_mov_b64 exec, %0"
                 : "=&s"(sv) : "s"(m), "v"(addr), "v"(v) : "memory");
}
__device__ __forceinline__ uint32_t grp_bperm(uint32_t src_lane, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

__global__ __launch_bounds__(64 * kGrpWaves) void log_group_kernel(LogLaunch a) {
    __shared__ uint32_t tab[kLdsBytes / 4];
    constexpr int WV = kGrpWaves;
    constexpr int G = kGrpG;
    const uint32_t Hall = *a.head_count;
    const uint32_t hb0 = (uint32_t)((uint64_t)Hall * blockIdx.x / gridDim.x);
    const uint32_t hb1 = (uint32_t)((uint64_t)Hall * (blockIdx.x + 1) / gridDim.x);
    if (hb0 < hb1) {
        fill_lds<64 * WV>(tab, static_cast<const uint4*>(a.image));
        const uint32_t lane = threadIdx.x & 63u;
        const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const uint32_t g = lane / kGrpLP, i = lane % kGrpLP;
        const uint32_t c0 = lane << 2 & 0x7Cu, c1 = c0 | 0x10000u;
        // final-map column order per lane: the 32 lanes of a bank group read 32
        // distinct columns mod 32
        const uint32_t rot = G == 4 ? ((g + 2u * (i >> 3)) & 3u) : ((i >> 4) & 1u);
        uint32_t cfq[G];
#pragma unroll
        for (int k = 0; k < G; k++) cfq[k] = kFinBase + 4u * ((uint32_t)G * i + ((k + rot) & (G - 1)));
        // heads cut among the workgroup's waves by SIMD age
        constexpr uint32_t kAges = WV / 4;
        auto weight = [&](uint32_t u) -> uint32_t {
            const uint32_t age = u / 4;
            return 100u - (kAges > 1 ? (24u * age) / (kAges - 1) : 0u);
        };
        auto wprefix = [&](uint32_t t) {
            uint32_t q = 0;
            for (uint32_t u = 0; u < t; u++) q += weight(u);
            return q;
        };
        const uint32_t Hb = hb1 - hb0, wsum = wprefix(WV);
        const uint32_t first = hb0 + (uint32_t)((uint64_t)Hb * wprefix(wave) / wsum);
        const uint32_t H = hb0 + (uint32_t)((uint64_t)Hb * wprefix(wave + 1) / wsum);
        const uint64_t pool = (uint64_t)(uintptr_t)a.pool;
        const uint64_t dummy = (uint64_t)(uintptr_t)a.image + 4096ull * ((blockIdx.x * WV + wave) % (kLdsBytes / 4096));
        for (uint32_t base = first; base < H; base += 64u) {
            const uint32_t ih = base + lane;
            const bool hv = ih < H;
            const uint32_t hslot = a.heads[hv ? ih : base];
            const unsigned long long ent = reinterpret_cast<const unsigned long long*>(a.table)[hslot];
            if (a.done && hv) a.table[hslot] = 0ull;
            const uint32_t key = (uint32_t)(ent >> 32) - 1u;
            const uint32_t pfirst = (uint32_t)ent - 1u;
            const uint32_t nxt = a.next[pfirst];
            const uint32_t u0 = pfirst / a.slots;
            const UpdateDesc d = a.upd[u0];
            const Piece hp = piece_in_page((uint64_t)key * 4096u, 4096u, d.dst, d.src, d.len, a.src);
            const uint32_t hrr = hp.rlo | hp.rhi << 16;
            const uint64_t hsp = (uint64_t)(uintptr_t)hp.sp;
            const uint32_t cnt = (uint32_t)__popcll(__ballot(hv));
            const uint64_t singles = __ballot(hv && nxt == kNoPiece);
            const uint64_t multis = __ballot(hv && nxt != kNoPiece);
            const uint32_t nq = (cnt + G - 1) / G;

            auto issue = [&](GrpSet& Y, uint32_t t) {
                __builtin_amdgcn_sched_barrier(0);
                const bool live = t < nq;
                const uint32_t h = (G * t + g) & 63u;
                Y.pg = live ? grp_bperm(h, key) : 0u;
                Y.rr = live ? grp_bperm(h, hrr) : 0u;
                Y.sp = live ? (uint64_t)grp_bperm(h, (uint32_t)hsp) | (uint64_t)grp_bperm(h, (uint32_t)(hsp >> 32)) << 32
                            : dummy;
                Y.valid = live && ((singles >> h) & 1ull);
                const GrpGeo q = grp_geo(Y.rr);
                const uint64_t P = (live ? pool + (uint64_t)Y.pg * 4096u : dummy) + kGrpCB * i;
                const uint64_t S = Y.sp + kGrpCB * i;
                const uint32_t len = q.rhi - q.rlo, lw = len >= kGrpCB ? len - (kGrpCB - 1u) : 0u;
                const uint32_t x0 = kGrpCB * i - q.rlo;
#pragma unroll
                for (int j = 0; j < 16; j++) {
                    uint64_t b = x0 + 256u * j < lw ? S : P;
                    asm("" : "+v"(b));
                    Y.X[j] = __builtin_nontemporal_load(reinterpret_cast<const ggvec*>(b) + (256 / kGrpCB) * j);
                }
                const uint64_t safe = (Y.sp + q.rlo) & ~(uint64_t)(kGrpCB - 1u);
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const uint64_t sc = Y.sp + q.ce[e];
                    const uint32_t sh = (uint32_t)sc & (kGrpCB - 1u);
                    const uint64_t B = sc - sh;
#pragma unroll
                    for (int m = 0; m < 2; m++) {
                        const int32_t lo = (int32_t)kGrpCB * m - (int32_t)sh;
                        const bool need = q.ex[e] && lo + (int32_t)kGrpCB > (int32_t)q.pa[e] && lo < (int32_t)q.pz[e];
                        uint64_t ad = need ? B + kGrpCB * m : safe;
                        Y.D[e][m] = *reinterpret_cast<const ggvec*>(ad);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
            };
            auto compute = [&](GrpSet& Y) {
                const GrpGeo q = grp_geo(Y.rr);
#pragma unroll
                for (int e = 0; e < 2; e++) {
                    const uint32_t sh = ((uint32_t)Y.sp + q.ce[e]) & (kGrpCB - 1u);
                    const bool own = q.ex[e] && ((q.ce[e] / kGrpCB) & (kGrpLP - 1u)) == i;
                    const uint32_t row = own ? q.ce[e] >> 8 : 0xFFu;
                    uint32_t F[2 * G];
#pragma unroll
                    for (int k = 0; k < G; k++) {
                        F[k] = Y.D[e][0][k];
                        F[G + k] = Y.D[e][1][k];
                    }
                    // shift down by sh >> 2 dwords (select stages on its bits), then sh & 3 bytes
                    const uint32_t s4 = 0u - ((sh >> 2) & 1u);
                    uint32_t F1[2 * G - 1];
#pragma unroll
                    for (int m = 0; m < 2 * G - 1; m++) F1[m] = (F[m + 1] & s4) | (F[m] & ~s4);
                    uint32_t F2[G + 1];
                    if constexpr (G == 4) {
                        const uint32_t s8 = 0u - ((sh >> 3) & 1u);
#pragma unroll
                        for (int m = 0; m < G + 1; m++) F2[m] = (F1[m + 2] & s8) | (F1[m] & ~s8);
                    } else {
#pragma unroll
                        for (int m = 0; m < G + 1; m++) F2[m] = F1[m];
                    }
                    uint32_t v[G], mk[G];
#pragma unroll
                    for (int k = 0; k < G; k++) {
                        v[k] = __builtin_amdgcn_alignbyte(F2[k + 1], F2[k], sh & 3u);
                        mk[k] = grp_dword_mask(q.pa[e], q.pz[e], k);
                    }
#pragma unroll
                    for (int j = 0; j < 16; j++) {
                        const bool at = row == (uint32_t)j;
#pragma unroll
                        for (int k = 0; k < G; k++) {
                            const uint32_t m = at ? mk[k] : 0u;
                            Y.X[j][k] = (v[k] & m) | (Y.X[j][k] & ~m);
                        }
                    }
                }
                const uint64_t P = pool + (uint64_t)Y.pg * 4096u + kGrpCB * i;
                const uint32_t len = q.rhi - q.rlo;
                const uint32_t y0 = kGrpCB * i + (kGrpCB - 1u) - q.rlo;
                grp_store_rows<0>(Y.X, Y.valid, y0, len + (kGrpCB - 1u), P);
                uint32_t sv[G];
#pragma unroll
                for (int k = 0; k < G; k++) sv[k] = Y.X[0][k];
#pragma unroll
                for (int j = 1; j < 16; j++)
#pragma unroll
                    for (int k = 0; k < G; k++) sv[k] = apply_g_xor(tab, sv[k], Y.X[j][k], c0, c1);
                // rotate the states by rot, then chain k' reads column G i + ((k' + rot) & (G-1))
                uint32_t sr[G];
                if constexpr (G == 4) {
                    const uint32_t rot1 = 0u - (rot & 1u), rot2 = 0u - ((rot >> 1) & 1u);
                    uint32_t s1[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) s1[k] = (sv[(k + 1) & 3] & rot1) | (sv[k] & ~rot1);
#pragma unroll
                    for (int k = 0; k < 4; k++) sr[k] = (s1[(k + 2) & 3] & rot2) | (s1[k] & ~rot2);
                } else {
                    const uint32_t rot1 = 0u - (rot & 1u);
                    sr[0] = (sv[1] & rot1) | (sv[0] & ~rot1);
                    sr[1] = (sv[0] & rot1) | (sv[1] & ~rot1);
                }
                uint32_t r = 0;
#pragma unroll
                for (int k = 0; k < G; k++) r ^= apply_fin(tab, sr[k], cfq[k]);
                r ^= __builtin_amdgcn_mov_dpp(r, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
                r ^= __builtin_amdgcn_mov_dpp(r, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
                r ^= __builtin_amdgcn_mov_dpp(r, 0x124, 0xF, 0xF, false);  // row_ror:4
                r ^= __builtin_amdgcn_mov_dpp(r, 0x128, 0xF, 0xF, false);  // row_ror:8
                uint32_t storer;  // the lane holding the page's total
                if constexpr (G == 2) {
                    // rows 1 and 3 add their lower neighbour row (row_bcast:15)
                    r ^= __builtin_amdgcn_update_dpp(0u, r, 0x142, 0xA, 0xF, false);
                    storer = 32u * g + 16u;
                } else {
                    storer = 16u * g;
                }
                grp_store1_if(Y.valid && lane == storer, r ^ a.kconst, (uint64_t)(uintptr_t)(a.page_crcs + Y.pg));
            };
            GrpSet SA, SB;
            issue(SA, 0);
            issue(SB, 1);
            for (uint32_t t = 0; t < nq; t += 2) {
                compute(SA);
                issue(SA, t + 2);
                if (t + 1 < nq) compute(SB);
                issue(SB, t + 3);
            }
            for (uint64_t m = multis; m; m &= m - 1) {
                const uint32_t h = (uint32_t)__builtin_ctzll(m);
                log_page_multi<16, false>(a, tab, __builtin_amdgcn_readlane(key, h), __builtin_amdgcn_readlane(u0, h),
                                          __builtin_amdgcn_readlane(nxt, h), lane);
            }
        }
    }
    if (a.done) {
        __syncthreads();
        if (threadIdx.x == 0 && atomicAdd(a.done, 1u) == gridDim.x - 1) {
            atomicExch(a.head_count, 0u);
            atomicExch(a.done, 0u);
        }
    }
}

'''
KERNEL = KERNEL.replace("@G@", str(G)).replace("@WV@", str(WV)).replace("@MULTI@", multi or "")
anchor = "// A small log (<= 64 writes of <= one page each: at most 2 pieces a write) in"
assert anchor in s
s = s.replace(anchor, KERNEL + anchor, 1)
old = """    switch (a.page_bytes / kWaveBytes) {
        CC_GCASE(1)"""
assert old in s
s = s.replace(old, """    if (a.page_bytes == 4096 && !a.delta) {
        hipLaunchKernelGGL(log_group_kernel, dim3(a.blocks), dim3(64 * kGrpWaves), 0, s, a);
        return hipGetLastError();
    }
""" + old, 1)
open(p, "w").write(s)
