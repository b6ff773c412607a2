// curve_amd/csrc/kernels.hip -- hand-written gfx950 (CDNA4) kernels for the
// per-page CRC32C hot path.  Bandwidth-bound integer GF(2) work: no MFMA.
//
// Page kernel (one wavefront per page, grid-stride over pages)
// ------------------------------------------------------------
// A page of P = 256*M bytes is M steps of one coalesced 256-byte wave load:
// lane l holds dwords w[l + 64 j], j = 0..M-1.  In the raw (zero-init) CRC
// domain the page register is XOR_i F^(n-i)(w_i), F = "multiply by x^32 mod P"
// (feeding one dword).  Lane l runs a Horner chain with the 256-byte jump
// G = F^64:   s = w[l]; s = G(s) ^ w[l + 64 j]   (j = 1..M-1)
// which leaves s = XOR_j F^(64(M-1-j)) w_j, so lane l's share of the page
// register is F^(64-l)(s) -- independent of M.  The wave XOR-reduces the 64
// shares and adds the length constant K(P) = ~shift(~0, P) to get V(page).
//
// G is applied with 4 byte lookups per dword from LDS tables replicated 32x
// so that lane l always reads bank (l mod 32): every ds_read_b32 is
// conflict-free (2 LDS cycles per wave instruction).  The address of a lookup
// is ONE v_perm_b32 that splices {lane slot, state byte k, region} into a
// dword; the lookups are XORed with v_bitop3_b32.  F^(64-l) is lane-specific: 8 nibble lookups into per-lane tables
// (bank = lane mod 32 again).  Layout: DESIGN.md "LDS image".
//
// Reference being replaced: the CRC32(buf, size) loop of the scan hasher
// (src/chunkserver/op_request.cpp:794, :847) and of the chunk/copyset hashers
// (src/chunkserver/datastore/chunkserver_chunkfile.cpp:805,
// src/chunkserver/copyset_node.cpp:964), all of which call
// curve::common::CRC32 (src/common/crc32.h:40-55).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <type_traits>
#include <stdint.h>

#include "kernels.h"

namespace cc {
namespace {

constexpr uint32_t kPolyDev = 0x82F63B78u;

__device__ __forceinline__ uint32_t lds_u32(const uint32_t* tab, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(tab) + byte_addr);
}

// One step of a lane's Horner chain: G(s) ^ w, G = x^(32*64) mod P.
// c0 = lane slot (region 0), c1 = lane slot | region 1 (bit 16).  v_perm_b32
// selector bytes: [0] = c.byte0 (lane*4), [1] = s.byte_k, [2] = c.byte2
// (region), [3] = 0x00.  The 4 lookups and w are XORed by two v_bitop3_b32
// (truth table 0x96 = 3-input XOR; gfx950 has no v_xor3): 6 VALU per step
// instead of 8 measured +3 % on the page kernel.
__device__ __forceinline__ uint32_t apply_g_xor(const uint32_t* tab, uint32_t s, uint32_t w, uint32_t c0,
                                                uint32_t c1) {
    const uint32_t a0 = __builtin_amdgcn_perm(c0, s, 0x0C060004u);
    const uint32_t a1 = __builtin_amdgcn_perm(c0, s, 0x0C060104u);
    const uint32_t a2 = __builtin_amdgcn_perm(c1, s, 0x0C060204u);
    const uint32_t a3 = __builtin_amdgcn_perm(c1, s, 0x0C060304u);
    const uint32_t t0 = lds_u32(tab, a0);
    const uint32_t t1 = lds_u32(tab, a1 + 128u);
    const uint32_t t2 = lds_u32(tab, a2);
    const uint32_t t3 = lds_u32(tab, a3 + 128u);
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(t0, t1, t2, 0x96), t3, w, 0x96);
}

// Lane-specific final shift F^(64-l) via 8 nibble lookups.  cf = kFinBase + 4*lane.
__device__ __forceinline__ uint32_t apply_fin(const uint32_t* tab, uint32_t s, uint32_t cf) {
    uint32_t r = 0;
#pragma unroll
    for (int n = 0; n < 8; n++) {
        const uint32_t v = (s >> (4 * n)) & 15u;
        r ^= lds_u32(tab, ((v << 8) | cf) + 4096u * n);
    }
    return r;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, uint32_t l) {
    // readlane returns int: go through uint32_t so the low half is not sign-extended
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), l) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)v, l);
}

// XOR over the 64 lanes, result wave-uniform (SGPR).
__device__ __forceinline__ uint32_t wave_xor(uint32_t r) {
    r ^= __builtin_amdgcn_mov_dpp(r, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    r ^= __builtin_amdgcn_mov_dpp(r, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    r ^= __builtin_amdgcn_mov_dpp(r, 0x124, 0xF, 0xF, false);  // row_ror:4
    r ^= __builtin_amdgcn_mov_dpp(r, 0x128, 0xF, 0xF, false);  // row_ror:8
    return __builtin_amdgcn_readlane(r, 0) ^ __builtin_amdgcn_readlane(r, 16) ^
           __builtin_amdgcn_readlane(r, 32) ^ __builtin_amdgcn_readlane(r, 48);
}

template <int THREADS = kBlockThreads>
__device__ __forceinline__ void fill_lds(uint32_t* tab, const uint4* __restrict__ image) {
    uint4* t4 = reinterpret_cast<uint4*>(tab);
#pragma unroll 2
    for (uint32_t i = threadIdx.x; i < kLdsBytes / 16; i += THREADS) t4[i] = image[i];
    __syncthreads();
}

template <int M>
__device__ __forceinline__ void load_page(uint32_t (&w)[M], const uint32_t* __restrict__ p) {
#pragma unroll
    for (int j = 0; j < M; j++)
        w[j] = __builtin_nontemporal_load(p + 64 * j);  // read-once stream: nt (probe: +12 % read BW)
    // keep the whole page's loads ahead of the chain that follows (the
    // machine scheduler otherwise sinks them into it, shrinking the prefetch)
    __builtin_amdgcn_sched_barrier(0);
}

template <int M>
__device__ __forceinline__ uint32_t chain(const uint32_t* tab, const uint32_t (&w)[M], uint32_t c0, uint32_t c1) {
    uint32_t s = w[0];
#pragma unroll
    for (int j = 1; j < M; j++) s = apply_g_xor(tab, s, w[j], c0, c1);
    return s;
}

template <int MODE>
__device__ __forceinline__ void emit(uint32_t crc, uint64_t page, uint32_t lane, uint32_t* __restrict__ out,
                                     const uint32_t* __restrict__ expected, const VerifySink& vs) {
    if (MODE == 0) {
        if (lane == 0) out[page] = crc;
    } else {
        const uint32_t want = expected[page];
        if (crc != want && lane == 0) {
            const unsigned long long at = atomicAdd(vs.bad_count, 1ull);
            atomicMin(vs.first_bad, (unsigned long long)page);
            if (vs.list && at < vs.max_list) vs.list[at] = page;
        }
    }
}

// Tile of 64 consecutive pages per wave: the page CRCs are gathered into one
// register (lane k <- page k of the tile) and leave as ONE coalesced 256-byte
// store (compute) or are compared against ONE 256-byte load of expected CRCs
// with a ballot (verify).  Sparse 4-byte single-lane stores cost ~10 % of HBM
// efficiency in the first version.
template <int MODE>
__device__ __forceinline__ void flush_tile(uint32_t acc, uint64_t tile_first, uint32_t cnt, uint32_t lane,
                                           uint32_t* __restrict__ out, const uint32_t* __restrict__ expected,
                                           const VerifySink& vs) {
    if (MODE != 1) {  // compute (0; 3 = the metapage pass) and the load-only probe (2) store the tile
        // nt: the CRC stream must not interleave cached partial-line writes with
        // the 16 GiB nt read stream (plain stores cost 3 % of HBM throughput)
        if (lane < cnt) __builtin_nontemporal_store(acc, out + tile_first + lane);
    } else {
        const uint32_t want = lane < cnt ? __builtin_nontemporal_load(expected + tile_first + lane) : acc;
        const uint64_t bad = __ballot(want != acc);
        if (bad) {  // rare: wave-uniform branch
            unsigned long long at = 0;
            if (lane == 0) {
                at = atomicAdd(vs.bad_count, (unsigned long long)__popcll(bad));
                atomicMin(vs.first_bad, (unsigned long long)(tile_first + __ffsll((long long)bad) - 1));
            }
            if (vs.list) {  // every bad page of the tile gets a slot after `at`
                at = (unsigned long long)__shfl((long long)at, 0);
                const unsigned long long idx = at + (unsigned long long)__popcll(bad & ((1ull << lane) - 1ull));
                if (((bad >> lane) & 1ull) && idx < vs.max_list) vs.list[idx] = tile_first + lane;
            }
        }
    }
}

constexpr int kPrefetch = 2;  // wave steps in flight ahead of the one being hashed (2..4 measured equal)

// Page sequence of one wave: its k-th page is wfirst + (k >> ts) * wstride + (k & tmask),
// strictly increasing in k.
struct Walk {
    uint64_t wfirst, wstride;
    uint32_t tshift, tmask;
    __device__ __forceinline__ uint64_t page(uint64_t k) const {
        return wfirst + (k >> tshift) * wstride + (k & tmask);
    }
};

constexpr int kPair = 1;  // pages hashed together per wave step (2 measured equal)

template <int M, int P>
__device__ __forceinline__ void load_pages(uint32_t (&w)[P][M], const uint32_t* __restrict__ base, const Walk& W,
                                           uint64_t k, uint64_t last) {
#pragma unroll
    for (int q = 0; q < P; q++) {
        const uint64_t pg = W.page(k + q);
        load_page<M>(w[q], base + (pg < last ? pg : last) * (64u * M));
    }
}

// P independent Horner chains, interleaved step by step so each wave keeps
// 4*P LDS lookups in flight instead of 4.
// LOADS_ONLY: the chain replaced by a rotate-XOR that keeps every loaded word
// live (the load-only probe, MODE 2: the kernel's own schedule and traffic
// without the CRC arithmetic)
template <int M, int P, bool LOADS_ONLY = false>
__device__ __forceinline__ void chains(const uint32_t* tab, const uint32_t (&w)[P][M], uint32_t c0, uint32_t c1,
                                       uint32_t (&s)[P]) {
#pragma unroll
    for (int q = 0; q < P; q++) s[q] = w[q][0];
#pragma unroll
    for (int j = 1; j < M; j++) {
#pragma unroll
        for (int q = 0; q < P; q++) {
            if (LOADS_ONLY)
                s[q] = ((s[q] << 1) | (s[q] >> 31)) ^ w[q][j];
            else
                s[q] = apply_g_xor(tab, s[q], w[q][j], c0, c1);
        }
    }
}

// MODE 0: compute CRCs into out[]; MODE 1: verify against expected[].
// Wave w walks tiles w, w+W, w+2W, ... (W = waves in the grid) of 2^ts pages,
// P pages per step.  kPrefetch+1 register buffers rotate so kPrefetch
// steps' loads are in flight while the current step is hashed.  Loads are
// unconditional (index clamped to the item's last page) so hipcc counts vmcnt
// exactly.
// Dynamic tail (dyn_ctr != null): the strided walk covers tiles [0, static_tiles)
// only; the remaining tiles are handed out kPageDynPages pages at a time through
// the atomic counter *dyn_ctr (zeroed by the caller) to whichever waves finish
// first.  Per-wave rates differ by XCD (a kernel trace shows odd XCDs ~10 %
// slower on the same work), so a purely static split waits for the slowest.
constexpr uint64_t kPageDynPages = 64;  // pages per dynamic chunk (A/B: 64 beats 128)
// Dynamic-tail heads (kernels.h kDynHeads): 1 = one counter for the whole grid;
// 8 = one per XCD (MI355X_MICROARCH.md "dequeue": one word saturates at ~88
// dequeues/us, shard above 64 pullers).  With 8 heads the tail's chunks are cut
// into 8 contiguous regions; a wave pulls from its own XCD's region
// (blockIdx.x % 8: workgroups go round-robin over the XCDs -- placement is
// speed only, never correctness) and, once that is drained, steals from the
// next regions in turn.
// Next chunk of a dynamic tail of n_chunks chunks, from kDynHeads counters
// kDynHeadStride words apart (zeroed before the launch).  With one head: a
// plain dequeue.  With 8: the chunks are cut into 8 contiguous regions, a wave
// pulls from its own XCD's region first (blockIdx.x % 8 -- workgroups go
// round-robin over the XCDs; placement is speed only, never correctness) and
// steals from the next regions once that is drained.  `head` / `tried` are the
// wave's (uniform) cursor, initialised by tail_cursor().  Returns n_chunks when
// every region is drained.  Lane 0 does the atomics.
template <uint32_t H = kDynHeads>
__device__ __forceinline__ void tail_cursor(uint32_t& head, uint32_t& tried) {
    head = blockIdx.x % H;
    tried = 0;
}
template <uint32_t H = kDynHeads>
__device__ __forceinline__ uint64_t tail_pull(unsigned long long* __restrict__ ctr, uint64_t n_chunks, uint32_t& head,
                                              uint32_t& tried, uint32_t lane) {
    static_assert(H >= 1 && H <= kDynHeads, "heads beyond the zeroed counters");
    if constexpr (H == 1) {
        unsigned long long c = 0;
        if (lane == 0) c = atomicAdd(ctr, 1ull);
        c = readlane64(c, 0);
        return c < n_chunks ? c : n_chunks;
    } else {
        const uint64_t per = (n_chunks + H - 1) / H;
        for (; tried < H; tried++, head = (head + 1) % H) {
            unsigned long long c = 0;
            if (lane == 0) c = atomicAdd(ctr + head * kDynHeadStride, 1ull);
            c = readlane64(c, 0);
            const uint64_t chunk = head * per + c;
            if (c < per && chunk < n_chunks) return chunk;
        }
        return n_chunks;
    }
}

struct ZeroRanges {
    uint32_t* p[2];
    uint64_t n[2];
    __device__ __forceinline__ void clear() const {
#pragma unroll
        for (int k = 0; k < 2; k++)
            for (uint64_t i = threadIdx.x; i < n[k]; i += blockDim.x) p[k][i] = 0u;
    }
};
// The dynamic tail's extras (PageLaunch::meta_pages / dyn_next): a second page
// array appended to the tail as chunks of its own, and the other slot set of
// the stream's tail block, which this launch zeroes for the stream's next one.
// (Round 3 reset the counters at the END: every wave added to an arrival word
// and the last one zeroed the heads -- 2,048 returning atomics on one word in
// the kernel's last microseconds, ~12 ns each when they queue.)
struct TailExtra {
    const uint32_t* pages;
    uint64_t n;
    uint32_t* out;
    unsigned long long* next;
};
__device__ __forceinline__ void tail_clear_next(const TailExtra& ex) {
    if (ex.next && blockIdx.x == 0 && threadIdx.x < kDynHeads) atomicExch(ex.next + threadIdx.x * kDynHeadStride, 0ull);
}

template <int M, int MODE>
__global__ __launch_bounds__(kBlockThreads) void page_crc_kernel(
    const uint32_t* __restrict__ pages, uint64_t n_pages, const uint4* __restrict__ image,
    uint32_t kconst, uint32_t* __restrict__ out, const uint32_t* __restrict__ expected, VerifySink vs,
    uint32_t tshift, unsigned long long* __restrict__ dyn_ctr, uint64_t static_tiles, ZeroRanges zr, TailExtra ex) {
    __shared__ uint32_t tab[kLdsBytes / 4];
    if (blockIdx.x == 0) zr.clear();
    tail_clear_next(ex);
    fill_lds(tab, image);

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t c0 = lane << 2 & 0x7Cu;
    const uint32_t c1 = c0 | 0x10000u;
    const uint32_t cf = kFinBase + (lane << 2);
    const uint32_t* base = pages + lane;
    uint32_t* dst = out;
    constexpr int D = kPrefetch;
    constexpr int P = (M <= 16) ? kPair : 1;  // register budget: P*(D+1)*M data VGPRs
    // item 0: the strided static walk over tiles [0, static_tiles); then dynamic chunks
    Walk W;
    W.tshift = tshift;
    W.tmask = (1u << tshift) - 1u;
    W.wstride = ((uint64_t)gridDim.x * kWavesPerBlock) << tshift;
    W.wfirst = ((uint64_t)blockIdx.x * kWavesPerBlock + wave) << tshift;
    uint64_t lim = dyn_ctr ? (static_tiles << tshift < n_pages ? static_tiles << tshift : n_pages) : n_pages;
    uint32_t dyn_head, dyn_tried;  // this XCD's tail region first
    tail_cursor(dyn_head, dyn_tried);
#pragma unroll 1
    for (;;) {
        if (W.wfirst < lim) {
            const uint64_t last = lim - 1;
            uint32_t acc = 0;
            // ring of D+1 register buffers; after full unrolling every index is a
            // compile-time constant, so the ring lives in VGPRs (no scratch)
            uint32_t ring[D + 1][P][M];
#pragma unroll
            for (int st = 0; st < D; st++) load_pages<M, P>(ring[st], base, W, (uint64_t)st * P, last);
            // Every step's loads are unconditional (clamped) and termination is tested
            // once per ring revolution: path-insensitive waitcnt dataflow then sees the
            // same D stages outstanding on every edge into a step and keeps each wait
            // at its exact count (a per-step early exit made hipcc over-wait a stage).
            for (uint64_t k = 0;; k += (uint64_t)(D + 1) * P) {
#pragma unroll
                for (int st = 0; st <= D; st++) {
                    const uint64_t kk = k + (uint64_t)st * P;
                    load_pages<M, P>(ring[(st + D) % (D + 1)], base, W, kk + (uint64_t)D * P, last);
                    uint32_t s[P];
                    chains<M, P, MODE == 2>(tab, ring[st], c0, c1, s);
#pragma unroll
                    for (int q = 0; q < P; q++) {
                        const uint64_t kq = kk + q;
                        const uint64_t pc = W.page(kq);
                        if (pc < lim) {
                            const uint64_t pn = W.page(kq + 1);
                            const uint32_t crc = MODE == 2 ? wave_xor(s[q]) : wave_xor(apply_fin(tab, s[q], cf)) ^ kconst;
                            const uint32_t slot = (uint32_t)(kq & W.tmask);
                            acc = lane == slot ? crc : acc;
                            if (slot == W.tmask || pn >= lim)
                                flush_tile<MODE>(acc, pc - slot, slot + 1u, lane, dst, expected, vs);
                        }
                    }
                }
                if (W.page(k + (uint64_t)(D + 1) * P) >= lim) break;
            }
        }
        if (!dyn_ctr) break;
        // next dynamic chunk: kPageDynPages consecutive pages of the fused
        // metapages (the first chunk indices: pulled early, so the tail's last
        // chunks stay data chunks that even out as before), then of the data
        const uint64_t tail0 = static_tiles << tshift;
        const uint64_t mchunks = (ex.n + kPageDynPages - 1) / kPageDynPages;
        const uint64_t chunks = mchunks + (n_pages - tail0 + kPageDynPages - 1) / kPageDynPages;
        const uint64_t chunk = tail_pull(dyn_ctr, chunks, dyn_head, dyn_tried, lane);
        if (chunk >= chunks) break;
        uint64_t p0, end;
        if (chunk >= mchunks) {
            base = pages + lane;
            dst = out;
            p0 = tail0 + (chunk - mchunks) * kPageDynPages;
            end = n_pages;
        } else {
            base = ex.pages + lane;
            dst = ex.out;
            p0 = chunk * kPageDynPages;
            end = ex.n;
        }
        W.wfirst = p0;
        W.wstride = 1ull << tshift;  // consecutive tiles: page(k) = p0 + k
        lim = p0 + kPageDynPages < end ? p0 + kPageDynPages : end;
    }
}

// Any M (page_bytes = 256*M): no register prefetch, dynamic chain length.
template <int MODE>
__global__ __launch_bounds__(kBlockThreads) void page_crc_kernel_dyn(
    const uint32_t* __restrict__ pages, uint64_t n_pages, uint32_t M, const uint4* __restrict__ image,
    uint32_t kconst, uint32_t* __restrict__ out, const uint32_t* __restrict__ expected, VerifySink vs,
    ZeroRanges zr) {
    __shared__ uint32_t tab[kLdsBytes / 4];
    if (blockIdx.x == 0) zr.clear();
    fill_lds(tab, image);

    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t stride = (uint64_t)gridDim.x * kWavesPerBlock;
    const uint32_t c0 = lane << 2 & 0x7Cu;
    const uint32_t c1 = c0 | 0x10000u;
    const uint32_t cf = kFinBase + (lane << 2);
    for (uint64_t page = (uint64_t)blockIdx.x * kWavesPerBlock + wave; page < n_pages; page += stride) {
        const uint32_t* p = pages + page * (64ull * M) + lane;
        uint32_t s = p[0];
        for (uint32_t j = 1; j < M; j++) s = apply_g_xor(tab, s, p[64ull * j], c0, c1);
        emit<MODE>(wave_xor(apply_fin(tab, s, cf)) ^ kconst, page, lane, out, expected, vs);
    }
}

// cache policy bits (aux) of the write log's buffer instructions: 2 = nontemporal.
// Row loads nt (A/B of 0-3 within 1 %); row stores nt (-20 us a batch); source
// loads default (nt measured 6 % slower).
constexpr int kLogRowAux = 2;
constexpr int kLogStoreAux = 2;
constexpr uint32_t kBufOOB = 0x80000000u;   // offset past num_records: load 0 / store dropped
constexpr uint32_t kBufFlags = 0x00020000u;  // buffer resource dword 3 for gfx9-family (CDNA)
// A per-row buffer offset is `sel + 256 j` with sel = (lane's dword wanted ?
// its offset : kBufOOB).  Left alone, the compiler folds the add into both arms
// of the select and keeps 2 x M loop-invariant row constants in VGPRs (32 at
// 4 KiB pages); with sel opaque the 256 j goes into the instruction's 12-bit
// offset field (kBufOOB + 256 j is still past num_records).
__device__ __forceinline__ uint32_t row_sel(uint32_t v) {
    asm("" : "+v"(v));
    return v;
}


// ---------------------------------------------------------------------------
// GF(2) helpers for the fold / shift kernels (tiny volume: 4 B per page).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mulmod_dev(uint32_t a, uint32_t b) {
    uint32_t prod = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) {
        prod ^= b & (0u - ((a >> (31 - i)) & 1u));
        b = (b >> 1) ^ (kPolyDev & (0u - (b & 1u)));
    }
    return prod;
}

struct X2k {
    uint32_t t[64];
};
__constant__ X2k c_x2k;  // x^(2^k) mod P, uploaded once per device by engine.hip

__device__ __forceinline__ uint32_t xpow_dev(uint64_t n) {
    uint32_t r = 0x80000000u;
    for (int k = 0; n; k++, n >>= 1)
        if (n & 1u) r = mulmod_dev(r, c_x2k.t[k]);
    return r;
}

// Compact forms for once-per-range code inside unrolled block loops (keeps
// the kernel's instruction footprint small; the unrolled ones are 6x larger).
__device__ __forceinline__ uint32_t mulmod_small(uint32_t a, uint32_t b) {
    uint32_t prod = 0;
#pragma unroll 4
    for (int i = 0; i < 32; i++) {
        prod ^= b & (0u - ((a >> (31 - i)) & 1u));
        b = (b >> 1) ^ (kPolyDev & (0u - (b & 1u)));
    }
    return prod;
}
__device__ __forceinline__ uint32_t xpow_wave_small(uint64_t n, uint32_t lane) {
    uint32_t f = ((n >> lane) & 1u) ? c_x2k.t[lane] : 0x80000000u;
#pragma unroll 1
    for (int t = 1; t < 64; t <<= 1) f = mulmod_small(f, __shfl_xor(f, t, 64));
    return f;
}

// Product over the wave of per-lane GF(2)[x]/P factors (lane k: x^(2^k) if bit k
// of n is set, else 1) = x^n mod P; result in every lane.
__device__ __forceinline__ uint32_t xpow_wave(uint64_t n, uint32_t lane) {
    uint32_t f = (lane < 64 && ((n >> lane) & 1u)) ? c_x2k.t[lane] : 0x80000000u;
#pragma unroll
    for (int t = 1; t < 64; t <<= 1) f = mulmod_dev(f, __shfl_xor(f, t, 64));
    return f;
}

// ---------------------------------------------------------------------------
// CRC32C of arbitrary byte ranges (WAL entries on replay, raw-file hashes).
// The range [off, off+len) is viewed as whole 256-byte rows starting at the
// row-aligned address a = off & ~255, bytes before off and at/after off+len
// masked to zero.  Leading zeros do not change a zero-init (raw) CRC, so the
// page-kernel chain yields raw(data' || 0^t) = x^(8t) raw(data'), t = pad after
// the range in its last 4 KiB block; multiplying by x^(-8t) removes the pad.  butil's
// init is folded into the data (len >= 4): for a reflected CRC, Value(M) =
// raw(M ^ (~0 || 0...)) ^ ~0, so the first four bytes of the range are XORed
// with 0xFF as they are loaded.  (len < 4: K(len) = ~shift(~0, len) instead.)
//
// Blocks are loaded as buffer loads with an out-of-range offset for rows past
// the range (no branches around them: exact vmcnt waits); the schedule is the
// flat block stream below (range_flat_kernel).
// ---------------------------------------------------------------------------
struct RangeGeo {
    uint64_t a;      // 256-byte-aligned start
    uint64_t lim;    // bytes from a to the range's end
    uint64_t len;
    uint32_t head;   // off - a
    uint32_t rows;   // 256-byte rows from a
    uint32_t nb;     // 4 KiB blocks from a
};
__device__ __forceinline__ RangeGeo range_geo(uint64_t off, uint64_t len) {
    RangeGeo g;
    g.a = off & ~255ull;  // row-aligned: a 256-byte row load touches 2 cache lines, not 3
    g.head = (uint32_t)(off - g.a);
    g.len = len;
    g.lim = len + g.head;
    g.rows = (uint32_t)((g.lim + 255) >> 8);
    g.nb = (g.rows + 15) >> 4;
    return g;
}

// Block k of range g (16 rows, lane l holds dwords l + 64j of the block) into
// w[0..15]; when k is the range's last block, w[16] of lane i < 32 =
// x^(-8t) * x^i, t = the zero pad after the range (the table behind the LDS
// image; one 128-byte load in flight with the block), so the pad is removed by
// a lane-parallel multiply (mul_xinv) instead of a 32-step serial one.
__device__ __forceinline__ void load_range_block(uint32_t (&w)[17], const unsigned char* buf, const RangeGeo& g,
                                                 uint32_t k, uint32_t lane, __amdgpu_buffer_rsrc_t xr,
                                                 bool live = true) {
    // the descriptor's record count ends the block at the range's last dword
    // (rounded up to 4 bytes: a dword that starts inside the range is in
    // bounds, the next one is not, whether the unit tests the dword's start or
    // its end), so rows past the range read 0 with no per-row select
    // (a stream position past the wave's last block -- `live` false -- loads nothing)
    const uint64_t rem = g.lim - ((uint64_t)k << 12);  // > 0 for every block of the range
    const uint32_t nr = !live ? 0u : rem >= 4096u ? 4096u : (((uint32_t)rem + 3u) & ~3u);
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(buf + g.a + ((uint64_t)k << 12)), 0, nr, kBufFlags);
#pragma unroll
    for (int j = 0; j < 16; j++) w[j] = __builtin_amdgcn_raw_buffer_load_b32(r, 4u * lane + 256u * j, 0, 2);
    const uint32_t xo = (live && k + 1 == g.nb) ? 128u * (uint32_t)(((uint64_t)g.nb << 12) - g.lim) + 4u * (lane & 31u)
                                                : kBufOOB;
    w[16] = __builtin_amdgcn_raw_buffer_load_b32(xr, xo, 0, 0);
}

// Zero the bytes outside the range (first / last dword) and fold butil's init
// into the first four bytes.  Block k; the row/lane tests are per-lane compares.
__device__ __forceinline__ void mask_range_block(uint32_t (&w)[17], const RangeGeo& g, uint32_t k, uint32_t lane) {
    const uint64_t last = g.lim - 1;  // byte offset (from a) of the range's last byte
    const uint32_t tail = (uint32_t)(g.lim & 3u);
    if (tail && k + 1 == g.nb) {  // uniform: only a range's last block has bytes after its end
        const uint32_t mhi = 0xFFFFFFFFu >> (8u * (4u - tail));
        const uint64_t lrow = last >> 8;
        uint32_t rl = lane == (uint32_t)((last >> 2) & 63u) ? (uint32_t)(lrow & 15u) : 0xFFFFu;
        asm volatile("" : "+v"(rl));
#pragma unroll
        for (int j = 0; j < 16; j++) w[j] = rl == (uint32_t)j ? w[j] & mhi : w[j];
    }
    if (k == 0) {  // uniform: row 0 holds the bytes before the range (head < 256) and its first 4
        const uint32_t hl = g.head >> 2, hb = g.head & 3u;
        const uint32_t lo = lane < hl ? 0u : (lane == hl ? 0xFFFFFFFFu << (8u * hb) : 0xFFFFFFFFu);
        uint32_t init = 0u, spill = 0u;  // butil's ~0 init over the range's first 4 bytes
        if (g.len >= 4) {
            const uint32_t rest = hb ? 0xFFFFFFFFu >> (8u * (4u - hb)) : 0u;  // bytes of it in the next dword
            init = lane == hl ? 0xFFFFFFFFu << (8u * hb) : (lane == hl + 1 ? rest : 0u);
            spill = (hl == 63u && lane == 0) ? rest : 0u;  // next dword is row 1, lane 0
        }
        w[0] = (w[0] & lo) ^ init;
        w[1] ^= spill;
    }
}

// ---------------------------------------------------------------------------
// Flat block schedule of a range batch (WAL replay, raw-file hashes), ONE
// launch.  The batch is one stream of 4 KiB blocks (range 0's blocks, then
// range 1's, ...), B blocks in all.  The first Bs = B - B/kDynDiv are dealt
// out statically: rounds * W equal pieces, wave w taking pieces w, w + W, ...
// whatever the range sizes.  The last B/kDynDiv blocks are kDynBlocks-block
// chunks handed out through an atomic counter to whichever waves finish first
// (per-wave rates differ by ~7 % -- some XCDs run slower -- so a purely static
// split waits for the slowest wave).
// Where a piece starts comes from kRangeTiles per-tile block counts, held in
// registers by every wave.  The launch computes them itself: wave g counts
// tiles g, g + W, ... and publishes each as one epoch-tagged word (a plain
// device-coherent store: the word carries its own data, so no fence); every
// wave then polls the words of the call's epoch while its workgroup's LDS
// fills.  No wave ever waits on another without a bound: a tile word still
// missing after kTileWaitTicks (a workgroup not resident -- CUs taken by other
// work) is counted by the waiting wave itself from the descriptors.
// A range cut by a piece or chunk boundary is hashed in segments: segment
// [kb, ke) of the range contributes raw(segment || 0-pad) * x^(8 * (lim -
// 4096*ke)) (x^(-8t) for the one that ends the range).  Segments meet in the
// range's accumulator pair acc[2r] (XOR of the contributions) / acc[2r+1]
// (blocks arrived): a segment XORs in, then adds its block count; the one
// whose count completes the range takes the XOR, stores out[r] and leaves the
// pair zero for the next call.  The tail's chunk counter alternates between
// two slots by epoch, each call zeroing the one the next call uses.  A range hashed whole by one wave is stored
// directly; an empty range (V = 0) by the wave that counts its tile.
// ---------------------------------------------------------------------------
constexpr uint64_t kTileWaitTicks = 10000;  // 100 us of s_memrealtime (100 MHz) before a wave counts a tile itself
constexpr uint32_t kEpochShift = 40;        // tile word: epoch << 40 | blocks

// Blocks of tile t (ranges [n t / T, n (t+1) / T)), uniform; zero_empty: store
// V = 0 for the tile's empty ranges.
__device__ __forceinline__ uint64_t range_tile_count(const RangeLaunch& a, uint32_t t, uint32_t lane, bool zero_empty) {
    const uint64_t lo = a.n * t / kRangeTiles, hi = a.n * (t + 1) / kRangeTiles;
    uint64_t sum = 0;
    for (uint64_t i = lo + lane; i < hi; i += 64) {
        const RangeDesc d = a.ranges[i];
        sum += d.len ? range_geo(d.off, d.len).nb : 0u;
        if (zero_empty && !d.len) a.out[i] = 0u;
    }
#pragma unroll
    for (int d = 32; d; d >>= 1) sum += __shfl_xor(sum, d, 64);
    return sum;
}

__device__ __forceinline__ uint64_t wave_scan_incl(uint64_t v, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v += o;
    }
    return v;
}

// Every tile count of this call into tb (lane l: tiles kTpl*l .. kTpl*l + kTpl-1):
// poll the epoch-tagged words (sc1 loads: a data-tagged granule needs no
// fence).  A tile whose word is still missing after kTileWaitTicks belongs to
// a workgroup that is not running (a kernel on another stream holds the CUs,
// or a CU mask): the waiting wave CLAIMS it -- one CAS of the word to this
// call's tag with kTileClaim set -- counts it with count(t) and publishes the
// count, so each missing tile is counted once, by the first wave to claim it,
// while the others keep polling (round 4 had every waiting wave count every
// missing tile itself: unbounded in practice when many workgroups wait).  The
// owner's own later store writes the same count.  No wave waits on another
// without a bound: every claimed tile is counted by a running wave.
constexpr uint64_t kTileClaim = 1ull << (kEpochShift - 1);  // tile word: claimed, count pending
template <int kTpl, typename Count>
__device__ __forceinline__ void wait_tiles(uint64_t (&tb)[kTpl], uint64_t* tiles, uint64_t tag, uint32_t lane,
                                           Count count) {
    constexpr uint64_t kCountMask = (1ull << kEpochShift) - 1;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t have = 0;  // bit j: tb[j] holds this call's count
    for (;;) {
#pragma unroll
        for (int j = 0; j < kTpl; j++) {
            const uint64_t v = __hip_atomic_load(tiles + kTpl * lane + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool ok = (v & ~kCountMask) == tag && !(v & kTileClaim);
            tb[j] = ok ? v & kCountMask : tb[j];
            have |= ok ? 1u << j : 0u;
        }
        if (!__ballot(have != (1u << kTpl) - 1u)) return;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTileWaitTicks) {
#pragma unroll
            for (int j = 0; j < kTpl; j++) {
                for (uint64_t m = __ballot(!((have >> j) & 1u)); m; m &= m - 1) {
                    const uint32_t l = (uint32_t)__builtin_ctzll(m);
                    const uint32_t t = kTpl * l + j;
                    uint32_t mine = 0;
                    if (lane == 0) {  // neither published nor claimed this call: claim it
                        const uint64_t cur = __hip_atomic_load(tiles + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        uint64_t exp = cur;
                        mine = (cur & ~kCountMask) != tag &&
                               __hip_atomic_compare_exchange_strong(tiles + t, &exp, tag | kTileClaim,
                                                                    __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (__builtin_amdgcn_readlane(mine, 0)) {
                        const uint64_t cnt = count(t);
                        if (lane == 0) __hip_atomic_store(tiles + t, tag | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        tb[j] = lane == l ? cnt : tb[j];
                        have |= lane == l ? 1u << j : 0u;
                    }
                }
            }
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// The tile holding unit u of the stream, and the units before it: lane tl's
// tiles (cum = inclusive prefix of the lanes' sums), then the first of them
// whose running count passes u.
struct TileHit {
    uint32_t tile;
    uint64_t before;
};
template <int kTpl>
__device__ __forceinline__ TileHit tile_of(uint64_t cum, const uint64_t (&tb)[kTpl], uint64_t u, uint32_t lane) {
    const uint32_t tl = (uint32_t)__builtin_ctzll(__ballot(cum > u));
    TileHit h;
    h.before = tl ? readlane64(cum, tl - 1) : 0;
    h.tile = kTpl * tl;
    bool found = false;
#pragma unroll
    for (int j = 0; j < kTpl; j++) {
        const uint64_t v = readlane64(tb[j], tl);
        if (!found) {
            if (h.before + v > u) {
                found = true;
                h.tile = kTpl * tl + j;
            } else {
                h.before += v;
            }
        }
    }
    return h;
}

constexpr int kFlatWaves = 8;  // waves per CU of the flat range kernel (A/B on WAL sizes: 8 beats 12 by ~4 %, 16 by ~10 %)
constexpr uint32_t kRangeRounds = 1;  // static pieces per wave (round 4, one launch: 1 beats 2 by 0.7 % on random and on equal sizes; 4 +4.7 %, 8 +10.6 %)
constexpr uint64_t kRangeDynDiv = 32;  // 1/32 of the blocks go to the dynamic tail (A/B: 1/8 and 1/16 lose to
                                       // the one counter's atomics, 1/64 leaves tail)
constexpr uint32_t kRangeHeads = 1;    // tail heads (A/B round 3: 8 per-XCD heads = one counter at 1/32)
constexpr uint64_t kRangeDynBlocks = 16;  // blocks per dynamic chunk (A/B: 8 slower, 16 = 32)
__global__ __launch_bounds__(64 * kFlatWaves) void range_flat_kernel(RangeLaunch a) {
    constexpr uint32_t rounds = kRangeRounds;
    __shared__ uint32_t tab[kLdsBytes / 4];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * kFlatWaves;
    const uint64_t w = (uint64_t)blockIdx.x * kFlatWaves + wave;
    const uint64_t tag = (uint64_t)a.epoch << kEpochShift;
    // this wave's tile counts, published before the LDS fill (which hides the
    // stores' and the other workgroups' latency)
    for (uint64_t t = w; t < kRangeTiles; t += W) {
        const uint64_t cnt = range_tile_count(a, (uint32_t)t, lane, true);
        if (lane == 0) __hip_atomic_store(a.tiles + t, tag | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    fill_lds<64 * kFlatWaves>(tab, static_cast<const uint4*>(a.image));
    const unsigned char* __restrict__ buf = a.buf;
    const RangeDesc* __restrict__ ranges = a.ranges;
    const uint64_t n = a.n;
    uint32_t* __restrict__ out = a.out;
    const uint32_t c0 = lane << 2 & 0x7Cu;
    const uint32_t c1 = c0 | 0x10000u;
    const uint32_t cf = kFinBase + (lane << 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint4*>(static_cast<const uint4*>(a.image)) + kLdsBytes / 16, 0, kXinvEntries * 128u, kBufFlags);

    // every tile count of this call: lane l holds tiles kTpl*l .. kTpl*l + kTpl-1,
    // cum = inclusive prefix of the lane sums
    constexpr int kTpl = kRangeTiles / 64;
    uint64_t tb[kTpl];
    wait_tiles<kTpl>(tb, a.tiles, tag, lane, [&](uint32_t t) { return range_tile_count(a, t, lane, false); });
    uint64_t lsum = 0;
#pragma unroll
    for (int j = 0; j < kTpl; j++) lsum += tb[j];
    const uint64_t cum = wave_scan_incl(lsum, lane);
    const uint64_t B = readlane64(cum, 63);
    const uint64_t Bs = kRangeDynDiv ? B - B / kRangeDynDiv : B;  // statically dealt blocks
    const uint64_t n_dyn = (B - Bs + kRangeDynBlocks - 1) / kRangeDynBlocks;
    // the tail's counter: slot epoch % 2 of the block; this call zeroes the
    // other slot for the stream's next call (nobody here touches it), so no
    // wave has to count arrivals at the end to reset it
    unsigned long long* dyn_ctr = a.tail + (a.epoch & 1u) * kDynCtrWords64;
    if (blockIdx.x == 0 && threadIdx.x < kRangeHeads)
        atomicExch(a.tail + ((a.epoch + 1u) & 1u) * kDynCtrWords64 + threadIdx.x * kDynHeadStride, 0ull);
    uint32_t dyn_head, dyn_tried;
    tail_cursor<kRangeHeads>(dyn_head, dyn_tried);

    // work items: static pieces item < rounds, then dynamic chunks until the counter runs out
#pragma unroll 1
    for (uint32_t item = 0;; item++) {
        uint64_t b0, b1;
        if (item < rounds) {
            const uint64_t RW = (uint64_t)rounds * W, c = (uint64_t)item * W + w;
            b0 = Bs * c / RW;
            b1 = Bs * (c + 1) / RW;
            if (b0 >= b1) continue;
        } else {
            const uint64_t c = tail_pull<kRangeHeads>(dyn_ctr, n_dyn, dyn_head, dyn_tried, lane);
            if (c >= n_dyn) break;
            b0 = Bs + c * kRangeDynBlocks;
            b1 = b0 + kRangeDynBlocks < B ? b0 + kRangeDynBlocks : B;
        }
        const TileHit th = tile_of(cum, tb, b0, lane);
        const uint32_t tile = th.tile;
        const uint64_t before = th.before;
        // range holding block b0: the tile's ranges 64 at a time
        uint64_t r = n * tile / kRangeTiles;
        uint64_t rel = b0 - before;
        uint32_t k0 = 0;
        // window of 64 descriptors (ranges wb + lane), refilled when passed; the
        // search's last 64 descriptors are the first window (no second load)
        uint64_t wb;
        RangeDesc wd;
        uint64_t wbits;  // lanes of the window holding a range with blocks
        for (;;) {
            const uint64_t ri = r + lane;
            wd = ranges[ri < n ? ri : n - 1];
            const uint64_t nbl = (ri < n && wd.len) ? range_geo(wd.off, wd.len).nb : 0u;
            const uint64_t c = wave_scan_incl(nbl, lane);
            const uint64_t tot = readlane64(c, 63);
            if (rel < tot) {
                const uint32_t h = (uint32_t)__builtin_ctzll(__ballot(c > rel));
                k0 = (uint32_t)(rel - (h ? readlane64(c, h - 1) : 0));
                wb = r;
                wbits = __ballot(ri < n && wd.len != 0);
                r += h;
                break;
            }
            rel -= tot;
            r += 64;
        }
        auto load_window = [&]() {
            const uint64_t ri = wb + lane;
            wd = ranges[ri < n ? ri : n - 1];
            wbits = __ballot(ri < n && wd.len != 0);
        };
        uint64_t left = b1 - b0;  // blocks not yet issued
        struct Pos {
            RangeGeo g;
            uint64_t r;              // range index
            uint32_t k;              // block of the range
            bool real, first, last;  // issued block / first and last block of the item
        };
        auto at = [&](uint64_t ri, uint32_t k) -> Pos {
            Pos p;
            const uint32_t h = (uint32_t)(ri - wb);
            p.g = range_geo(readlane64(wd.off, h), readlane64(wd.len, h));
            p.r = ri;
            p.k = k;
            p.real = true;
            p.first = false;
            p.last = --left == 0;
            return p;
        };
        auto adv = [&](const Pos& p) -> Pos {
            if (!p.real || p.last) {
                Pos q = p;
                q.real = false;
                q.first = q.last = false;
                return q;
            }
            if (p.k + 1 < p.g.nb) {
                Pos q = p;
                q.k = p.k + 1;
                q.first = false;
                q.last = --left == 0;
                return q;
            }
            uint32_t h = (uint32_t)(p.r - wb);
            uint64_t nx = h < 63 ? (wbits & (~0ull << (h + 1))) : 0ull;
            while (!nx) {  // window passed (rare): the next 64 descriptors
                wb += 64;
                load_window();
                nx = wbits;
            }
            return at(wb + (uint64_t)__builtin_ctzll(nx), 0);
        };
        // ring of 4 blocks: three blocks of loads in flight behind the one being folded
        uint32_t A[17], B4[17], Cq[17], Dq[17];
        Pos pA = at(r, k0);
        pA.first = true;
        load_range_block(A, buf, pA.g, pA.k, lane, xr);
        Pos pB = adv(pA);
        load_range_block(B4, buf, pB.g, pB.k, lane, xr, pB.real);
        Pos pC = adv(pB);
        load_range_block(Cq, buf, pC.g, pC.k, lane, xr, pC.real);
        Pos pD = pC;
        uint32_t s = 0;
        uint32_t segk = 0;  // block of the range the current segment began at
        // split-range segments of this item (at most its first and its last):
        // their accumulator atomics return values, and waiting on a returning
        // atomic waits for every load issued before it -- so they run after
        // the ring, when nothing is in flight (inside it: +1.8 % a batch)
        uint64_t seg_r0 = 0, seg_r1 = 0;
        uint32_t seg_v0 = 0, seg_v1 = 0, seg_n0 = 0, seg_n1 = 0, seg_nb0 = 0, seg_nb1 = 0, nseg = 0;
        auto step = [&](uint32_t (&X)[17], const Pos& px, uint32_t (&Y)[17], const Pos& py) {
            load_range_block(Y, buf, py.g, py.k, lane, xr, py.real);
            const RangeGeo& gx = px.g;
            const uint32_t kx = px.k;
            mask_range_block(X, gx, kx, lane);
            const bool start = kx == 0 || px.first;
            if (start) segk = kx;
            s = start ? X[0] : apply_g_xor(tab, s, X[0], c0, c1);
#pragma unroll
            for (int j = 1; j < 16; j++) s = apply_g_xor(tab, s, X[j], c0, c1);
            const bool end = kx + 1 == gx.nb;
            if (end || px.last) {
                const uint32_t raw_pad = wave_xor(apply_fin(tab, s, cf));
                // the item ends inside the range: shift over the range's bytes
                // after this block; a range of < 4 bytes: its K(len) (no folded init)
                const bool pw_needed = !end || gx.len < 4;
                const uint32_t pw =
                    pw_needed ? xpow_wave_small(end ? gx.len << 3 : (gx.lim - ((uint64_t)(kx + 1) << 12)) << 3, lane)
                              : 0u;
                // x^(-8t) * raw_pad = XOR over i of bit (31 - i) of raw_pad ? x^(-8t) x^i : 0
                const uint32_t bit = lane < 32u ? (raw_pad >> (31u - lane)) & 1u : 0u;
                uint32_t v = end ? wave_xor(bit ? X[16] : 0u) : mulmod_small(pw, raw_pad);
                if (end) v ^= gx.len >= 4 ? 0xFFFFFFFFu : ~mulmod_small(pw, 0xFFFFFFFFu);
                if (end && segk == 0) {
                    if (lane == 0) out[px.r] = v;
                } else {  // a segment of a split range: the item's first and/or last, met after the ring
                    // (selects, not an index: a dynamically indexed array lives in scratch)
                    const bool second = nseg != 0;
                    seg_r1 = second ? px.r : seg_r1;
                    seg_v1 = second ? v : seg_v1;
                    seg_n1 = second ? kx + 1 - segk : seg_n1;
                    seg_nb1 = second ? gx.nb : seg_nb1;
                    seg_r0 = second ? seg_r0 : px.r;
                    seg_v0 = second ? seg_v0 : v;
                    seg_n0 = second ? seg_n0 : kx + 1 - segk;
                    seg_nb0 = second ? seg_nb0 : gx.nb;
                    nseg++;
                }
            }
        };
        for (;;) {
            if (!pA.real) break;
            pD = adv(pC);
            step(A, pA, Dq, pD);
            if (!pB.real) break;
            pA = adv(pD);
            step(B4, pB, A, pA);
            if (!pC.real) break;
            pB = adv(pA);
            step(Cq, pC, B4, pB);
            if (!pD.real) break;
            pC = adv(pB);
            step(Dq, pD, Cq, pC);
        }
        // the item's split segments meet in their ranges' accumulator pairs:
        // XOR in, then add the blocks; the add that completes the range takes
        // the XOR, stores it and leaves the pair zero
        auto meet = [&](uint64_t r, uint32_t v, uint32_t nblk, uint32_t nb) {
            uint32_t* acc = a.acc + 2 * r;
            const uint32_t x = atomicXor(acc, v);
            asm volatile("" ::"v"(x) : "memory");  // the XOR is performed before the count says so
            if (atomicAdd(acc + 1, nblk) + nblk == nb) {
                out[r] = atomicExch(acc, 0u);
                atomicExch(acc + 1, 0u);
            }
        };
        if (lane == 0 && nseg > 0) meet(seg_r0, seg_v0, seg_n0, seg_nb0);
        if (lane == 0 && nseg > 1) meet(seg_r1, seg_v1, seg_n1, seg_nb1);
    }
}

// Fast path: per_group = 64*q.  One wave per group, grid-stride over groups;
// lane l folds units [l*q, (l+1)*q) by Horner with the constant multiplier
// m_unit applied through a 4 x 256-entry product table in LDS (4 lookups +
// 2 v_bitop3 instead of a 32-step multiply), then a 6-level shuffle tree merges
// lanes (one multiply per level).
__global__ __launch_bounds__(256) void fold_kernel_wave(const uint32_t* __restrict__ crcs, uint64_t n_groups,
                                                        uint32_t per_group, FoldLaunch a,
                                                        uint32_t* __restrict__ out) {
    __shared__ uint32_t mt[4][256];
    for (uint32_t i = threadIdx.x; i < 1024; i += 256) mt[i >> 8][i & 255] = mulmod_dev(a.m_unit, (i & 255u) << (8 * (i >> 8)));
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t q = per_group >> 6;
    for (uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g < n_groups; g += (uint64_t)gridDim.x * 4) {
        const uint32_t* p = crcs + g * per_group + (uint64_t)lane * q;
        uint32_t s = p[0];
        for (uint32_t i = 1; i < q; i++) {
            const uint32_t t = __builtin_amdgcn_bitop3_b32(mt[0][s & 255u], mt[1][(s >> 8) & 255u],
                                                           mt[2][(s >> 16) & 255u], 0x96);
            s = __builtin_amdgcn_bitop3_b32(t, mt[3][s >> 24], p[i], 0x96);
        }
#pragma unroll
        for (int t = 0; t < 6; t++) {
            const uint32_t other = __shfl_down(s, 1u << t, 64);
            if ((lane & ((2u << t) - 1u)) == 0) s = mulmod_dev(a.m_tree[t], s) ^ other;
        }
        if (lane == 0) out[g] = s;
    }
}

// ---------------------------------------------------------------------------
// Fused scan epilogue (one launch per batch instead of fold + fold + combine +
// digest): block b = chunk b, 256 threads.  Thread t loads its q page CRCs
// (coalesced), folds them by Horner through an LDS product table of
// x^(8*page_bytes), then a combine tree over threads (shuffles inside a wave,
// LDS across the 4 waves): after slice_shift levels thread (k << slice_shift)
// holds slice k's CRC (ScanMap.crc), after 8 levels thread 0 holds the chunk
// data CRC -> file CRC = combine(metapage CRC, data CRC, chunk_bytes) -> digest
// contribution atomicXor'ed into its copyset.
// ---------------------------------------------------------------------------
// multiply by a constant through its 4 x 256 product table (global, L1-resident)
__device__ __forceinline__ uint32_t mul_tab(const uint32_t* __restrict__ t, uint32_t s) {
    return __builtin_amdgcn_bitop3_b32(
        __builtin_amdgcn_bitop3_b32(t[s & 255u], t[256 + ((s >> 8) & 255u)], t[512 + ((s >> 16) & 255u)], 0x96),
        t[768 + (s >> 24)], 0u, 0x96);
}

__global__ __launch_bounds__(256) void epilogue_kernel(EpilogueLaunch a) {
    __shared__ uint32_t mt[1024];  // x^(8 page_bytes) product table (Horner), copied once per block
    __shared__ uint32_t part[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
    for (uint32_t i = t; i < 1024; i += 256) mt[i] = a.mtab[i];
    __syncthreads();
    const uint32_t slices = 256u >> a.slice_shift;
    const uint32_t* lvl = a.mtab + 1024;           // level k table at lvl + 1024 k
    const uint32_t* chk = a.mtab + 9 * 1024;
    for (uint64_t c = blockIdx.x; c < a.n_chunks; c += gridDim.x) {
        const uint32_t* p = a.page_crcs + c * a.pages_per_chunk + (uint64_t)t * a.q;
        auto horner = [&](uint32_t s, uint32_t w) {
            const uint32_t u = __builtin_amdgcn_bitop3_b32(mt[s & 255u], mt[256 + ((s >> 8) & 255u)],
                                                           mt[512 + ((s >> 16) & 255u)], 0x96);
            return __builtin_amdgcn_bitop3_b32(u, mt[768 + (s >> 24)], w, 0x96);
        };
        uint32_t s;
        if (a.q == 16 && ((uintptr_t)a.page_crcs & 15u) == 0) {
            // 16 MiB chunks of 4 KiB pages: the thread's 64 B in four 16-byte loads, all in flight
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = reinterpret_cast<const uint4*>(p)[k];
            s = v[0].x;
            s = horner(s, v[0].y);
            s = horner(s, v[0].z);
            s = horner(s, v[0].w);
#pragma unroll
            for (int k = 1; k < 4; k++) {
                s = horner(s, v[k].x);
                s = horner(s, v[k].y);
                s = horner(s, v[k].z);
                s = horner(s, v[k].w);
            }
        } else {
            s = p[0];
            for (uint32_t i = 1; i < a.q; i++) s = horner(s, p[i]);
        }
        if (a.slice_shift == 0) a.slice_crcs[c * 256 + t] = s;  // one thread per slice
        // levels 0..5 inside the wave
#pragma unroll
        for (uint32_t k = 0; k < 6; k++) {
            const uint32_t other = __shfl_down(s, 1u << k, 64);
            if ((lane & ((2u << k) - 1u)) == 0) s = mul_tab(lvl + 1024 * k, s) ^ other;
            if (k + 1 == a.slice_shift && (t & ((2u << k) - 1u)) == 0) a.slice_crcs[c * slices + (t >> a.slice_shift)] = s;
        }
        // levels 6..7 across the 4 waves
        if (lane == 0) part[wv] = s;
        __syncthreads();
        if (t == 0) {
            const uint32_t w0 = mul_tab(lvl + 6 * 1024, part[0]) ^ part[1];
            const uint32_t w1 = mul_tab(lvl + 6 * 1024, part[2]) ^ part[3];
            if (a.slice_shift == 7) {
                a.slice_crcs[c * 2] = w0;
                a.slice_crcs[c * 2 + 1] = w1;
            }
            const uint32_t data = mul_tab(lvl + 7 * 1024, w0) ^ w1;
            if (a.slice_shift == 8) a.slice_crcs[c] = data;
            const uint32_t file = mul_tab(chk, a.meta_crcs[c]) ^ data;
            if (a.file_crcs) a.file_crcs[c] = file;
            if (a.digest) atomicXor(a.digest + a.group[c], mulmod_dev(a.after_mult[c], file));
        }
        __syncthreads();
    }
}

__global__ void xpow8_kernel(const uint64_t* __restrict__ nbytes, uint64_t n, uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (uint64_t)gridDim.x * 4) {
        const uint32_t m = xpow_wave(nbytes[i] << 3, lane);
        if (lane == 0) out[i] = m;
    }
}

// Generic path: one thread per group, serial combine.
__global__ void fold_kernel_serial(const uint32_t* __restrict__ crcs, uint64_t n_groups, uint32_t per_group,
                                   uint32_t m_unit, uint32_t* __restrict__ out) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n_groups) return;
    const uint32_t* p = crcs + g * per_group;
    uint32_t s = per_group ? p[0] : 0u;
    for (uint32_t i = 1; i < per_group; i++) s = mulmod_dev(m_unit, s) ^ p[i];
    out[g] = s;
}

__global__ void shift_kernel(const uint32_t* __restrict__ crcs, const uint64_t* __restrict__ nbytes, uint64_t n,
                             uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = crcs[i];
    const uint64_t nb = nbytes[i];
    out[i] = (c == 0u || nb == 0u) ? c : mulmod_dev(xpow_dev(nb << 3), c);
}

// ---------------------------------------------------------------------------
// Write-log path (cc_apply_log_dev): ordering on the device, no host planning.
// ---------------------------------------------------------------------------
// Grouping by page without a sort.  Piece t = (update t / slots, its k-th page,
// k = t % slots).  Every piece inserts its page into an open-addressing table
// (linear probing, <= 12.5 % load: >= 8 x pieces, engine.hip) whose 64-bit entry holds {page + 1, piece + 1}
// of the page's most recently inserted piece: one CAS both claims the page and
// pushes the piece onto the page's list (next[piece] = the previous head).
// The piece that claims an empty entry appends the entry's slot to the head
// list (one atomic per wave).  The list order is arbitrary; the page kernel
// restores log order from the update indices.  An update that breaks the
// contract (len 0, len > max_len, beyond the pool) produces no pieces and is
// not applied at all (never half-applied).  The table and the counters were
// zeroed earlier on the stream.
__device__ __forceinline__ uint32_t page_hash(uint32_t page, uint32_t mask) {
    return (page * 2654435761u) & mask;  // Fibonacci hashing; sequential pages spread
}

// Piece t of the log (t >= n_pieces: none) into the table; its head record,
// if it claims a page, goes to the block's own segment (no global counter: a
// per-wave atomic on one counter serialised 2,048 waves, 26 of the kernel's 31
// us, and even one per block was a returning atomic on the critical path).
// Every thread of the block calls it; `wcount` = LDS scratch of blockDim/64 + 1
// words; `used` = the segment's records so far (uniform), advanced here.
// (A = LogLaunch for log_insert_kernel, LogInsert for the next batch's grouping
// inside log_pages_kernel: the same field names.)
template <class A>
__device__ __forceinline__ void insert_piece(const A& a, uint64_t t, uint32_t* wcount, uint32_t& used) {
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    bool fresh = false;
    uint32_t slot = 0;
    if (t < a.n_pieces) {
        const uint64_t i = t / a.slots;
        const uint32_t k = (uint32_t)(t - i * a.slots);
        const UpdateDesc d = a.upd[i];
        const bool ok = d.len >= 1 && d.len <= a.max_len && d.dst < a.pool_bytes && d.len <= a.pool_bytes - d.dst;
        const uint64_t p0 = ok ? d.dst / a.page_bytes : 0;
        const uint64_t p1 = ok ? (d.dst + d.len - 1) / a.page_bytes : 0;
        if (ok && p0 + k <= p1) {
            const uint32_t page = (uint32_t)(p0 + k);
            const unsigned long long tag = (unsigned long long)(page + 1u) << 32;
            unsigned long long* tab = reinterpret_cast<unsigned long long*>(a.table);
            slot = page_hash(page, a.table_mask);
            // CAS first (one atomic for a page seen first, the common case);
            // next[] is only read by later kernels, so it can follow the CAS
            unsigned long long cur = 0ull;
            for (;;) {
                const unsigned long long old = atomicCAS(tab + slot, cur, tag | (unsigned long long)(t + 1));
                if (old == cur) {  // claimed (cur == 0) or pushed onto the page's list
                    a.next[t] = cur ? (uint32_t)cur - 1u : kNoPiece;
                    fresh = cur == 0ull;
                    break;
                }
                if (old == 0ull || (old & 0xFFFFFFFF00000000ull) == tag) {
                    cur = old;  // the page's entry (or an empty one): retry against it
                    continue;
                }
                slot = (slot + 1u) & a.table_mask;  // another page: probe on, expecting empty
                cur = 0ull;
            }
        }
    }
    const uint64_t m = __ballot(fresh);
    if (lane == 0) wcount[wv] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t base = used, tot = 0;
    for (uint32_t w = 0; w < nw; w++) {
        base += w < wv ? wcount[w] : 0u;
        tot += wcount[w];
    }
    used += tot;
    // the head record: the page's table slot and the claiming piece (the list's
    // tail: a page whose entry still names it has no other piece)
    if (fresh)
        reinterpret_cast<uint2*>(a.heads)[(uint64_t)blockIdx.x * a.seg_cap + base +
                                          (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = make_uint2(slot, (uint32_t)t);
    __syncthreads();  // wcount reused by the next chunk
}

// Block b inserts chunks b, b + grid, ... of kInsertThreads pieces into its
// head segment and leaves its record count in seg_count[b].
__global__ __launch_bounds__(kInsertThreads) void log_insert_kernel(LogLaunch a) {
    __shared__ uint32_t wcount[kInsertThreads / 64 + 1];
    if (a.zero_ctrs && blockIdx.x == 0 && threadIdx.x < 3) a.zero_ctrs[threadIdx.x] = 0ull;  // the queue's counters
    uint32_t used = 0;
    const uint64_t chunks = (a.n_pieces + kInsertThreads - 1) / kInsertThreads;
    for (uint64_t c = blockIdx.x; c < chunks; c += gridDim.x)
        insert_piece(a, c * kInsertThreads + threadIdx.x, wcount, used);
    if (threadIdx.x == 0) a.seg_count[blockIdx.x] = used;
}

// The bytes of one update that fall inside one page, page-relative: page bytes
// [rlo, rhi); the source byte of page byte r is sp[r] (sp is uniform, so every
// load below is an SGPR base + the lane's 32-bit offset + an immediate).
struct Piece {
    uint32_t rlo, rhi;
    const unsigned char* sp;
};
__device__ __forceinline__ Piece piece_in_page(uint64_t pbase, uint32_t page_bytes, uint64_t dst, uint64_t src,
                                               uint32_t len, const unsigned char* __restrict__ srcbuf) {
    Piece p;
    const uint64_t end = dst + len, pend = pbase + page_bytes;
    p.rlo = (uint32_t)((dst > pbase ? dst : pbase) - pbase);
    p.rhi = (uint32_t)((end < pend ? end : pend) - pbase);
    p.sp = srcbuf + (src - dst) + pbase;  // modular: only sp[r], r in [rlo, rhi), is ever dereferenced
    return p;
}

// Source bytes of one piece in the layout of the page registers (lane l holds
// page dwords l + 64j, i.e. page byte r = 4l + 256j), fetched with buffer
// loads: a lane that needs nothing passes an out-of-range offset, which the
// buffer unit answers with 0 without touching memory.  So every load is issued
// unconditionally (no branches around loads: hipcc's vmcnt counts stay exact
// and the next page's fetch really overlaps this page's merge + hash) and no
// byte outside the update's source range is ever read.  A dword the piece
// covers WHOLLY is one unaligned buffer_load_dword (gfx950 serves unaligned
// dword loads).  The at most two partially covered dwords (the piece's first
// and last) are spliced from the aligned source dwords holding their needed
// bytes, kept in 4 edge registers instead of a second [M] array.

template <int M>
struct PieceSrc {
    uint32_t S[M];
    uint32_t ea[2], eb[2];  // aligned source dwords holding edge dword k's bytes
};

// page dword index of the partially covered first / last dword (none = 0xffffffff)
__device__ __forceinline__ void piece_edges(const Piece& p, uint32_t (&e)[2]) {
    const uint32_t df = p.rlo >> 2, dl = (p.rhi - 1) >> 2;
    const bool ff = (p.rlo & 3u) == 0 && 4 * df + 4 <= p.rhi;
    const bool fl = (p.rhi & 3u) == 0 && 4 * dl >= p.rlo;
    e[0] = ff ? 0xffffffffu : df;
    e[1] = (dl != df && !fl) ? dl : 0xffffffffu;
}

// Row structure of a piece (wave-uniform).  Row j = page bytes [256j, 256j+256)
// = dword l + 64j of every lane.  A piece is one contiguous byte range, so it
// touches rows [row0, row1] (the rows it dirties; in delta mode the rows read).
struct PieceRows {
    uint32_t row0, row1;
};
__device__ __forceinline__ PieceRows piece_rows(const Piece& p) {
    return {p.rlo >> 8, (p.rhi - 1) >> 8};
}

// Per-lane position of a piece: x_j = (page byte of the lane's row-j dword) -
// rlo, in wrapping 32-bit arithmetic, so "dword wholly inside the piece" is ONE
// unsigned compare per row, x_j < len - 3 (a dword below rlo wraps to >= 2^31),
// on the vector unit: no per-row scalar masks or uniform row selects.
struct PieceLane {
    uint32_t o;   // 4 * lane - rlo (wrapping)
    uint32_t l3;  // len - 3 if len >= 4, else 0 (no whole dword)
};
__device__ __forceinline__ PieceLane piece_lane(const Piece& p, uint32_t lane) {
    const uint32_t len = p.rhi - p.rlo;
    return {lane * 4u - p.rlo, len >= 4u ? len - 3u : 0u};
}

template <int M>
__device__ __forceinline__ void fetch_piece(PieceSrc<M>& r, const Piece& p, uint32_t lane) {
    const uint32_t sh = (uint32_t)(uintptr_t)p.sp & 3u;  // the same for every dword of the piece
    // whole dwords: base sp, offset = page byte; edges: aligned base sp - sh
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(p.sp), 0, 64u * 4u * M + 8u, kBufFlags);
    const __amdgpu_buffer_rsrc_t re =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(p.sp - sh), 0, 64u * 4u * M + 8u, kBufFlags);
    const uint32_t l4 = lane * 4u;
    const PieceLane pl = piece_lane(p, lane);
#pragma unroll
    for (int j = 0; j < M; j++) {
        const bool full = pl.o + 256u * j < pl.l3;
        r.S[j] = __builtin_amdgcn_raw_buffer_load_b32(
            rw, row_sel(full ? l4 : kBufOOB) + 256u * j, 0, 0);
    }
    uint32_t e[2];
    piece_edges(p, e);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t b = 4 * (e[k] & 0x3fffffffu);
        const bool mine = e[k] != 0xffffffffu && lane == (e[k] & 63u);
        const uint32_t k0 = p.rlo > b ? p.rlo - b : 0u;
        const uint32_t k1 = p.rhi < b + 4 ? p.rhi - b : 4u;
        r.ea[k] = __builtin_amdgcn_raw_buffer_load_b32(re, (mine && k0 < 4u - sh) ? b : kBufOOB, 0, 0);
        r.eb[k] = __builtin_amdgcn_raw_buffer_load_b32(re, (mine && sh && k1 > 4u - sh) ? b + 4 : kBufOOB, 0, 0);
    }
}

// Whole dwords: one compare + select per row, on the vector unit.  The <= 2
// partially covered dwords (the piece's first and last: each is one lane in
// one row) are spliced under their byte mask; the owning lane carries the row
// index, so each row costs a compare + select and there are no lane or row
// branches.  `dirty` (rows written) is uniform.
template <int M>
__device__ __forceinline__ void merge_piece(uint32_t (&w)[M], uint32_t& dirty, const PieceSrc<M>& r, const Piece& p,
                                            uint32_t lane) {
    const PieceLane pl = piece_lane(p, lane);
#pragma unroll
    for (int j = 0; j < M; j++) w[j] = pl.o + 256u * j < pl.l3 ? r.S[j] : w[j];
    uint32_t e[2];
    piece_edges(p, e);
    const uint32_t sh = (uint32_t)(uintptr_t)p.sp & 3u;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t v = sh ? __builtin_amdgcn_alignbyte(r.eb[k], r.ea[k], sh) : r.ea[k];
        const uint32_t b = 4 * (e[k] & 0x3fffffffu);
        const uint32_t k0 = p.rlo > b ? p.rlo - b : 0u;
        const uint32_t k1 = p.rhi < b + 4 ? p.rhi - b : 4u;
        const uint32_t mhi = k1 >= 4u ? 0xFFFFFFFFu : (1u << (8u * k1)) - 1u;
        const uint32_t mask = mhi & ~((1u << (8u * (k0 & 3u))) - 1u);  // uniform
        // row of edge k on its lane; no row elsewhere (or when there is no edge k)
        uint32_t row = (e[k] != 0xffffffffu && lane == (e[k] & 63u)) ? e[k] >> 6 : 0xFFFFu;
        asm volatile("" : "+v"(row));  // keep the per-row test one vector compare (not a scalar compare + mask)
#pragma unroll
        for (int j = 0; j < M; j++) w[j] = row == (uint32_t)j ? (v & mask) | (w[j] & ~mask) : w[j];
    }
    const PieceRows pr = piece_rows(p);
    const uint32_t top = pr.row1 >= 31 ? 0xFFFFFFFFu : (2u << pr.row1) - 1u;
    dirty |= top & ~((1u << pr.row0) - 1u);
}


// Full-mode fast path for a page with ONE piece (the common case).  Every row
// is, uniformly, untouched (read from the page), covered whole by the piece
// (read from the source: that row's buffer descriptor is the source's, chosen
// by a scalar select, with the same vector offset), or an edge row -- the
// first / last touched row when the piece starts / ends inside it (read from
// the page; its source dwords are fetched on their own and merged).  So no row
// but the <= 2 edge rows costs a vector compare or select (the generic path
// spends ~12 VALU a row on them: 411 VALU a page, the kernel's issue bound).
struct PieceEdges {
    uint32_t r[2];          // edge rows (uniform; kNoRow = none)
    uint32_t s[2];          // the lane's source dword in edge row q, if wholly inside the piece
    uint32_t ea[2], eb[2];  // the partially covered dwords' aligned source dwords (as PieceSrc)
};
constexpr uint32_t kNoRow = 0xFFFFu;

__device__ __forceinline__ void edge_rows(const Piece& p, uint32_t (&r)[2]) {
    const uint32_t row0 = p.rlo >> 8, row1 = (p.rhi - 1) >> 8;
    r[0] = (p.rlo & 255u) ? row0 : kNoRow;
    r[1] = ((p.rhi & 255u) && row1 != r[0]) ? row1 : kNoRow;
}

__device__ __forceinline__ uint32_t covered_rows(const Piece& p) {  // rows [f0, f1) the piece covers whole
    const uint32_t f0 = (p.rlo + 255u) >> 8, f1 = p.rhi >> 8;
    return f1 > f0 ? ((f1 >= 32u ? 0xFFFFFFFFu : (1u << f1) - 1u) & ~((1u << f0) - 1u)) : 0u;
}

template <int M>
__device__ __forceinline__ void load_rows_sel(uint32_t (&w)[M], const unsigned char* page, const unsigned char* sp,
                                              uint32_t cov, uint32_t lane) {
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(page), 0, 256u * M,
                                                                         kBufFlags);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(sp), 0, 256u * M,
                                                                         kBufFlags);
#pragma unroll
    for (int j = 0; j < M; j++)
        w[j] = __builtin_amdgcn_raw_buffer_load_b32(((cov >> j) & 1u) ? rs : rp, row_sel(4u * lane) + 256u * j, 0,
                                                    kLogRowAux);
}

template <int M>
__device__ __forceinline__ void fetch_edges(PieceEdges& r, const Piece& p, uint32_t lane) {
    const uint32_t sh = (uint32_t)(uintptr_t)p.sp & 3u;
    const __amdgpu_buffer_rsrc_t rw =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(p.sp), 0, 64u * 4u * M + 8u, kBufFlags);
    const __amdgpu_buffer_rsrc_t re =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(p.sp - sh), 0, 64u * 4u * M + 8u, kBufFlags);
    edge_rows(p, r.r);
    const PieceLane pl = piece_lane(p, lane);
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const bool in = r.r[q] != kNoRow && pl.o + 256u * r.r[q] < pl.l3;
        r.s[q] = __builtin_amdgcn_raw_buffer_load_b32(rw, in ? 4u * lane + 256u * r.r[q] : kBufOOB, 0, 0);
    }
    uint32_t e[2];
    piece_edges(p, e);
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t b = 4 * (e[k] & 0x3fffffffu);
        const bool mine = e[k] != 0xffffffffu && lane == (e[k] & 63u);
        const uint32_t k0 = p.rlo > b ? p.rlo - b : 0u;
        const uint32_t k1 = p.rhi < b + 4 ? p.rhi - b : 4u;
        r.ea[k] = __builtin_amdgcn_raw_buffer_load_b32(re, (mine && k0 < 4u - sh) ? b : kBufOOB, 0, 0);
        r.eb[k] = __builtin_amdgcn_raw_buffer_load_b32(re, (mine && sh && k1 > 4u - sh) ? b + 4 : kBufOOB, 0, 0);
    }
}

// w: rows loaded by load_rows_sel (covered rows already hold the new bytes)
template <int M>
__device__ __forceinline__ void merge_edges(uint32_t (&w)[M], uint32_t& dirty, const PieceEdges& r, const Piece& p,
                                            uint32_t lane) {
    const PieceLane pl = piece_lane(p, lane);
    uint32_t e[2];
    piece_edges(p, e);
    const uint32_t sh = (uint32_t)(uintptr_t)p.sp & 3u;
#pragma unroll
    for (int q = 0; q < 2; q++) {
        const uint32_t rq = r.r[q];
        if (rq == kNoRow) continue;  // uniform
        uint32_t v = w[rq];          // uniform dynamic row index
        v = pl.o + 256u * rq < pl.l3 ? r.s[q] : v;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            if (e[k] == 0xffffffffu || (e[k] >> 6) != rq) continue;  // uniform
            const uint32_t spl = sh ? __builtin_amdgcn_alignbyte(r.eb[k], r.ea[k], sh) : r.ea[k];
            const uint32_t b = 4 * e[k];
            const uint32_t k0 = p.rlo > b ? p.rlo - b : 0u;
            const uint32_t k1 = p.rhi < b + 4 ? p.rhi - b : 4u;
            const uint32_t mhi = k1 >= 4u ? 0xFFFFFFFFu : (1u << (8u * k1)) - 1u;
            const uint32_t mask = mhi & ~((1u << (8u * (k0 & 3u))) - 1u);
            v = lane == (e[k] & 63u) ? (spl & mask) | (v & ~mask) : v;
        }
        w[rq] = v;
    }
    const PieceRows pr = piece_rows(p);
    const uint32_t top = pr.row1 >= 31 ? 0xFFFFFFFFu : (2u << pr.row1) - 1u;
    dirty |= top & ~((1u << pr.row0) - 1u);
}

// One wave per touched page, balanced: wave w owns heads w, w + W, w + 2W, ...
// (W = waves in the grid), ~pages/W each.  Its lanes load the metadata of up to
// 64 of its heads at once (table entry: page + one piece, that piece's list
// link and update descriptor: a few round trips per 64 pages), then the wave
// software-pipelines them: while page k's pieces are merged, stored and
// hashed, page k+1's data AND the source bytes of its piece are in flight.  A
// page with several pieces (overlapping / neighbouring writes: rare) walks its
// list, ranks the pieces by update index and applies them in log order; for
// a page with more than 64 (a log hammering it) the wave replays the whole log
// in place.  Every page is owned by exactly one wave: no write races, no
// flags, no atomics on the data.
// Delta mode (cc_apply_log_delta_dev): the stored CRC of each touched page is
// taken as the CRC of its bytes before the batch and updated through
// linearity, V(new) = V(old) ^ raw0(old ^ new) (equal lengths: the init and
// xorout terms cancel), so only the rows the page's pieces touch are read --
// untouched rows get an out-of-range buffer offset (0, no memory traffic) and
// contribute 0 to old ^ new.  A page with several pieces reads all rows.
// Bit-identical to the full rehash whenever the stored CRC matched the page;
// if it did not (latent corruption), the mismatch survives the write instead
// of being laundered into a fresh CRC.
template <int M>
__device__ __forceinline__ void load_rows(uint32_t (&w)[M], const unsigned char* page, uint32_t rows, uint32_t lane) {
    const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(page), 0, 256u * M,
                                                                         kBufFlags);
#pragma unroll
    for (int j = 0; j < M; j++)
        w[j] = __builtin_amdgcn_raw_buffer_load_b32(rp, row_sel(((rows >> j) & 1u) ? 4u * lane : kBufOOB) + 256u * j, 0, 2);
}

// cc_apply_logs_dev: the next batch's grouping in this page kernel's tail.  A
// workgroup whose waves are all done with their pages (its LDS image no longer
// read: the insert's scratch) takes kGroupTake chunks of 64*WV pieces at a time
// from one counter until none is left or it holds `rounds` of them (its head
// segment's bound);
// the workgroups that finish first take them while the slow ones finish, so
// the grouping costs no kernel time and no launch.  Every workgroup stores its
// segment's count.  Block 0 zeroes the counter the grouping after next uses
// (the one before this used it; it has completed).
template <int WV>
__device__ __forceinline__ void group_next(const LogInsert& nx, uint32_t* tab) {
    if (!nx.n_pieces) return;  // uniform
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicExch(nx.zero, 0ull);
    __syncthreads();  // every wave of the workgroup is past its pages
    constexpr uint32_t T = 64u * WV;
    const uint64_t chunks = (nx.n_pieces + T - 1) / T;
    uint32_t used = 0;
    for (uint32_t r = 0; r + kGroupTake <= nx.rounds; r += kGroupTake) {
        if (threadIdx.x == 0) tab[T] = (uint32_t)atomicAdd(nx.take, 1ull);  // (< 2^32 takes: n_pieces < 2^31)
        __syncthreads();
        const uint64_t c = (uint64_t)kGroupTake * tab[T];
        if (c >= chunks) break;  // uniform
        for (uint32_t i = 0; i < kGroupTake && c + i < chunks; i++)
            insert_piece(nx, (c + i) * T + threadIdx.x, tab, used);  // ends with a barrier: tab[T] free again
    }
    if (threadIdx.x == 0) nx.seg_count[blockIdx.x] = used;
}

template <int M, bool Delta>
__device__ __forceinline__ void log_pages_body(const LogLaunch& a, uint32_t* tab) {
    constexpr int WV = log_waves(M, Delta);
    // the insert blocks' segment counts: lane l holds segments 4l .. 4l+3,
    // scum = inclusive prefix of the lanes' sums; head h (in segment order) is
    // record h - (heads before its segment) of its segment
    constexpr int kSpl = kInsertBlocks / 64;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t sc[kSpl];  // (32-bit: these stay live over the page loop)
#pragma unroll
    for (int j = 0; j < kSpl; j++) {
        const uint32_t sg = kSpl * lane + j;
        sc[j] = sg < a.n_segs ? a.seg_count[sg] : 0u;
    }
    uint32_t ssum = 0;
#pragma unroll
    for (int j = 0; j < kSpl; j++) ssum += sc[j];
    uint32_t scum = ssum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(scum, d, 64);
        if (lane >= (uint32_t)d) scum += o;
    }
    // an equal share of the heads per workgroup: [hb0, hb1); a workgroup without
    // one (a small log) leaves before filling its 160 KiB of LDS
    const uint32_t Hall = __builtin_amdgcn_readlane(scum, 63);
    const uint32_t hb0 = (uint32_t)((uint64_t)Hall * blockIdx.x / gridDim.x);
    const uint32_t hb1 = (uint32_t)((uint64_t)Hall * (blockIdx.x + 1) / gridDim.x);
    if (hb0 >= hb1) {
        group_next<WV>(a.nx, tab);
        return;
    }
    fill_lds<64 * WV>(tab, static_cast<const uint4*>(a.image));
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t c0 = lane << 2 & 0x7Cu;
    const uint32_t c1 = c0 | 0x10000u;
    const uint32_t cf = kFinBase + (lane << 2);
    constexpr uint32_t pb = 256u * M;  // = a.page_bytes (launch_log_pages picks M = page_bytes / 256): shifts, not 64-bit multiplies
    // The workgroup's heads are cut among its waves by age.  Its waves sit 4 to a
    // SIMD (wave t on SIMD t % 4, the (t / 4)-th oldest there) and the SIMD
    // issues oldest-first: with equal shares the four age groups ended at 80, 92,
    // 103 and 113 us (per-wave clocks, scripts/trace_log.py) and the workgroup
    // ran its last ~30 us with fewer waves than pages in flight.  Shares
    // weighted by age group (kSkew[t / 4]) end them within ~10 us of each other:
    // -3 % a batch (a priority that rotates every step instead: -1.5 %).  A/B
    // (profiles/write_log_skew_ab_r03.txt): 33/27/22/18 = 32/28/22/18 =
    // 34/26/22/18 < 30/26/23/21 < 28/26/24/22 < 36/28/21/15 < equal.
    constexpr uint32_t kSkew[4] = {33, 27, 22, 18};
    auto wprefix = [&](uint32_t t) {  // sum of the weights of waves 0 .. t-1
        uint32_t p = 0;
        for (uint32_t u = 0; u < t; u++) p += kSkew[(u / 4) & 3];
        return p;
    };
    const uint32_t Hb = hb1 - hb0, wsum = wprefix(WV);
    const uint32_t H = hb0 + (uint32_t)((uint64_t)Hb * wprefix(wave + 1) / wsum);  // this wave: [first, H)
    const uint32_t first = hb0 + (uint32_t)((uint64_t)Hb * wprefix(wave) / wsum);
    constexpr uint32_t W = 1;  // lane k <- head base + k
    // static shares only: a dynamic tail (the last 1/8 or 1/16 of the heads in
    // chunks of 4-16 through one atomic counter, as the page kernel does) measured
    // 7-19 % slower here (0.177-0.197 vs 0.165 ms a batch)
    for (uint32_t base = first; base < H; base += 64u * W) {
        // lane k <- head base + k*W (clamped loads: no branches around them)
        const uint64_t ih = (uint64_t)base + (uint64_t)lane * W;
        const bool hv = ih < H;
        // the lane's head in its segment: the segment holding head `base` (lane
        // tl's segments, then the first of them past it), then a walk over the
        // (few) segments the batch spans
        const uint32_t hi = hv ? (uint32_t)ih : base;
        uint32_t seg, sbefore;
        {
            const uint32_t tl = (uint32_t)__builtin_ctzll(__ballot(scum > base));
            uint32_t st = tl ? __builtin_amdgcn_readlane(scum, tl - 1) : 0u, s = kSpl * tl;
            bool found = false;
#pragma unroll
            for (int j = 0; j < kSpl; j++) {
                const uint32_t v = __builtin_amdgcn_readlane(sc[j], tl);
                if (!found) {
                    if (st + v > base) {
                        found = true;
                        s = kSpl * tl + j;
                    } else {
                        st += v;
                    }
                }
            }
            seg = s;
            sbefore = st;
            const uint32_t last = base + 63u < H - 1u ? base + 63u : H - 1u;
            for (;;) {
                uint32_t v = sc[0];
#pragma unroll
                for (int j = 1; j < kSpl; j++) v = (s % kSpl) == (uint32_t)j ? sc[j] : v;
                const uint32_t cnt = __builtin_amdgcn_readlane(v, s / kSpl);
                if (st + cnt > last || s + 1 >= a.n_segs) break;
                st += cnt;
                s++;
                seg = hi >= st ? s : seg;
                sbefore = hi >= st ? st : sbefore;
            }
        }
        // the head record gives the table slot AND the claiming piece, so the
        // claimer's descriptor loads beside the table entry: two dependent
        // round trips to a page's geometry instead of three (the list link is
        // needed by pages with several pieces only, far behind)
        const uint2 hrec = reinterpret_cast<const uint2*>(a.heads)[(uint64_t)seg * a.seg_cap + (hi - sbefore)];
        const uint32_t hslot = hrec.x, claimer = hrec.y;
        const unsigned long long ent = reinterpret_cast<const unsigned long long*>(a.table)[hslot];
        const UpdateDesc d = a.upd[claimer / a.slots];
        if (a.clear_table && hv) a.table[hslot] = 0ull;  // the slot is this lane's alone (one head per page)
        const uint32_t key = (uint32_t)(ent >> 32) - 1u;  // the page
        const uint32_t pfirst = (uint32_t)ent - 1u;       // the list head (the latest piece)
        const uint32_t nxt = a.next[pfirst];              // consumed by the several-piece path only
        const uint32_t u0 = pfirst / a.slots;  // the head piece's update
        // the claimer's geometry in its page (the only piece when single), packed:
        // rlo | rhi << 16 and the source pointer (3 VGPRs instead of the 5 of its descriptor)
        const Piece hp0 = piece_in_page((uint64_t)key * pb, pb, d.dst, d.src, d.len, a.src);
        const uint32_t hrr = hp0.rlo | hp0.rhi << 16;
        const uint64_t hsp = (uint64_t)(uintptr_t)hp0.sp;
        const bool single = pfirst == claimer;  // nobody pushed onto the claimer: the page's only piece
        const uint64_t singles = __ballot(single);
        const uint32_t cnt = (uint32_t)__popcll(__ballot(hv));  // valid lanes are 0 .. cnt-1
        // two pages in flight: k (being merged + hashed) and k+1.  (A third
        // bought nothing, round 3: 0.1488 vs 0.1454 ms in a timing ablation.  A
        // page iteration issues ~39 VMEM instructions in full mode -- 16 row
        // loads, 6 edge loads, 16 row stores, the CRC -- and ~53 on the generic
        // path; gfx950's 6-bit vmcnt counts at most 63 outstanding.)
        uint32_t A[M], B[M];
        constexpr bool kRowSel = !Delta;  // full mode: one-piece pages through the per-row source/page select
        using Src = typename std::conditional<kRowSel, PieceEdges, PieceSrc<M>>::type;
        Src S0, S1;
        auto fetch = [&](Src& r, const Piece& p) {
            if constexpr (kRowSel) {
                fetch_edges<M>(r, p, lane);
            } else {
                fetch_piece<M>(r, p, lane);
            }
        };
        auto head_piece = [&](uint32_t k) {
            const uint32_t rr = __builtin_amdgcn_readlane(hrr, k);
            return Piece{rr & 0xFFFFu, rr >> 16, reinterpret_cast<const unsigned char*>(readlane64(hsp, k))};
        };
        // one page step: merge + store + rehash page `pg` from (X, SX, px) while
        // the loads of the next page go into (Y, SY); false after the last page
        // delta mode: rows of page h to read (the head piece's if it is the
        // page's only piece) and the page's stored CRC (a vector load: a scalar
        // one would share lgkmcnt with the chain's LDS lookups)
        auto load_next = [&](uint32_t (&Y)[M], const Piece& py, uint32_t pgy, uint32_t h, uint32_t& ocy) {
            if constexpr (Delta) {
                const PieceRows r = piece_rows(py);
                const uint32_t top = r.row1 >= 31 ? 0xFFFFFFFFu : (2u << r.row1) - 1u;
                const uint32_t rows = ((singles >> h) & 1ull) ? top & ~((1u << r.row0) - 1u) : 0xFFFFFFFFu;
                load_rows<M>(Y, a.pool + (uint64_t)pgy * pb, rows, lane);
                uint32_t vz = 0;
                asm volatile("" : "+v"(vz));
                ocy = a.page_crcs[pgy + vz];
            } else {
                // rows the page's only piece covers whole come straight from the source
                load_rows_sel<M>(Y, a.pool + (uint64_t)pgy * pb, py.sp, ((singles >> h) & 1ull) ? covered_rows(py) : 0u,
                                 lane);
            }
        };
        auto step = [&](uint32_t (&X)[M], Src& SX, const Piece& px, uint32_t pg, uint32_t hh, uint32_t ocx,
                        uint32_t (&Y)[M], Src& SY, Piece& py, uint32_t& pgy, uint32_t& ocy) {
            const bool more = hh + 1 < cnt;
            // next page + its first piece's source bytes in flight (clamped to the
            // last page: a harmless re-read, so every step issues the same loads
            // and the vmcnt waits stay exact)
            const uint32_t h1 = more ? hh + 1 : hh;
            pgy = __builtin_amdgcn_readlane(key, h1);
            py = head_piece(h1);
            load_next(Y, py, pgy, h1, ocy);
            fetch(SY, py);
            const uint64_t pbase = (uint64_t)pg * pb;
            uint32_t dirty = 0;
            uint32_t O[Delta ? M : 1];
            if constexpr (Delta) {
#pragma unroll
                for (int j = 0; j < M; j++) O[j] = X[j];
            }
            if ((singles >> hh) & 1ull) {
                if constexpr (kRowSel) {
                    merge_edges<M>(X, dirty, SX, px, lane);
                } else {
                    merge_piece<M>(X, dirty, SX, px, lane);
                }
            } else {  // several pieces: collect the list, apply in log (update index) order
                // the list's first two pieces came with the metadata; their
                // descriptors (lanes 0, 1) and the link after the second load
                // together, so a two-piece page (nearly every page with several)
                // pays one round trip for its list instead of four.  (Loading these
                // with the previous step's edge loads instead measured equal.)
                const uint32_t u0h = __builtin_amdgcn_readlane(u0, hh);
                const uint32_t u1h = (uint32_t)__builtin_amdgcn_readlane(nxt, hh) / a.slots;  // the second piece's update
                uint32_t cnt = 2, mu = lane == 0 ? u0h : (lane == 1 ? u1h : 0xFFFFFFFFu);  // update of lane's piece
                const UpdateDesc dq = a.upd[lane < 2 ? mu : u0h];
                uint32_t q = a.next[__builtin_amdgcn_readlane(nxt, hh)];
                uint64_t dd = dq.dst, ds = dq.src;
                uint32_t dn = dq.len;
                while (q != kNoPiece && cnt < 64u) {
                    mu = lane == cnt ? q / a.slots : mu;
                    cnt++;
                    q = a.next[q];
                }
                if (cnt > 2 && q == kNoPiece) {  // rare: the other descriptors
                    const UpdateDesc dq = a.upd[lane < cnt ? mu : u0h];
                    dd = dq.dst, ds = dq.src, dn = dq.len;
                }
                if (q != kNoPiece) {  // > 64 pieces (a log hammering this page: rare)
                    // its own wave replays the whole log for this page, 64 records per round
                    // (a ballot of the records touching it), in log order
                    for (uint64_t b = 0; b < a.n_updates; b += 64) {
                        const uint64_t i = b + lane;
                        const UpdateDesc dr = a.upd[i < a.n_updates ? i : b];
                        const bool ok = i < a.n_updates && dr.len >= 1 && dr.len <= a.max_len &&
                                        dr.dst < a.pool_bytes && dr.len <= a.pool_bytes - dr.dst &&
                                        dr.dst < pbase + pb && dr.dst + dr.len > pbase;
                        for (uint64_t m = __ballot(ok); m; m &= m - 1) {
                            const uint32_t l = (uint32_t)__builtin_ctzll(m);
                            const Piece pq = piece_in_page(pbase, pb, readlane64(dr.dst, l), readlane64(dr.src, l),
                                                           __builtin_amdgcn_readlane(dr.len, l), a.src);
                            PieceSrc<M> T;
                            fetch_piece<M>(T, pq, lane);
                            merge_piece<M>(X, dirty, T, pq, lane);
                        }
                    }
                } else {
                    uint32_t rank = lane < cnt ? 0u : 0xFFFFu;  // lanes < cnt: distinct updates
                    for (uint32_t j = 0; j < cnt; j++) rank += (uint32_t)__builtin_amdgcn_readlane(mu, j) < mu;
                    auto lane_piece = [&](uint32_t l) {
                        return piece_in_page(pbase, pb, readlane64(dd, l), readlane64(ds, l),
                                             __builtin_amdgcn_readlane(dn, l), a.src);
                    };
                    if (kRowSel && cnt == 2) {  // both pieces' source bytes in flight together
                        const uint32_t l0 = (uint32_t)__builtin_ctzll(__ballot(rank == 0)), l1 = l0 ^ 1u;
                        const Piece q0 = lane_piece(l0), q1 = lane_piece(l1);
                        PieceSrc<M> T0, T1;
                        fetch_piece<M>(T0, q0, lane);
                        fetch_piece<M>(T1, q1, lane);
                        merge_piece<M>(X, dirty, T0, q0, lane);
                        merge_piece<M>(X, dirty, T1, q1, lane);
                    } else
                    for (uint32_t r = 0; r < cnt; r++) {
                        const Piece pq = lane_piece((uint32_t)__builtin_ctzll(__ballot(rank == r)));
                        if constexpr (kRowSel) {
                            PieceSrc<M> T;
                            fetch_piece<M>(T, pq, lane);
                            merge_piece<M>(X, dirty, T, pq, lane);
                        } else {
                            fetch_piece<M>(SX, pq, lane);  // SX (the prefetched head piece) is not used: reuse it
                            merge_piece<M>(X, dirty, SX, pq, lane);
                        }
                    }
                }
            }
            {  // changed rows only; the others get an out-of-range offset and are dropped
                const __amdgpu_buffer_rsrc_t rp =
                    __builtin_amdgcn_make_buffer_rsrc(a.pool + pbase, 0, 256u * M, kBufFlags);
#pragma unroll
                for (int j = 0; j < M; j++)
                    __builtin_amdgcn_raw_buffer_store_b32(
                        X[j], rp,
                        row_sel(((dirty >> j) & 1u) ? 4u * lane : kBufOOB) + 256u * j, 0, kLogStoreAux);
            }
            uint32_t crc;
            if constexpr (Delta) {
#pragma unroll
                for (int j = 0; j < M; j++) O[j] ^= X[j];  // old ^ new: 0 outside the changed bytes
                crc = wave_xor(apply_fin(tab, chain<M>(tab, O, c0, c1), cf)) ^ ocx;
            } else {
                crc = wave_xor(apply_fin(tab, chain<M>(tab, X, c0, c1), cf)) ^ a.kconst;
            }
            if (lane == 0) a.page_crcs[pg] = crc;
            return more;
        };
        // the two register sets alternate (no copies): page k in one while page
        // k+1's loads land in the other
        uint32_t pgA = __builtin_amdgcn_readlane(key, 0), pgB = pgA;
        uint32_t ocA = 0, ocB = 0;
        Piece pA = head_piece(0), pB = pA;
        load_next(A, pA, pgA, 0, ocA);
        fetch(S0, pA);
        for (uint32_t h = 0;; h += 2) {
            if (!step(A, S0, pA, pgA, h, ocA, B, S1, pB, pgB, ocB)) break;
            if (!step(B, S1, pB, pgB, h + 1, ocB, A, S0, pA, pgA, ocA)) break;
        }
    }
    group_next<WV>(a.nx, tab);
}

template <int M, bool Delta>
__global__ __launch_bounds__(64 * log_waves(M, Delta)) void log_pages_kernel(LogLaunch a) {
    __shared__ uint32_t tab[kLdsBytes / 4];
    log_pages_body<M, Delta>(a, tab);
}

// A small log (<= 64 writes of <= one page each: at most 2 pieces a write) in
// ONE launch, for the per-request latency of the write path: no table memset,
// no insert.  Every wave loads the log into its lanes and finds the distinct
// touched pages itself (a page belongs to the first write touching it: a
// 64-step scan over the earlier lanes); page u goes to wave u, which applies
// every write touching it in log order (a ballot over the lanes, set bits in
// lane order) through the generic piece merge, stores the changed rows and
// rehashes the page.  Blocks without a page exit before filling LDS.
template <int M, bool Delta>
__global__ __launch_bounds__(64 * log_small_waves(M, Delta)) void log_small_kernel(LogLaunch a) {
    constexpr int WV = log_small_waves(M, Delta);
    __shared__ uint32_t tab[kLdsBytes / 4];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t pb = a.page_bytes;
    uint32_t vz = 0;
    asm volatile("" : "+v"(vz));
    const bool valid = lane < a.n_updates;
    const UpdateDesc d = a.upd[(valid ? lane : 0u) + vz];
    const bool ok = valid && d.len >= 1 && d.len <= a.max_len && d.dst < a.pool_bytes && d.len <= a.pool_bytes - d.dst;
    const uint64_t q0 = ok ? d.dst / pb : 0, q1 = ok ? (d.dst + d.len - 1) / pb : 0;
    // write `lane` owns its page q0 (q1) unless an earlier write touches it
    bool own0 = ok, own1 = ok && q1 != q0;
    for (uint32_t j = 0; j < 63u && j + 1 < a.n_updates; j++) {
        const bool okj = __builtin_amdgcn_readlane((uint32_t)ok, j) != 0u;
        const uint64_t j0 = readlane64(q0, j), j1 = readlane64(q1, j);
        if (okj && lane > j) {
            own0 = own0 && !(j0 <= q0 && q0 <= j1);
            own1 = own1 && !(j0 <= q1 && q1 <= j1);
        }
    }
    const uint64_t m0 = __ballot(own0), m1 = __ballot(own1);
    const uint32_t D = (uint32_t)__popcll(m0) + (uint32_t)__popcll(m1);  // distinct touched pages
    const uint32_t Wg = gridDim.x * WV, W = D < Wg ? D : Wg;
    if (blockIdx.x * (uint32_t)WV >= W) return;  // uniform per block (an empty log: every block)
    fill_lds<64 * WV>(tab, static_cast<const uint4*>(a.image));
    const uint32_t c0 = lane << 2 & 0x7Cu;
    const uint32_t c1 = c0 | 0x10000u;
    const uint32_t cf = kFinBase + (lane << 2);
    const uint32_t* pages = reinterpret_cast<const uint32_t*>(a.pool) + lane;
    const uint32_t n0 = (uint32_t)__popcll(m0);
    for (uint32_t u = blockIdx.x * WV + wave; u < D; u += W) {
        // page u: the u-th owned q0 (lane order), then the owned q1s
        uint64_t mm = u < n0 ? m0 : m1;
        for (uint32_t r = u < n0 ? u : u - n0; r; r--) mm &= mm - 1;  // drop the lowest r set bits
        const uint32_t l = (uint32_t)__builtin_ctzll(mm);
        const uint64_t pg = u < n0 ? readlane64(q0, l) : readlane64(q1, l);
        const uint64_t pbase = pg * pb;
        uint32_t X[M], O[Delta ? M : 1];
        load_page<M>(X, pages + pg * (64u * M));
        if constexpr (Delta) {
#pragma unroll
            for (int j = 0; j < M; j++) O[j] = X[j];
        }
        uint32_t dirty = 0;
        const bool hit = ok && d.dst < pbase + pb && d.dst + d.len > pbase;
        for (uint64_t m = __ballot(hit); m; m &= m - 1) {  // the writes touching the page, in log order
            const uint32_t wl = (uint32_t)__builtin_ctzll(m);
            const Piece pq = piece_in_page(pbase, pb, readlane64(d.dst, wl), readlane64(d.src, wl),
                                           __builtin_amdgcn_readlane(d.len, wl), a.src);
            PieceSrc<M> T;
            fetch_piece<M>(T, pq, lane);
            merge_piece<M>(X, dirty, T, pq, lane);
        }
        const __amdgpu_buffer_rsrc_t rp = __builtin_amdgcn_make_buffer_rsrc(a.pool + pbase, 0, 256u * M, kBufFlags);
#pragma unroll
        for (int j = 0; j < M; j++)
            __builtin_amdgcn_raw_buffer_store_b32(X[j], rp, row_sel(((dirty >> j) & 1u) ? 4u * lane : kBufOOB) + 256u * j, 0, 0);
        uint32_t crc;
        if constexpr (Delta) {
#pragma unroll
            for (int j = 0; j < M; j++) O[j] ^= X[j];
            crc = wave_xor(apply_fin(tab, chain<M>(tab, O, c0, c1), cf)) ^ a.page_crcs[pg + vz];
        } else {
            crc = wave_xor(apply_fin(tab, chain<M>(tab, X, c0, c1), cf)) ^ a.kconst;
        }
        if (lane == 0) a.page_crcs[pg] = crc;
    }
}

// ---------------------------------------------------------------------------
// Write-log traffic probe (diagnostic, cc_apply_log_probe_dev): the memory
// traffic of the write log's page pass with everything else removed -- no
// hash table, no head segments, no list walk, no CRC.  The touched pages come
// as a host-built list (one descriptor a page: rows the page's only piece
// covers whole, read from the source as the real kernel reads them; rows the
// page's pieces dirty, stored back nt).  Same grid and occupancy as
// log_pages_kernel<16, false> (one workgroup of kLogWavesFull waves per CU),
// each wave an equal contiguous share of the pages, kProbeDepth pages in
// flight (the next pages' rows load while page k's dirty rows are stored; 2,
// as the page pass holds).  The stores write back
// what was loaded, so run right after the log it describes was applied, the
// probe changes no byte; `out` gets an XOR of each page's words (keeps every
// load live).  Its time is the ceiling of the write log's access pattern.
// ---------------------------------------------------------------------------
constexpr int kProbeDepth = 2;
template <int M>
__global__ __launch_bounds__(64 * kLogWavesFull) void log_probe_kernel(LogProbeLaunch a) {
    constexpr int D = kProbeDepth;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * kLogWavesFull, gw = (uint64_t)blockIdx.x * kLogWavesFull + wave;
    const uint64_t first = a.n * gw / W, last = a.n * (gw + 1) / W;
    for (uint64_t base = first; base < last; base += 64) {
        const uint64_t ih = base + lane;
        LogProbeDesc d = a.desc[ih < last ? ih : base];
        if (d.page >= a.pool_pages) d = LogProbeDesc{0, 0, 0u, 0u};  // past the pool: read page 0, store nothing
        const uint32_t cnt = (uint32_t)(last - base < 64 ? last - base : 64);
        uint32_t ring[D][M];
        auto load = [&](uint32_t (&Y)[M], uint32_t k) {
            const uint64_t pg = readlane64(d.page, k);
            const uint64_t so = readlane64(d.src_off, k);
            load_rows_sel<M>(Y, a.pool + pg * (256u * M), a.src + so, __builtin_amdgcn_readlane(d.covered, k), lane);
        };
        auto finish = [&](uint32_t (&X)[M], uint32_t k) {
            const uint64_t pg = readlane64(d.page, k);
            const uint32_t dirty = __builtin_amdgcn_readlane(d.dirty, k);
            const __amdgpu_buffer_rsrc_t rp =
                __builtin_amdgcn_make_buffer_rsrc(a.pool + pg * (256u * M), 0, 256u * M, kBufFlags);
            uint32_t x = 0;
#pragma unroll
            for (int j = 0; j < M; j++) {
                __builtin_amdgcn_raw_buffer_store_b32(X[j], rp, row_sel(((dirty >> j) & 1u) ? 4u * lane : kBufOOB) + 256u * j,
                                                      0, kLogStoreAux);
                x ^= X[j];
            }
            x = wave_xor(x);
            if (lane == 0) a.out[base + k] = x;
        };
#pragma unroll
        for (int st = 0; st < D - 1; st++) load(ring[st], (uint32_t)st < cnt ? st : cnt - 1);
        for (uint32_t k = 0;; k += D) {
            bool done = false;
#pragma unroll
            for (int st = 0; st < D; st++) {
                if (!done) {  // uniform
                    const uint32_t kn = k + st + D - 1;
                    load(ring[(st + D - 1) % D], kn < cnt ? kn : cnt - 1);  // clamped: every step issues the same loads
                    finish(ring[st], k + st);
                    done = k + st + 1 >= cnt;
                }
            }
            if (done) break;
        }
    }
}

// ---------------------------------------------------------------------------
// Diagnostic: the read traffic of a page list (cc_page_list_probe_dev) -- the
// access pattern of a batch of datastore reads with everything else removed:
// verify-on-read's grid and occupancy (kRvWaves waves a CU, LDS unused), each
// wave an equal contiguous share of the list (64 indices a lane-load), two
// pages in flight behind the one being reduced, a rotate-XOR instead of the
// CRC, one word a page out.
// ---------------------------------------------------------------------------
constexpr int kListProbeWaves = 8;  // = kRvWaves (verify-on-read's occupancy)
constexpr uint64_t kRvDynDivList = 16;   // = kRvDynDiv: the last 1/16 of the list is the dynamic tail
constexpr uint64_t kRvDynSlotsList = 32;  // = kRvDynSlots: pages per tail chunk
template <int M>
__global__ __launch_bounds__(64 * kListProbeWaves) void page_list_probe_kernel(PageListProbeLaunch a) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t W = (uint64_t)gridDim.x * kListProbeWaves, gw = (uint64_t)blockIdx.x * kListProbeWaves + wave;
    // the stream's other slot set, every head of it (the page kernel's next launch may pull from all)
    if (a.dyn_next && blockIdx.x == 0 && threadIdx.x < kDynHeads) atomicExch(a.dyn_next + threadIdx.x * kDynHeadStride, 0ull);
    // static shares of the first Ts entries, then 32-entry chunks of the rest from
    // one counter (verify-on-read's tail: kRvDynDiv, kRvDynSlots)
    const uint64_t Ts = a.dyn_ctr ? a.n - a.n / kRvDynDivList : a.n;
    const uint64_t n_dyn = (a.n - Ts + kRvDynSlotsList - 1) / kRvDynSlotsList;
    uint64_t first = Ts * gw / W, last = Ts * (gw + 1) / W;
    const uint32_t* pages = a.pool + lane;
    for (;;) {
    for (uint64_t base = first; base < last; base += 64) {
        const uint64_t ih = base + lane;
        const uint64_t pg0 = a.pages[ih < last ? ih : base];
        const uint64_t pg = pg0 < a.pool_pages ? pg0 : 0;  // a bad index reads page 0, never past the pool
        const uint32_t cnt = (uint32_t)(last - base < 64 ? last - base : 64);
        auto at = [&](uint32_t k) { return readlane64(pg, k < cnt ? k : cnt - 1); };  // clamped: same loads every step
        uint32_t A[M], B[M], Cq[M];
        load_page<M>(A, pages + at(0) * (64u * M));
        load_page<M>(B, pages + at(1) * (64u * M));
        auto step = [&](uint32_t (&X)[M], uint32_t k, uint32_t (&Y)[M]) {
            load_page<M>(Y, pages + at(k + 2) * (64u * M));
            uint32_t x = X[0];
#pragma unroll
            for (int j = 1; j < M; j++) x = ((x << 1) | (x >> 31)) ^ X[j];
            x = wave_xor(x);
            if (lane == 0) a.out[base + k] = x;
            return k + 1 < cnt;
        };
        for (uint32_t k = 0;; k += 3) {
            if (!step(A, k, Cq)) break;
            if (!step(B, k + 1, A)) break;
            if (!step(Cq, k + 2, B)) break;
        }
    }
    if (!a.dyn_ctr) break;
    unsigned long long c = 0;
    if (lane == 0) c = atomicAdd(a.dyn_ctr, 1ull);
    c = readlane64(c, 0);
    if (c >= n_dyn) break;
    first = Ts + c * kRvDynSlotsList;
    last = first + kRvDynSlotsList < a.n ? first + kRvDynSlotsList : a.n;
    }
}

// ---------------------------------------------------------------------------
// Verify-on-read for a batch of datastore reads (cc_verify_reads_dev)
// ---------------------------------------------------------------------------
// Pages a read touches (0 for an empty read and for one past the pool).
__device__ __forceinline__ uint64_t read_pages(const ReadVerifyLaunch& a, const RangeDesc& r) {
    if (!r.len || r.off >= a.pool_bytes || r.len > a.pool_bytes - r.off) return 0;
    return ((r.off + r.len - 1) >> a.page_shift) - (r.off >> a.page_shift) + 1;
}

// Pages of tile t (reads [n t / T, n (t+1) / T)), uniform; mark: reads past the
// pool get bad_per_read = UINT32_MAX (the tile's counting wave marks them).
__device__ __forceinline__ uint64_t read_tile_count(const ReadVerifyLaunch& a, uint32_t t, uint32_t lane, bool mark) {
    const uint64_t lo = a.n_reads * t / kReadTiles, hi = a.n_reads * (t + 1) / kReadTiles;
    uint64_t sum = 0;
    for (uint64_t i = lo + lane; i < hi; i += 64) {
        const RangeDesc r = a.reads[i];
        sum += read_pages(a, r);
        if (mark && r.len && (r.off >= a.pool_bytes || r.len > a.pool_bytes - r.off)) a.bad_per_read[i] = 0xFFFFFFFFu;
    }
#pragma unroll
    for (int d = 32; d; d >>= 1) sum += __shfl_xor(sum, d, 64);
    return sum;
}

// Every page a read touches is one slot; the batch's slots are read 0's pages,
// then read 1's, ...  ONE launch, scheduled as the range kernel is (§7): the
// waves count kReadTiles tiles of reads themselves (epoch-tagged words, a
// bounded wait) and hold the counts in registers; wave w owns the slots
// [Ts w / W, Ts (w+1) / W) at PAGE granularity (a read may be split over
// waves; its mismatches are counted by atomics), the last T / kRvDynDiv slots
// are dynamic chunks.  A share starts at the read holding its first slot
// (tile search in registers, then the tile's reads 64 at a time); the wave
// takes its reads 64 at a time (lane j <- one read: first page, page count)
// and lays their pages out as one stream with a wave prefix sum: page k of
// the stream belongs to the first lane whose running count exceeds k (a
// ballot), so the stream is walked with uniform scalar math only -- no loads
// in the per-page path -- hashed with the next two pages' loads in flight
// (three register sets rotating).  The stored CRCs come in with VECTOR loads
// (an opaque zero in the address) so they never share lgkmcnt with the chain's
// LDS lookups.  A mismatch is counted on its read (rare: atomics).
// (Rounds 2-3: a count kernel and rocPRIM's two-launch exclusive scan ran
// first, 16-24 us of a 0.67 ms call.)
constexpr int kRvWaves = 8;  // waves per CU of the verify-on-read kernel
constexpr uint64_t kRvDynDiv = 16;  // 1/16 of the slots form the dynamic tail (A/B: 2-3 % over none; 1/8, 1/32 less)
constexpr uint32_t kRvHeads = 1;  // tail heads (A/B round 3: 8 per-XCD heads = one counter at 1/16)
constexpr uint64_t kRvDynSlots = 32;  // slots (pages) per dynamic chunk (64: -1 %, 128: -5 %, 256: -18 % -- too coarse)
constexpr uint64_t kRvMinSlots = 8;  // a small batch goes to the fewest waves that give each >= 8 page slots
constexpr uint32_t kRvSmallMinSlots = 2;  // the one-launch path (<= 64 reads): >= 2 pages per wave
template <int M>
__global__ __launch_bounds__(64 * kRvWaves) void read_verify_kernel(ReadVerifyLaunch a) {
    __shared__ uint32_t tab[kLdsBytes / 4];
    const uint64_t n = a.n_reads;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t Wg = (uint64_t)gridDim.x * kRvWaves;
    const uint64_t w = (uint64_t)blockIdx.x * kRvWaves + wave;
    const uint64_t tag = (uint64_t)a.epoch << kEpochShift;
    // this wave's tile counts, published before the LDS fill
    for (uint64_t t = w; t < kReadTiles; t += Wg) {
        const uint64_t cnt = read_tile_count(a, (uint32_t)t, lane, true);
        if (lane == 0) __hip_atomic_store(a.tiles + t, tag | cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the tail's counter: slot epoch % 2; this call zeroes the other for the next
    unsigned long long* dyn_ctr = a.tail + (a.epoch & 1u) * kDynCtrWords64;
    if (blockIdx.x == 0 && threadIdx.x < kRvHeads)
        atomicExch(a.tail + ((a.epoch + 1u) & 1u) * kDynCtrWords64 + threadIdx.x * kDynHeadStride, 0ull);
    fill_lds<64 * kRvWaves>(tab, static_cast<const uint4*>(a.image));
    const uint32_t c0 = lane << 2 & 0x7Cu;
    const uint32_t c1 = c0 | 0x10000u;
    const uint32_t cf = kFinBase + (lane << 2);
    const uint32_t* pages = a.pool + lane;
    uint32_t vz = 0;
    asm volatile("" : "+v"(vz));  // opaque zero: keeps uniform-address loads on the vector path

    constexpr int kTpl = kReadTiles / 64;
    uint64_t tb[kTpl];
    wait_tiles<kTpl>(tb, a.tiles, tag, lane, [&](uint32_t t) { return read_tile_count(a, t, lane, false); });
    uint64_t lsum = 0;
#pragma unroll
    for (int j = 0; j < kTpl; j++) lsum += tb[j];
    const uint64_t cum = wave_scan_incl(lsum, lane);
    const uint64_t T = readlane64(cum, 63);
    // W waves share the slots: all of the grid for a large batch, fewer for a small one
    const uint64_t Wt = (T + kRvMinSlots - 1) / kRvMinSlots;
    const uint64_t W = Wt < Wg ? (Wt ? Wt : 1) : Wg;
    if ((uint64_t)blockIdx.x * kRvWaves >= W) return;  // uniform per block: no share, no tail
    auto stored_crc = [&](uint64_t g) { return a.page_crcs[g + vz]; };
    // static shares of the first Ts slots, then dynamic chunks of kRvDynSlots
    // slots (the page kernel's tail: the XCDs run at different rates)
    const uint64_t Ts = T - T / kRvDynDiv;
    uint32_t dyn_head, dyn_tried;
    tail_cursor<kRvHeads>(dyn_head, dyn_tried);
    uint64_t lo_slot = w < W ? Ts * w / W : Ts, hi_slot = w < W ? Ts * (w + 1) / W : Ts;  // waves past W: tail only
#pragma unroll 1
    for (;;) {
        // slots [lo_slot, hi_slot) at PAGE granularity: from the read holding
        // slot lo_slot through the reads starting before hi_slot, cut at both ends
        uint64_t base = n, S = 0;  // the group's first read and the slot of its page 0
        RangeDesc rs;              // the search's last 64 descriptors: the first group's (no second load)
        bool have_rs = false;
        if (lo_slot < hi_slot) {
            const TileHit th = tile_of(cum, tb, lo_slot, lane);
            base = n * th.tile / kReadTiles;
            S = th.before;
            // the tile's reads 64 at a time, to the group whose pages pass lo_slot
            for (;;) {
                const uint64_t ri = base + lane;
                rs = a.reads[(ri < n ? ri : base) + vz];
                const uint64_t c = wave_scan_incl(ri < n ? read_pages(a, rs) : 0u, lane);
                const uint64_t tot = readlane64(c, 63);
                if (S + tot > lo_slot || base + 64 >= n) break;
                S += tot;
                base += 64;
            }
            have_rs = true;
        }
        for (; base < n && S < hi_slot; base += 64) {
            const uint64_t ri = base + lane;
            const bool valid = ri < n;
            const RangeDesc r = have_rs ? rs : a.reads[(valid ? ri : base) + vz];
            have_rs = false;
            const uint32_t cnt = valid ? (uint32_t)read_pages(a, r) : 0u;  // 0 also for reads past the pool
            const uint64_t p0 = r.off >> a.page_shift;
            uint32_t cum32 = cnt;  // inclusive prefix sum over the lanes
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint32_t o = __shfl_up(cum32, d, 64);
                if (lane >= (uint32_t)d) cum32 += o;
            }
            const uint32_t P = __builtin_amdgcn_readlane(cum32, 63);
            const uint32_t ks = lo_slot > S ? (uint32_t)(lo_slot - S) : 0u;
            const uint32_t ke = hi_slot - S < (uint64_t)P ? (uint32_t)(hi_slot - S) : P;
            S += P;
            if (ks >= ke) continue;
            auto page_at = [&](uint32_t k, uint32_t& owner) -> uint64_t {
                owner = (uint32_t)__builtin_ctzll(__ballot(cum32 > k));
                const uint32_t before = owner ? (uint32_t)__builtin_amdgcn_readlane(cum32, owner - 1) : 0u;
                const uint64_t first = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(p0 >> 32), owner) << 32) |
                                       (uint32_t)__builtin_amdgcn_readlane((uint32_t)p0, owner);
                return first + (k - before);
            };
            uint32_t A[M], B[M], Cq[M];
            uint32_t oA, oB, oC;
            uint64_t gA = page_at(ks, oA), gB = page_at(ks + 1 < ke ? ks + 1 : ks, oB), gC = gB;
            oC = oB;
            uint32_t sA = stored_crc(gA), sB = stored_crc(gB), sC = sB;
            load_page<M>(A, pages + gA * (64u * M));
            load_page<M>(B, pages + gB * (64u * M));
            // hash X (page k: stored CRC sx, owner lane ox); page k+2's loads go into Y
            auto step = [&](uint32_t (&X)[M], uint32_t sx, uint32_t ox, uint32_t k, uint32_t (&Y)[M], uint64_t& gy,
                            uint32_t& sy, uint32_t& oy) {
                const bool more = k + 1 < ke;
                gy = page_at(k + 2 < ke ? k + 2 : ke - 1, oy);  // clamped: same loads every step
                sy = stored_crc(gy);
                load_page<M>(Y, pages + gy * (64u * M));
                const uint32_t crc = wave_xor(apply_fin(tab, chain<M>(tab, X, c0, c1), cf)) ^ a.kconst;
                if (crc != sx && lane == 0) {
                    atomicAdd(a.bad_per_read + base + ox, 1u);
                    atomicAdd(a.bad_total, 1ull);
                }
                return more;
            };
            for (uint32_t k = ks;; k += 3) {
                if (!step(A, sA, oA, k, Cq, gC, sC, oC)) break;
                if (!step(B, sB, oB, k + 1, A, gA, sA, oA)) break;
                if (!step(Cq, sC, oC, k + 2, B, gB, sB, oB)) break;
            }
        }
        const uint64_t n_dyn = (T - Ts + kRvDynSlots - 1) / kRvDynSlots;
        const uint64_t c = tail_pull<kRvHeads>(dyn_ctr, n_dyn, dyn_head, dyn_tried, lane);
        if (c >= n_dyn) break;
        lo_slot = Ts + c * kRvDynSlots;
        hi_slot = lo_slot + kRvDynSlots < T ? lo_slot + kRvDynSlots : T;
    }
}


// A small batch (<= 64 reads: one per lane) in ONE launch, for the per-request
// latency of the read path: no count kernel and no scan.  Every wave loads the
// batch's descriptors, computes the pages per read (a read past the pool is
// marked as read_counts_kernel marks it) and their wave prefix sum; the P pages
// are split evenly over the fewest waves that give each >= kRvMinSlots, at
// PAGE granularity (a 32-page read is verified by 4 waves), and the blocks left
// without pages exit before filling LDS.
template <int M>
__global__ __launch_bounds__(64 * kRvWaves) void read_verify_small_kernel(ReadVerifyLaunch a) {
    __shared__ uint32_t tab[kLdsBytes / 4];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t vz = 0;
    asm volatile("" : "+v"(vz));
    const bool valid = lane < a.n_reads;
    const RangeDesc r = a.reads[(valid ? lane : 0u) + vz];
    const bool past = r.off >= a.pool_bytes || r.len > a.pool_bytes - r.off;
    uint32_t cnt = 0;
    if (valid && !past && r.len) cnt = (uint32_t)((r.off + r.len - 1) / a.page_bytes - r.off / a.page_bytes + 1);
    if (valid && past && r.len && blockIdx.x == 0 && wave == 0) a.bad_per_read[lane] = 0xFFFFFFFFu;
    const uint64_t p0 = r.off / a.page_bytes;
    uint32_t cum = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(cum, d, 64);
        if (lane >= (uint32_t)d) cum += o;
    }
    const uint32_t P = __builtin_amdgcn_readlane(cum, 63);
    const uint32_t Wg = gridDim.x * kRvWaves, Wt = (P + kRvSmallMinSlots - 1) / kRvSmallMinSlots;
    const uint32_t W = Wt < Wg ? Wt : Wg;
    if (blockIdx.x * (uint32_t)kRvWaves >= W) return;  // uniform per block (P == 0: every block)
    fill_lds<64 * kRvWaves>(tab, static_cast<const uint4*>(a.image));
    const uint32_t w = blockIdx.x * kRvWaves + wave;
    if (w >= W) return;
    const uint32_t k0 = (uint32_t)((uint64_t)P * w / W), k1 = (uint32_t)((uint64_t)P * (w + 1) / W);
    const uint32_t c0 = lane << 2 & 0x7Cu;
    const uint32_t c1 = c0 | 0x10000u;
    const uint32_t cf = kFinBase + (lane << 2);
    const uint32_t* pages = a.pool + lane;
    auto page_at = [&](uint32_t k, uint32_t& owner) -> uint64_t {
        owner = (uint32_t)__builtin_ctzll(__ballot(cum > k));
        const uint32_t before = owner ? (uint32_t)__builtin_amdgcn_readlane(cum, owner - 1) : 0u;
        return readlane64(p0, owner) + (k - before);
    };
    // pages k0 .. k1-1, the next page's loads in flight while one is hashed
    uint32_t X[M], Y[M];
    uint32_t ox, oy;
    uint64_t gx = page_at(k0, ox);
    uint32_t sx = a.page_crcs[gx + vz];
    load_page<M>(X, pages + gx * (64u * M));
    for (uint32_t k = k0; k < k1; k++) {
        const uint64_t gy = page_at(k + 1 < k1 ? k + 1 : k, oy);  // clamped: same loads every step
        const uint32_t sy = a.page_crcs[gy + vz];
        load_page<M>(Y, pages + gy * (64u * M));
        const uint32_t crc = wave_xor(apply_fin(tab, chain<M>(tab, X, c0, c1), cf)) ^ a.kconst;
        if (crc != sx && lane == 0) {
            atomicAdd(a.bad_per_read + ox, 1u);
            atomicAdd(a.bad_total, 1ull);
        }
#pragma unroll
        for (int j = 0; j < M; j++) X[j] = Y[j];
        sx = sy;
        ox = oy;
    }
}

__global__ void combine_kernel(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, uint32_t m,
                               uint64_t n, uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = mulmod_dev(m, a[i]) ^ b[i];
}

// One wave per file: x^(8*after) as a wave-parallel product of x^(2^k)
// factors (6 shuffle-multiply levels instead of ~40 serial multiplies).
__global__ __launch_bounds__(256) void digest_kernel(const uint32_t* __restrict__ crcs,
                                                     const uint64_t* __restrict__ after,
                                                     const uint32_t* __restrict__ group, uint64_t n,
                                                     uint32_t* __restrict__ digest) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += (uint64_t)gridDim.x * 4) {
        const uint32_t c = crcs[i];
        const uint64_t nb = after[i];
        const uint32_t m = xpow_wave(nb << 3, lane);
        if (lane == 0) atomicXor(digest + group[i], mulmod_dev(m, c));
    }
}

// out[i] = XOR over r of gathered[r*n + i]: the local fold after the RCCL
// all-gather of per-copyset digest partials (XOR is not an RCCL op).
__global__ void xor_fold_kernel(const uint32_t* __restrict__ gathered, uint32_t nranks, uint64_t n,
                                uint32_t* __restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t v = 0;
    for (uint32_t r = 0; r < nranks; r++) v ^= gathered[(uint64_t)r * n + i];
    out[i] = v;
}

// Fused metapages only ride a dynamic tail (the static walk knows one array).
TailExtra tail_extra(const PageLaunch& a) {
    const bool meta = a.dyn_ctr && a.meta_pages && a.n_meta;
    return {meta ? a.meta_pages : nullptr, meta ? a.n_meta : 0, meta ? a.meta_out : nullptr,
            a.dyn_ctr ? a.dyn_next : nullptr};
}

template <int MODE>
hipError_t launch_page(const PageLaunch& a, hipStream_t s) {
    const dim3 grid(a.blocks), block(kBlockThreads);
    const uint4* img = static_cast<const uint4*>(a.image);
    const ZeroRanges zr = {{a.zero[0], a.zero[1]}, {a.zero[0] ? a.zero_words[0] : 0, a.zero[1] ? a.zero_words[1] : 0}};
    const TailExtra ex = tail_extra(a);
#define CC_CASE(MM)                                                                                     \
    case MM:                                                                                            \
        hipExtLaunchKernelGGL((page_crc_kernel<MM, MODE>), grid, block, 0, s, a.ev_begin, a.ev_end, 0u,  \
                              a.pages, a.n_pages, img, a.kconst, a.out, a.expected, a.sink, a.tile_shift, \
                              a.dyn_ctr, a.static_tiles, zr, ex);                                       \
        break;
    switch (a.words_per_lane) {
        CC_CASE(1)
        CC_CASE(2)
        CC_CASE(4)
        CC_CASE(8)
        CC_CASE(16)
        CC_CASE(32)
        default:
            hipExtLaunchKernelGGL((page_crc_kernel_dyn<MODE>), grid, block, 0, s, a.ev_begin, a.ev_end, 0u, a.pages,
                                  a.n_pages, a.words_per_lane, img, a.kconst, a.out, a.expected, a.sink, zr);
    }
#undef CC_CASE
    return hipGetLastError();
}

}  // namespace

hipError_t launch_page_crc(const PageLaunch& a, hipStream_t s) { return launch_page<0>(a, s); }

// The scan step's metapage pass: the compute kernel as its own instantiation
// (MODE 3 = MODE 0), so a kernel trace reports the 1,024-page metapage launches
// apart from the 16 GiB data launches instead of averaging the two.
hipError_t launch_page_meta(const PageLaunch& a, hipStream_t s) {
    if (a.words_per_lane != 16) return launch_page<0>(a, s);
    const ZeroRanges zr = {{a.zero[0], a.zero[1]}, {a.zero[0] ? a.zero_words[0] : 0, a.zero[1] ? a.zero_words[1] : 0}};
    hipLaunchKernelGGL((page_crc_kernel<16, 3>), dim3(a.blocks), dim3(kBlockThreads), 0, s, a.pages, a.n_pages,
                       static_cast<const uint4*>(a.image), a.kconst, a.out, a.expected, a.sink, a.tile_shift,
                       a.dyn_ctr, a.static_tiles, zr, tail_extra(a));
    return hipGetLastError();
}

hipError_t launch_page_load_probe(const PageLaunch& a, hipStream_t s) {
    if (a.words_per_lane != 16) return hipErrorInvalidValue;  // 4 KiB pages only
    const ZeroRanges zr = {{nullptr, nullptr}, {0, 0}};
    hipLaunchKernelGGL((page_crc_kernel<16, 2>), dim3(a.blocks), dim3(kBlockThreads), 0, s, a.pages, a.n_pages,
                       static_cast<const uint4*>(a.image), a.kconst, a.out, a.expected, a.sink, a.tile_shift,
                       a.dyn_ctr, a.static_tiles, zr, tail_extra(a));
    return hipGetLastError();
}

// Read-only probe (diagnostic): dwordx4 nt loads, 4 in flight per lane, the
// fastest pure-read shape found by scripts/hbm_probe.hip.  Static strided
// schedule: it waits for the slowest XCD as the page kernel did before its
// dynamic tail (a dynamic-tail version of this probe measured slower, 6.7 TB/s).
__global__ __launch_bounds__(1024) void read_probe_kernel(const uint4* __restrict__ p, uint64_t n16,
                                                          uint32_t* __restrict__ sink) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint64_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6);
    const uint64_t waves = (uint64_t)gridDim.x * 16;
    constexpr uint64_t kStep = 64 * 4;  // 16-byte elements per wave per step
    uint32_t acc = 0;
    const u32x4* q = reinterpret_cast<const u32x4*>(p);
    for (uint64_t b = wave * kStep; b + kStep <= n16; b += waves * kStep) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = __builtin_nontemporal_load(q + b + u * 64 + lane);
#pragma unroll
        for (int u = 0; u < 4; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    acc ^= __shfl_xor(acc, 32);
    if (lane == 0) sink[wave] = acc;
}

hipError_t launch_read_probe(const void* buf, uint64_t bytes, uint32_t* sink, int blocks, hipStream_t s) {
    hipLaunchKernelGGL(read_probe_kernel, dim3(blocks), dim3(1024), 0, s, static_cast<const uint4*>(buf), bytes / 16,
                       sink);
    return hipGetLastError();
}
hipError_t launch_page_verify(const PageLaunch& a, hipStream_t s) { return launch_page<1>(a, s); }

hipError_t launch_fold(const FoldLaunch& a, hipStream_t s) {
    if (a.n_groups == 0) return hipSuccess;
    if (a.per_group >= 64 && a.per_group % 64 == 0) {
        uint64_t blocks = (a.n_groups + 3) / 4;
        if (blocks > 2048) blocks = 2048;  // grid-stride: the LDS product table is built once per block
        hipLaunchKernelGGL(fold_kernel_wave, dim3((uint32_t)blocks), dim3(256), 0, s, a.crcs, a.n_groups,
                           a.per_group, a, a.out);
    } else {
        const uint64_t blocks = (a.n_groups + 255) / 256;
        hipLaunchKernelGGL(fold_kernel_serial, dim3((uint32_t)blocks), dim3(256), 0, s, a.crcs, a.n_groups,
                           a.per_group, a.m_unit, a.out);
    }
    return hipGetLastError();
}



hipError_t launch_range_flat(const RangeLaunch& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(range_flat_kernel, dim3(a.blocks), dim3(64 * kFlatWaves), 0, s, a);
    return hipGetLastError();
}

hipError_t upload_x2k(const uint32_t* t64) { return hipMemcpyToSymbol(HIP_SYMBOL(c_x2k), t64, sizeof(X2k)); }

hipError_t launch_shift(const uint32_t* crcs, const uint64_t* shift_bytes, uint64_t n, uint32_t* out,
                        hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(shift_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, crcs, shift_bytes, n, out);
    return hipGetLastError();
}

hipError_t launch_log_insert(const LogLaunch& a, hipStream_t s) {
    if (a.n_pieces == 0) return hipSuccess;
    if (a.n_segs == 0 || a.n_segs > kInsertBlocks) return hipErrorInvalidValue;
    hipLaunchKernelGGL(log_insert_kernel, dim3(a.n_segs), dim3(kInsertThreads), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_log_pages(const LogLaunch& a, hipStream_t s) {
    if (a.n_pieces == 0) return hipSuccess;
#define CC_GCASE(MM)                                                                                        \
    case MM:                                                                                                \
        if (a.delta)                                                                                        \
            hipLaunchKernelGGL((log_pages_kernel<MM, true>), dim3(a.blocks), dim3(64 * log_waves(MM, true)), 0, s,  \
                               a);                                                                          \
        else                                                                                                \
            hipLaunchKernelGGL((log_pages_kernel<MM, false>), dim3(a.blocks), dim3(64 * log_waves(MM, false)), 0, \
                               s, a);                                                                       \
        break;
    switch (a.page_bytes / kWaveBytes) {
        CC_GCASE(1)
        CC_GCASE(2)
        CC_GCASE(4)
        CC_GCASE(8)
        CC_GCASE(16)
        CC_GCASE(32)
        default: return hipErrorInvalidValue;
    }
#undef CC_GCASE
    return hipGetLastError();
}

hipError_t launch_log_small(const LogLaunch& a, hipStream_t s) {
    if (a.n_updates == 0 || a.n_updates > 64 || a.slots > 2) return hipErrorInvalidValue;
#define CC_SMCASE(MM)                                                                                         \
    case MM:                                                                                                  \
        if (a.delta)                                                                                          \
            hipLaunchKernelGGL((log_small_kernel<MM, true>), dim3(a.blocks), dim3(64 * log_small_waves(MM, true)), 0, s, \
                               a);                                                                            \
        else                                                                                                  \
            hipLaunchKernelGGL((log_small_kernel<MM, false>), dim3(a.blocks), dim3(64 * log_small_waves(MM, false)), 0, \
                               s, a);                                                                         \
        break;
    switch (a.page_bytes / kWaveBytes) {
        CC_SMCASE(1)
        CC_SMCASE(2)
        CC_SMCASE(4)
        CC_SMCASE(8)
        CC_SMCASE(16)
        CC_SMCASE(32)
        default: return hipErrorInvalidValue;
    }
#undef CC_SMCASE
    return hipGetLastError();
}


hipError_t launch_page_list_probe(const PageListProbeLaunch& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(page_list_probe_kernel<16>, dim3(a.blocks), dim3(64 * kListProbeWaves), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_log_probe(const LogProbeLaunch& a, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(log_probe_kernel<16>, dim3(a.blocks), dim3(64 * kLogWavesFull), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_read_verify_small(const ReadVerifyLaunch& a, hipStream_t s) {
    if (a.n_reads == 0 || a.n_reads > 64) return hipErrorInvalidValue;
#define CC_SCASE(MM) \
    case MM: hipLaunchKernelGGL((read_verify_small_kernel<MM>), dim3(a.blocks), dim3(64 * kRvWaves), 0, s, a); break;
    switch (a.page_bytes / kWaveBytes) {
        CC_SCASE(1)
        CC_SCASE(2)
        CC_SCASE(4)
        CC_SCASE(8)
        CC_SCASE(16)
        CC_SCASE(32)
        default: return hipErrorInvalidValue;
    }
#undef CC_SCASE
    return hipGetLastError();
}

hipError_t launch_read_verify(const ReadVerifyLaunch& a, hipStream_t s) {
    if (a.n_reads == 0) return hipSuccess;
#define CC_RCASE(MM) \
    case MM: hipLaunchKernelGGL((read_verify_kernel<MM>), dim3(a.blocks), dim3(64 * kRvWaves), 0, s, a); break;
    switch (a.page_bytes / kWaveBytes) {
        CC_RCASE(1)
        CC_RCASE(2)
        CC_RCASE(4)
        CC_RCASE(8)
        CC_RCASE(16)
        CC_RCASE(32)
        default: return hipErrorInvalidValue;
    }
#undef CC_RCASE
    return hipGetLastError();
}

hipError_t launch_epilogue(const EpilogueLaunch& a, hipStream_t s) {
    if (a.n_chunks == 0) return hipSuccess;
    const uint64_t blocks = a.n_chunks < 8192 ? a.n_chunks : 8192;
    hipLaunchKernelGGL(epilogue_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_xpow8(const uint64_t* nbytes, uint64_t n, uint32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(xpow8_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, nbytes, n, out);
    return hipGetLastError();
}

hipError_t launch_combine(const uint32_t* a, const uint32_t* b, uint32_t m_len_b, uint64_t n, uint32_t* out,
                          hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(combine_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, a, b, m_len_b, n, out);
    return hipGetLastError();
}

hipError_t launch_xor_fold(const uint32_t* gathered, uint32_t nranks, uint64_t n, uint32_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(xor_fold_kernel, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, gathered, nranks, n, out);
    return hipGetLastError();
}

hipError_t launch_digest(const uint32_t* crcs, const uint64_t* after_bytes, const uint32_t* group, uint64_t n,
                         uint32_t* digest, hipStream_t s) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 3) / 4;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(digest_kernel, dim3((uint32_t)blocks), dim3(256), 0, s, crcs, after_bytes, group, n, digest);
    return hipGetLastError();
}

}  // namespace cc
