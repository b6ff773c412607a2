// curve_amd/csrc/kernels.h -- internal launcher interface between engine.hip
// (C ABI, device contexts) and kernels.hip (gfx950 kernels).  Not exported.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cc {

// LDS image geometry of the page kernel (see DESIGN.md "LDS image").
constexpr uint32_t kLdsBytes = 163840;  // all 160 KiB of a CU's LDS
// The device image is the LDS image followed by the x^(-8t) * x^i product table
// (kXinvEntries x 32 words).
constexpr uint32_t kFinBase = 131072;   // per-lane final-shift nibble tables [128K, 160K)
constexpr uint32_t kWordsPerWaveStep = 64;  // one dword per lane per step
constexpr uint32_t kWaveBytes = 256;        // bytes consumed per wave step
constexpr int kWavesPerBlock = 8;  // waves per CU (one workgroup per CU: the LDS image fills it); 8 beat 16 by 4-5 %
constexpr int kBlockThreads = 64 * kWavesPerBlock;
constexpr uint32_t kDynHeads = 8;  // dynamic-tail counters of the page kernel: one per XCD
constexpr uint32_t kDynHeadStride = 16;  // 128 bytes between heads: one cache line each
constexpr uint32_t kDynCtrBytes = kDynHeads * kDynHeadStride * 8;
constexpr uint32_t kDynCtrWords64 = kDynHeads * kDynHeadStride;  // the heads as uint64 words
// A stream's tail-counter block: two slot sets of heads; a launch pulls from
// one and zeroes the other for the stream's next launch (engine.hip tail_block).
constexpr uint32_t kTailBlockWords64 = 2 * kDynCtrWords64;
constexpr uint32_t kTailBlockBytes = kTailBlockWords64 * 8;

// Host builder of the 160 KiB LDS image (engine.hip).
void build_lds_image(uint32_t* image /* kLdsBytes/4 words */);

// Verify outputs: mismatch count, first bad page, and (optional) the list of
// bad page indices (unordered, at most max_list kept; count may exceed it).
struct VerifySink {
    unsigned long long* bad_count;
    unsigned long long* first_bad;
    unsigned long long* list;
    unsigned long long max_list;
};

struct PageLaunch {
    const uint32_t* pages;
    uint64_t n_pages;
    uint32_t words_per_lane;  // page_bytes / 256
    const void* image;        // device copy of the LDS image
    uint32_t kconst;          // V-domain correction for this page size
    uint32_t* out;            // compute: CRC per page
    const uint32_t* expected; // verify: expected CRC per page
    VerifySink sink;          // verify only
    int blocks;
    uint32_t tile_shift;      // 2^tile_shift consecutive pages per wave tile (0..6)
    // dynamic tail: null = every tile in the strided static walk; else tiles
    // [static_tiles, all) are handed out through this zeroed counter
    unsigned long long* dyn_ctr;  // kDynHeads counters, kDynHeadStride words apart (zeroed before the launch)
    uint64_t static_tiles;
    // non-null: dyn_ctr is one slot set of the stream's tail block and this the
    // other, which the launch zeroes for the stream's next launch
    unsigned long long* dyn_next;
    // fused metapages (cc_pool_scan_dev when metapage size == page size): n_meta
    // more pages of the same size, appended to the dynamic tail as chunks of their own
    const uint32_t* meta_pages;
    uint64_t n_meta;
    uint32_t* meta_out;
    // block 0 zeroes these word ranges before its walk (stream-ordered for the
    // kernels after it: the next launch's tail counter, a digest to XOR into)
    uint32_t* zero[2];
    uint64_t zero_words[2];
    // non-null: timing events carried by the kernel's own dispatch
    // (hipExtLaunchKernel), so timing it adds no marker packets to the stream
    hipEvent_t ev_begin, ev_end;
};

hipError_t launch_page_crc(const PageLaunch& a, hipStream_t s);
// engine.hip, for cc_pool_scan_dev: metapage launch (clears the data launch's
// tail counter and the digest) then the data launch, bracketed by the events
int pool_page_launches(const void* d_data, uint64_t n_data_pages, uint32_t page_bytes, uint32_t* d_page_crcs,
                       const void* d_meta, uint64_t n_meta, uint32_t meta_bytes, uint32_t* d_meta_crcs,
                       uint32_t* d_digest, uint64_t digest_words, hipStream_t s, void* ev_begin, void* ev_end);
hipError_t launch_read_probe(const void* buf, uint64_t bytes, uint32_t* sink, int blocks, hipStream_t s);
hipError_t launch_page_verify(const PageLaunch& a, hipStream_t s);
// the page kernel with its CRC arithmetic replaced by a rotate-XOR (4 KiB pages):
// the same schedule, loads and stores -- the ceiling the real kernel is held to
hipError_t launch_page_load_probe(const PageLaunch& a, hipStream_t s);
// the scan step's metapage pass (a separate instantiation, same code as compute)
hipError_t launch_page_meta(const PageLaunch& a, hipStream_t s);

struct FoldLaunch {
    const uint32_t* crcs;
    uint64_t n_groups;
    uint32_t per_group;
    uint32_t m_unit;      // x^(8*unit_bytes) mod P
    uint32_t m_tree[7];   // x^(8*unit_bytes*q*2^t), t=0..5 (fast path, q = per_group/64)
    uint32_t* out;
};
hipError_t launch_fold(const FoldLaunch& a, hipStream_t s);

// x^(2^k) mod P table for the shift kernel, uploaded once per device.
hipError_t upload_x2k(const uint32_t* t64);

hipError_t launch_shift(const uint32_t* crcs, const uint64_t* shift_bytes, uint64_t n,
                        uint32_t* out, hipStream_t s);

struct UpdateDesc {
    uint64_t dst, src;
    uint32_t len, reserved;
};

// Write-log path (cc_apply_log_dev): every update of an ORDERED log becomes
// `slots` pieces, one per page it touches; an open-addressing table keyed by
// page groups them (each entry heads a linked list of the page's pieces) with
// no sort; one wave per touched page (balanced over the grid) then applies its
// pieces in log order in registers, stores the changed rows and rehashes it.
// A page with more than 64 pieces is finished by its wave replaying the log.
constexpr uint32_t kNoPiece = 0xFFFFFFFFu;
constexpr uint32_t kInsertThreads = 512;   // pieces per insert chunk, one a thread (512: every CU busy; profiles/write_log_insert_threads_ab_r04.txt)
constexpr uint32_t kInsertBlocks = 256;    // insert blocks at most (grid-stride over chunks): head segments
constexpr int kLogWaves = 12;  // waves per CU of the write-log page kernel at 8 KiB pages (A/B at 4 KiB, round 1: 12 beats 8 by ~6 %)
constexpr int kLogWavesFull = 16;   // full mode, pages <= 4 KiB: 103 VGPRs since the row offsets went into the offset field
constexpr int kLogWavesDelta = 16;  // delta mode, pages <= 4 KiB: 120 VGPRs at 16 waves (was 12 waves: 129 would spill)
// waves per workgroup of log_pages_kernel<M, Delta>
constexpr int log_waves(int m, bool delta) { return m > 16 ? kLogWaves : (delta ? kLogWavesDelta : kLogWavesFull); }
// waves per workgroup of log_small_kernel<M, Delta>
constexpr int log_small_waves(int m, bool delta) { return (!delta && m <= 16) ? kLogWavesFull : kLogWaves; }
// The NEXT batch's grouping, done by the page kernel of the current one
// (cc_apply_logs_dev): its pieces go into its own table and head segments, in
// the kernel's tail -- a workgroup done with its pages takes chunks of the next
// batch (one counter) while the slower ones finish -- so the kernel boundary
// before the next page kernel is the only barrier the next batch needs.  The
// fields insert_piece reads, for that batch; n_pieces = 0: nothing to insert.
// chunks a workgroup claims per take of the tail grouping's counter (A/B: 2 beats
// 1 by ~0.6 %: half as many, earlier-finishing workgroups do the inserts); a
// compile-time knob for the A/B builds
#ifndef CC_GROUP_TAKE
#define CC_GROUP_TAKE 2
#endif
constexpr uint32_t kGroupTake = CC_GROUP_TAKE;
struct LogInsert {
    const UpdateDesc* upd;
    uint64_t n_pieces;
    uint64_t pool_bytes;
    uint32_t page_bytes, max_len, slots, table_mask;
    uint64_t* table;
    uint32_t* next;
    uint32_t* heads;            // one segment of seg_cap records per block of the inserting kernel
    uint32_t* seg_count;        // [gridDim.x of the inserting kernel]
    uint32_t seg_cap;           // >= rounds x the block's threads
    uint32_t rounds;            // chunks (of the block's threads) one workgroup may take: a multiple of kGroupTake
    unsigned long long* take;   // the chunk counter, zero at launch (the grouping kernel before zeroed it)
    unsigned long long* zero;   // the counter the grouping kernel after next takes from: zeroed here
};
struct LogLaunch {
    unsigned char* pool;
    uint64_t pool_bytes;
    const unsigned char* src;
    const UpdateDesc* upd;
    uint64_t n_updates;
    uint32_t page_bytes;
    uint32_t max_len;
    uint32_t slots;             // pieces per update: (max_len - 1) / page_bytes + 2
    uint64_t n_pieces;          // n_updates * slots
    uint64_t* table;            // [table_mask + 1] {page + 1, piece + 1} of the page's list head (0 = empty)
    uint32_t table_mask;
    uint32_t* next;             // [n_pieces] next piece of the same page (kNoPiece = end)
    // head records {table slot, claiming piece} of the touched pages (uint2), in
    // one segment of seg_cap records per insert block: block b's at b * seg_cap,
    // seg_count[b] of them (written by the insert, no clearing needed)
    uint32_t* heads;
    uint32_t* seg_count;        // [n_segs]
    uint32_t seg_cap;
    uint32_t n_segs;            // insert blocks (<= kInsertBlocks)
    int clear_table;            // the table is the engine's per-stream one: the page kernel leaves it zero
    const void* image;
    uint32_t kconst;
    uint32_t* page_crcs;        // out; in delta mode also in (the CRCs before the batch)
    int blocks;
    int delta;                  // 1: update the stored CRCs through linearity (reads touched rows only)
    LogInsert nx;               // the next batch's grouping, in this batch's page kernel (launch_log_pages)
    unsigned long long* zero_ctrs;  // log_insert_kernel zeroes these 3 words (the queue's chunk counters) or null
};
hipError_t launch_log_insert(const LogLaunch& a, hipStream_t s);
hipError_t launch_log_pages(const LogLaunch& a, hipStream_t s);
// <= 64 writes of <= 2 pieces each in one launch (no table, no insert)
hipError_t launch_log_small(const LogLaunch& a, hipStream_t s);
// diagnostic: the write log's page traffic alone (4 KiB pages; kernels.hip log_probe_kernel)
struct LogProbeDesc {
    uint64_t page;      // touched page
    uint64_t src_off;   // source byte of page byte 0 (mod 2^64) when covered != 0
    uint32_t covered;   // rows read from the source (the page's only piece covers them whole)
    uint32_t dirty;     // rows stored back
};
struct LogProbeLaunch {
    unsigned char* pool;
    uint64_t pool_pages;  // a descriptor naming a page >= this touches nothing (reads page 0, stores none)
    const unsigned char* src;
    const LogProbeDesc* desc;
    uint64_t n;
    uint32_t* out;  // [n]
    int blocks;
};
hipError_t launch_log_probe(const LogProbeLaunch& a, hipStream_t s);
// diagnostic: the read traffic of a page list alone (4 KiB pages; kernels.hip page_list_probe_kernel)
struct PageListProbeLaunch {
    const uint32_t* pool;
    uint64_t pool_pages;  // an index >= this reads page 0 instead (never outside the pool)
    const uint64_t* pages;
    uint64_t n;
    uint32_t* out;  // [n]
    int blocks;
    // dynamic tail, as verify-on-read's: the last 1/16 of the list in 32-page
    // chunks through *dyn_ctr (zero at launch); the launch zeroes *dyn_next (the
    // stream's other slot set) for the next one.  Null: a static split only.
    unsigned long long* dyn_ctr;
    unsigned long long* dyn_next;
};
hipError_t launch_page_list_probe(const PageListProbeLaunch& a, hipStream_t s);

struct RangeDesc {
    uint64_t off, len;
};

// Verify-on-read for a batch of reads (cc_verify_reads_dev): every page a read
// touches is a "slot"; the batch's slots are read 0's pages, then read 1's, ...;
// ONE launch on the range kernel's schedule: the waves count kRangeTiles tiles
// of reads themselves (epoch-tagged words in the stream's range scratch) and
// each rehashes an equal share of the slots, the last 1/16 dynamically.
struct ReadVerifyLaunch {
    const uint32_t* pool;
    uint64_t pool_bytes;
    uint32_t page_bytes;
    uint32_t page_shift;        // log2(page_bytes)
    const RangeDesc* reads;
    uint64_t n_reads;
    const uint32_t* page_crcs;  // stored CRC per pool page
    uint32_t* bad_per_read;     // [n_reads] += mismatching pages; UINT32_MAX for a read beyond the pool
    unsigned long long* bad_total;
    uint64_t* tiles;            // [kReadTiles] epoch << 40 | pages of the tile
    unsigned long long* tail;   // dynamic-tail counter slots (epoch % 2: this call's; the other zeroed for the next)
    uint32_t epoch;
    const void* image;
    uint32_t kconst;
    int blocks;
};
hipError_t launch_read_verify(const ReadVerifyLaunch& a, hipStream_t s);
// <= 64 reads in one launch (no tiles; pages split over waves)
hipError_t launch_read_verify_small(const ReadVerifyLaunch& a, hipStream_t s);
// CRC32C (butil Value) of arbitrary byte ranges of one device buffer, on the
// flat block schedule, ONE launch: range_flat_kernel counts the
// 4 KiB blocks of kRangeTiles contiguous tiles of the batch itself (epoch-tagged
// words in `tiles`), gives every wave an equal share of the blocks, and ranges
// cut by a share boundary meet in their accumulator pair (acc[2r], acc[2r+1]).
// The per-stream scratch (engine.hip range_work) is zero on first use and left
// so by every launch: tiles are overwritten each call (the epoch tells this
// call's words), the accumulators self-reset and each call zeroes the tail
// counter slot the next call uses.
constexpr uint32_t kRangeTiles = 1024;
// verify on read counts its reads in fewer tiles (half the words every wave
// polls; A/B round 6, profiles/range_tiles_ab_r06.txt); the scratch holds kRangeTiles
constexpr uint32_t kReadTiles = 512;
static_assert(kReadTiles <= kRangeTiles && kReadTiles % 64 == 0, "read tiles share the range scratch");
struct RangeLaunch {
    const unsigned char* buf;
    const RangeDesc* ranges;
    uint64_t n;
    uint64_t* tiles;             // [kRangeTiles] epoch << 40 | blocks of the tile
    unsigned long long* tail;    // dynamic-tail counter slots (epoch % 2: this call's; the other zeroed for the next)
    uint32_t* acc;               // [2 n] split-range XOR / block-count pairs, zero at rest
    uint32_t epoch;              // 1 .. 2^24 - 1, the next one (parity alternating) per call on the scratch
    const void* image;
    uint32_t* out;
    int blocks;
};
hipError_t launch_range_flat(const RangeLaunch& a, hipStream_t s);
// x^(-8t) mod P for t = 0..kXinvEntries-1 (undoing the zero pad after a range in its last 4 KiB block)
constexpr uint32_t kXinvEntries = 4100;  // x^(-8t), t < 4096 + 4: the zero pad after a range in its last 4 KiB block

// Fused scan epilogue: one 256-thread block per chunk.
struct EpilogueLaunch {
    const uint32_t* page_crcs;  // [n_chunks * pages_per_chunk]
    const uint32_t* meta_crcs;  // [n_chunks]
    uint64_t n_chunks;
    uint32_t pages_per_chunk;   // 256 * q
    uint32_t q;                 // pages per thread
    uint32_t slice_shift;       // log2(threads per slice)
    const uint32_t* mtab;       // product tables [10][4][256]: 0 = x^(8 page), 1..8 = level k-1, 9 = chunk
    uint32_t* slice_crcs;       // [n_chunks * 256 >> slice_shift]
    uint32_t* file_crcs;        // [n_chunks] (may be null)
    const uint32_t* after_mult; // digest inputs x^(8 * after_bytes) (all three null = no digest)
    const uint32_t* group;
    uint32_t* digest;
};
hipError_t launch_epilogue(const EpilogueLaunch& a, hipStream_t s);
hipError_t launch_xpow8(const uint64_t* nbytes, uint64_t n, uint32_t* out, hipStream_t s);

hipError_t launch_combine(const uint32_t* a, const uint32_t* b, uint32_t m_len_b, uint64_t n, uint32_t* out,
                          hipStream_t s);

hipError_t launch_digest(const uint32_t* crcs, const uint64_t* after_bytes, const uint32_t* group, uint64_t n,
                         uint32_t* digest, hipStream_t s);

// out[i] = XOR_r gathered[r*n + i]  (digest fold after the RCCL all-gather)
hipError_t launch_xor_fold(const uint32_t* gathered, uint32_t nranks, uint64_t n, uint32_t* out, hipStream_t s);

}  // namespace cc
