/*
 * include/curve_crc.h -- C ABI of libcurvecrc, the MI355X-native chunk-checksum
 * engine for Curve's per-page CRC32C integrity path.
 *
 * Plain C: no C++ or torch types cross this boundary; pointers + sizes only.
 * Every entry point cites the reference interface it replaces (paths relative
 * to the opencurve/curve tree).
 *
 * Conventions
 *   - CRC values are CRC-32C (Castagnoli, reflected poly 0x82F63B78) with
 *     butil semantics: crc32c_extend(c, A||B) == crc32c_extend(crc32c_extend(c, A), B),
 *     crc32c_value(p, n) == crc32c_extend(0, p, n), value of the empty buffer = 0.
 *   - Functions returning `int` return CC_OK (0) or a negative CC_E* code.
 *   - `*_dev` calls take caller-owned device memory on the calling thread's
 *     current HIP device, enqueue on `stream` (a hipStream_t, NULL = default
 *     stream) and return without synchronising.  They never fall back to the
 *     CPU: with no usable GPU they return CC_ENODEV.
 */
#ifndef CURVE_CRC_H_
#define CURVE_CRC_H_

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h> /* struct iovec */

#ifdef __cplusplus
extern "C" {
#endif

#define CC_OK 0
#define CC_EINVAL (-22)   /* bad argument (size, alignment, null pointer) */
#define CC_ENODEV (-19)   /* no HIP device / device code unavailable */
#define CC_ENOMEM (-12)   /* device or pinned-host allocation failed */
#define CC_EHIP (-5)      /* a HIP runtime call failed */
#define CC_ECORRUPT (-74) /* verify found mismatching pages (host verify) */
#define CC_EIO (-5001)    /* reading or writing a file failed (errno is kept where the call says so) */
#define CC_ESTALE (-116)  /* a per-page CRC table no longer describes its chunk (sn / write generation) */
#define CC_ETIMEDOUT (-110) /* a bounded wait expired (communicator init whose peers never joined) */
#define CC_EFORMAT (-5002) /* a chunk file's size is not metapage + chunk (CSErrorCode::FileFormatError,
                              chunkserver_chunkfile.cpp:233-238) */

/* ------------------------------------------------------------------------
 * CPU primitive -- drop-in for the inline header src/common/crc32.h
 * ------------------------------------------------------------------------ */

/* Replaces curve::common::CRC32(const char*, size_t)  (src/common/crc32.h:40-42)
 * = butil::crc32c::Value.  Also nebd::common::CRC32 (nebd/src/common/crc32.h). */
uint32_t crc32c_value(const void* p, size_t n);

/* Replaces curve::common::CRC32(uint32_t, const char*, size_t) (src/common/crc32.h:53-55)
 * = butil::crc32c::Extend.  Pure, reentrant, any length/alignment. */
uint32_t crc32c_extend(uint32_t crc, const void* p, size_t n);

/* GF(2) algebra (new; needed to derive the reference digests from page CRCs).
 * crc32c_combine(V(A), V(B), |B|) == V(A||B)  (zlib crc32_combine identity).
 * crc32c_shift(c, n) multiplies the 32-bit register by x^(8n) mod P. */
uint32_t crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
uint32_t crc32c_shift(uint32_t crc, uint64_t nbytes);
/* V(n zero bytes); e.g. crc32c_zeros(4096) == 0x98F94189, the CRC of every page
 * of a freshly formatted pool chunk (src/tools/curve_format_main.cpp:132). */
uint32_t crc32c_zeros(uint64_t nbytes);

/* CRC32C over a scattered buffer: crc32c_extend(crc, iov[0] || iov[1] || ...).
 * Replaces braft::crc32(const butil::IOBuf&) -- the checksum CurveSegment::append
 * takes over every WAL entry's data IOBuf (src/chunkserver/raftlog/curve_segment.cpp:405,
 * get_checksum :283-288) -- which walks the IOBuf's blocks and extends one CRC
 * across them.  Fragments of any length/alignment (0 allowed). */
uint32_t crc32c_extend_iov(uint32_t crc, const struct iovec* iov, size_t n);

/* Fold n page CRCs (each over page_bytes) into the CRC of their concatenation. */
uint32_t cc_fold_host(const uint32_t* page_crcs, uint64_t n, uint64_t page_bytes);

/* Batched host fold: out[s] = CRC of pages s*pages_per_slice ..
 * (s+1)*pages_per_slice - 1, for n_pages / pages_per_slice slices; e.g. the
 * 1024 page CRCs of a 4 MiB scan slice -> its ScanMap.crc (proto/scan.proto:28,
 * op_request.cpp:794).  n_pages must be a multiple of pages_per_slice. */
int cc_slice_fold(const uint32_t* page_crcs, uint64_t n_pages, uint32_t pages_per_slice, uint32_t page_bytes,
                  uint32_t* out);

/* ------------------------------------------------------------------------
 * Engine lifetime -- created next to ScanManager::Init and torn down at
 * ChunkServer::Fini (src/chunkserver/chunkserver.cpp:298-303, :455).
 * Optional: device calls initialise per-device state lazily.
 * ------------------------------------------------------------------------ */
typedef struct cc_opts {
    uint32_t page_bytes;     /* default 4096 (conf/chunkserver.conf:22 blocksize) */
    uint32_t slice_bytes;    /* default 4 MiB (copyset.scan_size_byte, conf/chunkserver.conf:114) */
    uint64_t staging_bytes;  /* pinned host staging per device for *_host calls, default 256 MiB */
} cc_opts;

int cc_engine_init(const cc_opts* opts);  /* NULL = defaults */
int cc_engine_fini(void);
/* Free the device memory the engine caches per stream on the calling thread's
 * device: the write log's hash tables (cc_apply_log_dev) and the range /
 * verify-on-read scratch (cc_crc_ranges_dev, cc_verify_reads_dev); the next
 * call re-creates what it needs.  The entries are detached under the engine's
 * locks, then the call waits for the device to be idle WITHOUT holding them
 * (other threads' calls proceed meanwhile) and frees them.  Entries of
 * hipStreamPerThread are also dropped when their thread exits. */
int cc_engine_trim(void);
/* Diagnostic: the per-stream entries (tail blocks, write-log tables, range
 * scratch) the engine holds on the calling thread's device right now. */
uint64_t cc_engine_stream_entries(void);
int cc_device_count(void);
const char* cc_strerror(int code);
const char* cc_version(void);

/* ------------------------------------------------------------------------
 * Device batch calls -- the hot path (replace the CRC32() loops of the scan
 * hasher, op_request.cpp:794/:847, and of the chunk/copyset hashers,
 * chunkserver_chunkfile.cpp:805, copyset_node.cpp:964).
 * ------------------------------------------------------------------------ */

/* d_out[i] = crc32c_value(d_pages + i*page_bytes, page_bytes).
 * page_bytes: multiple of 256, 256..1 MiB.  d_pages 4-byte aligned. */
int cc_page_crc_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes,
                    uint32_t* d_out, void* stream);

/* Recompute and compare against d_expected.  *d_bad_count += mismatches;
 * *d_first_bad = min(*d_first_bad, first mismatching page index).  The caller
 * zeroes d_bad_count and sets d_first_bad to UINT64_MAX before the call. */
int cc_page_verify_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes,
                       const uint32_t* d_expected, uint64_t* d_bad_count,
                       uint64_t* d_first_bad, void* stream);

/* cc_page_verify_dev plus the indices of the mismatching pages: the first
 * min(count, max_bad_pages) of them land in d_bad_pages[*d_bad_count_before ..]
 * in no particular order (the caller sorts).  Lets a scan report every bad page
 * (SURVEY §8d C1 "verify must flag exactly those") without a second pass.
 * d_bad_pages may be NULL only when max_bad_pages == 0. */
int cc_page_verify_list_dev(const void* d_pages, uint64_t n_pages, uint32_t page_bytes,
                            const uint32_t* d_expected, uint64_t* d_bad_count,
                            uint64_t* d_first_bad, uint64_t* d_bad_pages,
                            uint64_t max_bad_pages, void* stream);

/* Group fold: d_out[g] = CRC of the concatenation of units g*per_group ..
 * g*per_group+per_group-1, each unit_bytes long, from their CRCs d_crcs.
 * E.g. 1024 page CRCs -> one 4 MiB ScanMap.crc (proto/scan.proto:28). */
int cc_fold_dev(const uint32_t* d_crcs, uint64_t n_groups, uint32_t per_group,
                uint64_t unit_bytes, uint32_t* d_out, void* stream);

/* A byte range of a device buffer. */
typedef struct cc_range {
    uint64_t off;
    uint64_t len;
} cc_range;

/* d_out[i] = crc32c_value(d_buf + off_i, len_i) for arbitrary offsets,
 * alignments and lengths (0 allowed), e.g. raft WAL entries on replay -- the
 * data and header checksums CurveSegment::_load_entry verifies with
 * braft::crc32 (= butil::crc32c::Value), src/chunkserver/raftlog/curve_segment.cpp:307-371 --
 * or GetChunkHash's raw-file range (chunkserver_chunkfile.cpp:785-811).  The
 * batch is one stream of 4 KiB blocks split evenly over the device whatever
 * the range sizes (a range cut between waves is hashed in segments and
 * recombined), the last 1/32 handed out dynamically: ranges of any size mix
 * freely.  ONE launch: the waves count the batch's tiles themselves.  The
 * engine keeps scratch per stream for it (tile words, tail counters and the
 * split ranges' accumulator pairs: 8 B x the next power of two >= n, at least
 * 64 Ki pairs, plus ~9 KiB; at most 32 MiB + 9 KiB a stream -- a batch of more
 * than 4 Mi ranges takes scratch of its own for the call -- for at most 256
 * streams; shared with cc_verify_reads_dev; cc_engine_trim releases it).  The
 * scratch is left zero by every launch that completes; after a device fault
 * the context is unusable anyway (HIP errors are sticky) -- call
 * cc_engine_fini, or cc_engine_trim, before using the engine again. */
int cc_crc_ranges_dev(const void* d_buf, const cc_range* d_ranges, uint64_t n, uint32_t* d_out,
                      void* stream);

/* Host-resident variant for many separate buffers (e.g. the data of a batch
 * of WAL entries read from a segment file, CurveSegment::_load_entry,
 * curve_segment.cpp:307-371): h_out[i] = crc32c_value(h_bufs[i], h_lens[i]).
 * Buffers are packed into the pinned staging ring and hashed on the device by
 * the range kernel; a buffer larger than a staging slot is hashed in pieces
 * combined on the host.  Blocking, thread-safe. */
int cc_crc_bufs_host(const void* const* h_bufs, const uint64_t* h_lens, uint64_t n, uint32_t* h_out);

/* d_out[i] = x^(8 * d_nbytes[i]) mod P: the multiplier that shifts a CRC by
 * d_nbytes[i] bytes (precompute once per static pool layout for the epilogue's
 * digest). */
int cc_xpow8_dev(const uint64_t* d_nbytes, uint64_t n, uint32_t* d_out, void* stream);

/* Fused scan epilogue for whole chunks, ONE launch (replaces fold + fold +
 * combine + digest): from the page CRCs of n_chunks chunks (pages_per_chunk
 * each, contiguous) and their metapage CRCs produce
 *   d_slice_crcs[c*S + k]  S = pages_per_chunk / pages_per_slice   (ScanMap.crc)
 *   d_file_crcs[c]         CRC of metapage || data  (NULL = skip)
 *   d_digest[d_group[c]] ^= file CRC * d_after_mult[c]             (all three NULL = skip)
 * with d_after_mult[c] = x^(8 * bytes after file c in its copyset's sorted-name
 * chain) from cc_xpow8_dev.  Geometry: pages_per_chunk = 256*q; pages_per_slice
 * = q * 2^j, j in [0, 8] (16 MiB chunks, 4 KiB pages, 4 MiB slices: q = 16,
 * j = 6); CC_EINVAL otherwise. */
int cc_scan_epilogue_dev(const uint32_t* d_page_crcs, const uint32_t* d_meta_crcs, uint64_t n_chunks,
                         uint32_t pages_per_chunk, uint32_t page_bytes, uint32_t pages_per_slice,
                         uint32_t* d_slice_crcs, uint32_t* d_file_crcs, const uint32_t* d_after_mult,
                         const uint32_t* d_group, uint32_t* d_digest, void* stream);

/* Linear-domain digest contributions (per-copyset digest):
 * d_out[i] = crc32c_shift(d_crcs[i], d_shift_bytes[i]).  XOR of contributions
 * plus a length-only constant reproduces CopysetNode::GetHash's chain. */
int cc_shift_dev(const uint32_t* d_crcs, const uint64_t* d_shift_bytes, uint64_t n,
                 uint32_t* d_out, void* stream);

/* d_out[i] = crc32c_combine(d_a[i], d_b[i], len_b): e.g. a chunk FILE's CRC from
 * its metapage CRC and its 16 MiB data CRC (the file is metapage || data,
 * chunkserver_chunkfile.cpp:497-536 reads data at offset + metaPageSize). */
int cc_combine_dev(const uint32_t* d_a, const uint32_t* d_b, uint64_t len_b, uint64_t n,
                   uint32_t* d_out, void* stream);

/* Per-copyset digest partials: for each file i,
 *   d_digest[d_group[i]] ^= crc32c_shift(d_file_crcs[i], d_after_bytes[i])
 * where d_after_bytes[i] = bytes of the copyset's files that sort after file i
 * (CopysetNode::GetHash chains files in std::sort name order, copyset_node.cpp:938).
 * The XOR is order-free, so ranks holding disjoint file sets produce partials
 * whose XOR is exactly the reference's chained copyset hash.  d_digest is
 * caller-zeroed. */
int cc_digest_dev(const uint32_t* d_file_crcs, const uint64_t* d_after_bytes,
                  const uint32_t* d_group, uint64_t n_files, uint32_t* d_digest,
                  void* stream);

/* Device XOR fold of gathered digest partials: d_digest[i] = XOR over r <
 * nranks of d_gathered[r * n + i].  The local half of the per-copyset digest
 * exchange for callers that move the partials themselves (any
 * transport: RCCL all-gather, the MDS, a TCP store); cc_digest_allreduce_dev
 * runs it after its own RCCL all-gather. */
int cc_digest_fold_dev(const uint32_t* d_gathered, uint32_t nranks, uint64_t n, uint32_t* d_digest, void* stream);

/* ------------------------------------------------------------------------
 * Host-in / host-out convenience (blocking; thread-safe).  Starts and ends in
 * host memory like the reference's datastore read path (chunkserver_chunkfile.cpp:497-536).
 * ------------------------------------------------------------------------ */
/* h_out[i] = crc32c_value(h_pages + i*page_bytes, page_bytes).  A call of at
 * most 16 MiB (the scan op's shape: one 4 MiB slice or the 4 KiB metapage per
 * ScanChunkRequest, op_request.cpp:776-794, from up to wconcurrentapply.size =
 * 10 apply threads) runs on a LANE of its own -- device buffer, stream,
 * completion signal; up to 16 lanes per device, made on first demand, a caller
 * finding none idle waits -- so concurrent callers overlap their copies and
 * kernels.  A larger call takes the device's two-slot pinned staging ring,
 * held for the whole call.  Pinned input is DMA'd directly; pageable input is
 * copied through pinned staging.  The caller sleeps until done: a lane call on
 * a word its stream writes after the kernel (no HIP wait, so no thread spins
 * for it: ~10 us of process CPU for a 4 KiB call, ~40 us for 4 MiB), a large
 * call on a condition variable. */
int cc_page_crc_host(const void* h_pages, uint64_t n_pages, uint32_t page_bytes,
                     uint32_t* h_out);

/* One byte-range write into a device-resident pool (client partial write). */
typedef struct cc_update {
    uint64_t dst; /* byte offset in the pool */
    uint64_t src; /* byte offset in the source buffer */
    uint32_t len; /* bytes, >= 1 */
    uint32_t reserved;
} cc_update;

/* Client partial-write path (BASELINE config 3), the drop-in for the write
 * loop of WriteChunkRequest::OnApply -> CSChunkFile::Write (op_request.cpp:429-481,
 * chunkserver_chunkfile.cpp:287-427, which applies writes in raft-log order);
 * the per-page CRC table is new.  d_log[0..n) is the ORDERED write
 * log: entries may overlap, have any alignment and straddle pages; later
 * entries win.  Every entry becomes one piece per page it touches; the pieces
 * are grouped by page in a device hash table (one 64-bit CAS per piece: no
 * sort, no host planning), and one wave per touched page applies that page's
 * pieces in log order in registers, stores the changed 256-byte rows and
 * writes the page's new CRC to d_page_crcs (untouched pages keep theirs).
 * Two launches (insert, pages); a log of <= 64 entries no longer than a page
 * takes one.  The hash table is the engine's, one per stream, created (and
 * grown) on the stream on first use and left clear by every call, so no call
 * clears it; calls sharing a stream are serialised by the engine while they
 * enqueue.  Retained device memory: 8 B x the next power of two >= 8 x the
 * pieces (n_updates x ((max_len - 1) / page_bytes + 2)) per stream, at most
 * 64 MiB a stream (a log needing more takes a table for that call only), for
 * at most 256 streams; the null stream and hipStreamLegacy are one stream,
 * hipStreamPerThread counts once per calling thread (its entry is dropped when
 * the thread exits).  cc_engine_trim releases them.  Contract per entry: 1 <= len <= max_len and
 * dst + len <= pool_bytes -- an entry that breaks it is skipped whole (never
 * half-applied); d_src must not alias d_pool.  page_bytes = 256 * 2^k
 * (k = 0..5).  d_work: >= cc_apply_log_work_bytes(n, max_len, page_bytes) bytes
 * (the pieces' list links and the touched-page list; no clearing needed;
 * 0 = unsupported sizes: a table of more than 2^32 slots). */
uint64_t cc_apply_log_work_bytes(uint64_t n_updates, uint32_t max_len, uint32_t page_bytes);
int cc_apply_log_dev(void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const void* d_src,
                     const cc_update* d_log, uint64_t n_updates, uint32_t max_len, uint32_t* d_page_crcs,
                     void* d_work, uint64_t work_bytes, void* stream);

/* The same write log, with d_page_crcs[p] taken as the CRC of page p BEFORE
 * the batch and updated incrementally: V(new) = V(old) ^ raw(old ^ new) for
 * equal-length pages, so only the 256-byte rows the writes touch are read
 * (a page with several writes reads whole).  Identical output to
 * cc_apply_log_dev whenever the stored CRCs matched the pages; a page whose
 * stored CRC did not match (latent corruption) keeps mismatching after the
 * write instead of receiving a fresh CRC over the corrupt bytes.  Same
 * contract and work size as cc_apply_log_dev. */
int cc_apply_log_delta_dev(void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const void* d_src,
                           const cc_update* d_log, uint64_t n_updates, uint32_t max_len, uint32_t* d_page_crcs,
                           void* d_work, uint64_t work_bytes, void* stream);

/* A QUEUE of write logs applied in order, as n_batches cc_apply_log_dev calls
 * (delta = 0) or cc_apply_log_delta_dev calls (delta = 1) would be on `stream`:
 * the same pool bytes and page CRCs, bit for bit.  Pipelined: the page kernel
 * of batch k also groups batch k+1's pieces in its tail (workgroups done with
 * their pages insert them into the other half of the stream's engine table,
 * which is kept at twice the single-batch size, and the other of two work
 * regions), so only the first batch (and one after a <= 64-write batch, which
 * takes the one-launch path) pays the separate grouping launch and the kernel
 * boundary behind it.  `batches` is a
 * HOST array (its device pointers: as for cc_apply_log_dev, valid until the
 * stream has run the call's work); empty batches are skipped.  d_work: >=
 * cc_apply_logs_work_bytes(largest batch's n_updates, max_len, page_bytes).
 * A stream without an engine table (more than 256 streams hold one) takes one
 * call per batch.  Replaces a chunkserver's apply loop over its queued write
 * requests (ChunkOpRequest::OnApply per write, op_request.cpp:429-481). */
typedef struct cc_log_batch {
    const void* d_src;        /* device: the batch's data (its records' src offsets) */
    const cc_update* d_log;   /* device: the batch's records, log order */
    uint64_t n_updates;
} cc_log_batch;
uint64_t cc_apply_logs_work_bytes(uint64_t max_updates, uint32_t max_len, uint32_t page_bytes);
int cc_apply_logs_dev(void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const cc_log_batch* batches,
                      uint32_t n_batches, uint32_t max_len, uint32_t* d_page_crcs, int delta, void* d_work,
                      uint64_t work_bytes, void* stream);

/* Verify-on-read for a batch of datastore reads (the read path of
 * CSChunkFile::Read, chunkserver_chunkfile.cpp:497-536, which today returns the
 * bytes unchecked): every page that read i = d_reads[i] (pool byte range, any
 * offset/length; a partly covered page is verified whole) touches is rehashed
 * and compared with its stored CRC in d_page_crcs.  d_bad_per_read[i] += the
 * mismatching pages of read i (caller zeroes it; UINT32_MAX marks a read that
 * runs past the pool); *d_bad_total += all mismatches.  Every touched page is
 * one work slot and the slots are split evenly over the device, so reads of
 * any size mix freely.  page_bytes = 256 * 2^k (k = 0..5).  ONE launch on the
 * range kernel's schedule, using the stream's range scratch the engine keeps
 * (see cc_crc_ranges_dev).  d_work / work_bytes are kept for ABI stability
 * only: cc_verify_reads_work_bytes returns a constant 256 and d_work must be
 * non-NULL, but the engine does not touch it. */
uint64_t cc_verify_reads_work_bytes(uint64_t n_reads);
int cc_verify_reads_dev(const void* d_pool, uint64_t pool_bytes, uint32_t page_bytes, const cc_range* d_reads,
                        uint64_t n_reads, const uint32_t* d_page_crcs, uint32_t* d_bad_per_read,
                        uint64_t* d_bad_total, void* d_work, uint64_t work_bytes, void* stream);

/* One chunk file as the datastore holds it: metapage + data
 * (file = metapage || data, chunkserver_chunkfile.cpp:497-536). */
typedef struct cc_chunk_src {
    const void* meta; /* meta_bytes of host memory */
    const void* data; /* chunk_bytes of host memory */
} cc_chunk_src;

/* Streaming scan of host-resident chunk files (BASELINE config 4; the scan
 * hasher ScanChunkRequest::OnApply, op_request.cpp:769-820, for every scan op
 * of every chunk in ScanManager::ScanJobProcess order, scan_manager.cpp:250-283).
 * Per chunk c:
 *   h_meta_crcs[c]                          = CRC32(metapage)          (the readMetaPage op)
 *   h_slice_crcs[c*S + k], S = chunk/slice  = CRC32(data[k*slice, +slice))
 *   h_file_crcs[c]                          = CRC32(metapage || data)  (chunk-file CRC for
 *                                             the copyset chain, copyset_node.cpp:964)
 * Pipelined over two pinned staging slots and two HIP streams: the H2D copy of
 * batch i+1 overlaps the hashing of batch i.  Pinned (hipHostMalloc'ed or
 * registered) sources are DMA'd directly; pageable ones are staged by memcpy
 * (decided per buffer).  Any output pointer may be NULL.  Every chunk pointer
 * is checked before any work starts; on an error no batch of the call is left
 * in flight.  Blocking; thread-safe (per-device lock). */
int cc_scan_host(const cc_chunk_src* chunks, uint64_t n_chunks, uint32_t chunk_bytes,
                 uint32_t meta_bytes, uint32_t page_bytes, uint32_t slice_bytes,
                 uint32_t* h_meta_crcs, uint32_t* h_slice_crcs, uint32_t* h_file_crcs);

/* Per-copyset digest of a streamed scan (BASELINE config 4: "per-copyset
 * digest", CopysetNode::GetHash, copyset_node.cpp:925-975). */
typedef struct cc_scan_digest {
    const uint64_t* h_after_bytes; /* [n_chunks] bytes of the chunk's copyset that sort after its file */
    const uint32_t* h_group;       /* [n_chunks] copyset index of the chunk, < n_groups */
    uint64_t n_groups;
    uint32_t* h_digest;            /* [n_groups] out: XOR_c shift(file CRC of c, after bytes of c) over the
                                      call's chunks -- the copyset's GetHash value when all its files are in
                                      the call, else this call's partial (XOR partials of disjoint calls) */
} cc_scan_digest;

/* cc_scan_host plus the per-copyset digest, computed on the device by the
 * fused epilogue of every batch (no host pass over the file CRCs).  The chunk
 * list may mix pinned and pageable buffers.  dg NULL = cc_scan_host. */
int cc_scan_host_digest(const cc_chunk_src* chunks, uint64_t n_chunks, uint32_t chunk_bytes,
                        uint32_t meta_bytes, uint32_t page_bytes, uint32_t slice_bytes,
                        uint32_t* h_meta_crcs, uint32_t* h_slice_crcs, uint32_t* h_file_crcs,
                        const cc_scan_digest* dg);

/* Per-file outcome of cc_scan_files. */
typedef struct cc_file_result {
    int32_t status;    /* 0 ok; -errno from open/fstat/pread; CC_EFORMAT: size != meta+chunk
                          (CSChunkFile::Open's FileFormatError, chunkserver_chunkfile.cpp:233-238) */
    uint32_t meta_crc; /* CRC32(metapage) */
    uint32_t file_crc; /* CRC32(metapage || data) == CopysetNode::GetHash's per-file chain step */
    uint32_t reserved;
} cc_file_result;

/* Native datastore read path + scan: open/fstat/pread every chunk FILE (the
 * whole-file read of CopysetNode::GetHash, copyset_node.cpp:942-962, and the
 * metapage + data reads of the scan ops, chunkserver_chunkfile.cpp:497-548)
 * with `io_threads` reader threads (0 = cc_default_io_threads(); the caller is
 * one of them) into pinned staging, overlapping the reads of batch i+1 with the
 * H2D copy + kernels of batch i.  The readers are persistent: created once per
 * device on first use, parked between batches.  Outputs as cc_scan_host (slice
 * CRCs may be NULL); a file whose size is not meta_bytes + chunk_bytes gets
 * CC_EFORMAT, one that cannot be read -errno, and neither gets CRCs (the caller
 * chains such files on the CPU).  Blocking, thread-safe. */
int cc_scan_files(const char* const* paths, uint64_t n_files, uint32_t chunk_bytes, uint32_t meta_bytes,
                  uint32_t page_bytes, uint32_t slice_bytes, uint32_t io_threads, uint32_t* h_slice_crcs,
                  cc_file_result* h_results);
/* The reader count io_threads = 0 selects: half the CPUs this process may use
 * (its affinity mask, capped by the cgroup v2 cpu.max quota), in [2, 8]. */
uint32_t cc_default_io_threads(void);

/* ------------------------------------------------------------------------
 * Full-pool integrity scan sharded over the GPUs of a node (BASELINE config 5,
 * SURVEY §8e).  One process per GPU; each rank scans the chunk-index range it
 * owns with no data-path collective.  The only exchange is the per-copyset
 * digest of CopysetNode::GetHash (copyset_node.cpp:925-975): order-free XOR
 * partials, all-gathered over RCCL (xGMI) and XOR-folded on the device (XOR is
 * not an RCCL reduction op).  Per-chunk work is the scan hasher's
 * (ScanChunkRequest::OnApply, op_request.cpp:769-820, for every op that
 * ScanManager::ScanJobProcess schedules, scan_manager.cpp:210-296).
 * ------------------------------------------------------------------------ */
#define CC_ECOMM (-71) /* an RCCL call failed */
#define CC_COMM_ID_BYTES 128

typedef struct cc_comm cc_comm; /* opaque: an RCCL communicator + gather scratch */

/* Rank 0 creates the id and hands its CC_COMM_ID_BYTES bytes to every rank
 * out of band (the MDS, a TCP store, ...). */
int cc_comm_unique_id(void* id, size_t bytes);
/* Collective: every rank calls it with the same id, on the HIP device it owns
 * (the calling thread's current device).  Returns once all ranks joined, or
 * after `timeout_ms` (0 = $CC_COMM_INIT_TIMEOUT_MS, else 120 s) with
 * CC_ETIMEDOUT and the half-built communicator aborted: a rank whose peers
 * never arrive (one failed before reaching RCCL) is never blocked forever.
 * The communicator is RCCL non-blocking (ncclConfig_t.blocking = 0); every
 * call below waits for its own enqueue to settle.  The reference's exchange
 * (FollowScanMap, chunk_closure.cpp:82-104) is likewise bounded (retry x
 * timeout, scan_manager.cpp:285-289).  Ranks that disagree on whether their
 * init succeeded must all fall back together (bench.py / pool.agreed_comm
 * reduce a success flag before the first collective). */
int cc_comm_init_timeout(cc_comm** comm, int nranks, int rank, const void* id, size_t bytes, uint32_t timeout_ms);
int cc_comm_init(cc_comm** comm, int nranks, int rank, const void* id, size_t bytes); /* default timeout */
/* destroy: finalize (flush this rank's work) + free.  abort: free without
 * waiting for the peers (a rank leaving a communicator its peers gave up on). */
int cc_comm_destroy(cc_comm* comm);
int cc_comm_abort(cc_comm* comm);
int cc_comm_size(const cc_comm* comm);
int cc_comm_rank(const cc_comm* comm);

/* d_digest[0..n) <- XOR over all ranks of their d_digest[0..n) (in place;
 * collective, stream-ordered, enqueue only): ncclAllGather of the partials,
 * then cc_digest_fold_dev.  Calls on one communicator must be issued in the
 * same order on every rank, from one stream at a time. */
int cc_digest_allreduce_dev(cc_comm* comm, uint32_t* d_digest, uint64_t n, void* stream);

/* Bounded wait for everything enqueued on `stream` so far -- the digest
 * exchanges of cc_pool_scan_dev / cc_digest_allreduce_dev included -- with the
 * communicator's health polled meanwhile (ncclCommGetAsyncError).  CC_OK once
 * the stream has reached this point; if a peer stopped participating after
 * init the collective never completes: after `timeout_ms` (0 =
 * $CC_COMM_WAIT_TIMEOUT_MS, else 60 s) the communicator is aborted (its
 * kernels released, the stream drains) and CC_ETIMEDOUT is returned; an RCCL
 * async error aborts it at once with CC_ECOMM.  An aborted communicator
 * answers CC_ECOMM to every later exchange; free it with cc_comm_abort.  The
 * reference bounds its exchange the same way (FollowScanMap retry x timeout,
 * chunk_closure.cpp:82-104).  Blocking (sleep-polls, never spins a core). */
int cc_comm_wait(cc_comm* comm, void* stream, uint32_t timeout_ms);

/* One rank's shard of the pool and the outputs of one scan pass over it. */
typedef struct cc_pool_shard {
    const void* d_data;       /* n_chunks x chunk_bytes, chunk c's data at c*chunk_bytes */
    const void* d_meta;       /* n_chunks x meta_bytes metapages (file = metapage || data) */
    uint64_t n_chunks;
    uint32_t chunk_bytes;     /* 16 MiB (conf/chunkserver.conf chunksize) */
    uint32_t meta_bytes;      /* 4 KiB metapage */
    uint32_t page_bytes;      /* 4 KiB */
    uint32_t slice_bytes;     /* 4 MiB scan slice (copyset.scan_size_byte) */
    const uint32_t* d_after_mult; /* [n_chunks] x^(8*bytes after the file in its copyset chain), cc_xpow8_dev */
    const uint32_t* d_group;      /* [n_chunks] copyset index of each file */
    uint64_t n_groups;            /* copysets in the WHOLE pool (same on every rank) */
    /* outputs (device) */
    uint32_t* d_page_crcs;    /* [n_chunks * chunk_bytes/page_bytes] */
    uint32_t* d_meta_crcs;    /* [n_chunks]  ScanMap.crc of the readMetaPage op */
    uint32_t* d_slice_crcs;   /* [n_chunks * chunk_bytes/slice_bytes]  ScanMap.crc of the data ops */
    uint32_t* d_file_crcs;    /* [n_chunks]  CRC32(metapage || data), may be NULL */
    uint32_t* d_digest;       /* [n_groups]  full per-copyset digests after the call */
    /* optional hipEvent_t recorded on `stream` right before / after the page
     * kernel over the data (NULL = none): lets a bench time the hot kernel
     * inside the one call */
    void* ev_pages_begin;
    void* ev_pages_end;
    /* optional hipEvent_t recorded on `stream` right before the digest
     * exchange's all-gather and right after its XOR fold (comm non-NULL only;
     * NULL = none): the exchange's own share of a scan step at N > 1 */
    void* ev_exchange_begin;
    void* ev_exchange_end;
} cc_pool_shard;

/* One integrity scan pass over the shard: page CRCs of every data page and
 * metapage, slice CRCs (ScanMap.crc), file CRCs, digest partials, then (comm
 * non-NULL) the digest all-reduce, after which d_digest[g] on every rank is
 * copyset g's CopysetNode::GetHash value over the WHOLE pool
 * (V(f1||..||fn) = XOR_i shift(V(fi), bytes after fi): exact, no constant).
 * Enqueue only; comm NULL = single-rank pool.  Needs chunk_bytes = 256*q
 * pages with slice_bytes = q*2^j pages (the fused epilogue's geometry). */
int cc_pool_scan_dev(const cc_pool_shard* shard, cc_comm* comm, void* stream);

/* ------------------------------------------------------------------------
 * Per-page CRC persistence -- the table verify-on-read and
 * the integrity jobs of proto/integrity.proto (IntegrityService, :55-61;
 * declared and compiled in the reference, never implemented) check against.
 * The reference keeps no data CRC anywhere: the metapage holds a CRC of its own
 * header only (chunkserver_chunkfile.cpp:64-130), so the table is a NEW sidecar
 * file per chunk, kept OUTSIDE the copyset data directory (CopysetNode::GetHash
 * chains every file listed there, copyset_node.cpp:931-970).  It records the
 * chunk's sn (metapage) and the chunk file's mtime and size when it was
 * written: a table whose chunk changed since is STALE and never condemns data.
 * (mtime comes from the kernel's coarse clock: a write path that changes a
 * chunk must store its table -- cc_pcrc_store after the write, e.g. from the
 * CRCs cc_apply_log_delta_dev keeps current -- staleness is the safety net.)
 * ------------------------------------------------------------------------ */
#define CC_PCRC_HEADER_BYTES 64

typedef struct cc_pcrc_header {
    uint32_t page_bytes;
    uint32_t n_pages;
    uint64_t chunk_sn;      /* metapage sn when the table was written */
    int64_t data_mtime_ns;  /* the chunk file's st_mtim then */
    uint64_t data_size;     /* the chunk file's size then */
    int64_t stamp_ns;       /* CLOCK_REALTIME when the CRCs' bytes were known current: a check's
                               time just before it read the chunk; cc_pcrc_store_expect's
                               expect->stamp_ns (or the mtime); cc_pcrc_store's call time */
} cc_pcrc_header;

/* Racy tables (git's "racily clean" index entries).  File mtimes come from a
 * coarse clock: a write landing in the same clock tick as data_mtime_ns leaves
 * the identity unchanged.  A table is trusted to condemn data only when that
 * cannot have happened after its CRCs were taken, i.e. when
 *     data_mtime_ns + tick < stamp_ns      (tick = clock_getres(CLOCK_REALTIME_COARSE);
 *                                           1 s -- 2 s on an even second -- when the mtime
 *                                           has no sub-second part: a filesystem keeping
 *                                           whole seconds, or FAT's 2 s)
 * Otherwise it is RACY: its pages are still compared, a match re-stamps it
 * (the table is rewritten with a later stamp), and a mismatch is reported as
 * STALE -- refreshed by policy -- never as bad pages. */
int cc_pcrc_is_racy(const cc_pcrc_header* h);

/* In-memory codec.  decode: CC_ECORRUPT for a bad magic / version / header CRC
 * / table CRC / length; page_crcs may be NULL (header only). */
uint64_t cc_pcrc_encoded_bytes(uint32_t n_pages);
int cc_pcrc_encode(const cc_pcrc_header* h, const uint32_t* page_crcs, void* out, uint64_t out_bytes);
int cc_pcrc_decode(const void* buf, uint64_t bytes, cc_pcrc_header* h, uint32_t* page_crcs, uint32_t max_pages);

/* sn of a chunk metapage, after ChunkFileMetaPage::decode's checks
 * (chunkserver_chunkfile.cpp:90-130: header CRC, version 1 or 2), bounds-checked;
 * CC_ECORRUPT otherwise. */
int cc_chunk_meta_sn(const void* metapage, uint32_t bytes, uint64_t* sn);

/* Write the table of chunk file `chunk_path` (metapage of meta_bytes, then
 * n_pages data pages) to `table_path`, atomically (temp file + fsync + rename),
 * recording the chunk's current sn, mtime and size.  Call it after the data
 * write it describes (the write path's CSChunkFile::Write, chunkserver_chunkfile.cpp:287-427),
 * under the chunk's write lock (CSChunkFile::rwLock_) so no other write lands
 * between the two.  CC_EFORMAT when the file's size is not meta_bytes +
 * n_pages x page_bytes (FileFormatError). */
int cc_pcrc_store(const char* chunk_path, uint32_t meta_bytes, const char* table_path, const uint32_t* page_crcs,
                  uint32_t n_pages, uint32_t page_bytes);
/* The same, but only if the chunk's identity is still `expect` (its sn,
 * data_mtime_ns and data_size; the caller stats the file right after its
 * pwrite): CC_ESTALE and nothing written otherwise, so a store that runs after
 * a LATER write cannot pair the newer identity with the older CRCs.  The table
 * is stamped with expect->stamp_ns -- the caller's CLOCK_REALTIME taken BEFORE
 * its pwrite -- or, when that is 0, with data_mtime_ns (racy until a check
 * re-stamps it); never with the store's own clock, which could clear a table
 * whose chunk took a second same-size write within the mtime's tick. */
int cc_pcrc_store_expect(const char* chunk_path, uint32_t meta_bytes, const char* table_path,
                         const uint32_t* page_crcs, uint32_t n_pages, uint32_t page_bytes,
                         const cc_pcrc_header* expect);
/* Read + decode a table file (-errno if it cannot be read, -ENOENT if absent).
 * With page_crcs, a file larger than a table of max_pages pages is CC_ECORRUPT
 * before anything is allocated; without, only the 64-byte header is read. */
int cc_pcrc_load(const char* table_path, cc_pcrc_header* h, uint32_t* page_crcs, uint32_t max_pages);

/* Table state of one chunk after a check. */
#define CC_TABLE_OK 0        /* table describes the chunk; bad_pages counted against it */
#define CC_TABLE_CREATED 1   /* no table: one was written from the current bytes */
#define CC_TABLE_CORRUPT 2   /* table unreadable (CRC / geometry): reported, not used */
#define CC_TABLE_STALE 3     /* chunk changed since the table was written: not used */
#define CC_TABLE_REFRESHED 4 /* stale, and rewritten from the current bytes */
#define CC_TABLE_MISSING 5   /* no table, none written */
#define CC_TABLE_REBUILT 6   /* corrupt, and rewritten from the current bytes */

typedef struct cc_integrity_opts {
    uint32_t chunk_bytes;    /* 16 MiB */
    uint32_t meta_bytes;     /* 4 KiB */
    uint32_t page_bytes;     /* 4 KiB */
    uint32_t io_threads;     /* readers of cc_scan_files (0 = cc_default_io_threads()) */
    uint32_t create_missing; /* write a table for a chunk that has none */
    uint32_t refresh_stale;  /* rewrite stale / corrupt tables from the current bytes */
} cc_integrity_opts;

typedef struct cc_integrity_result {
    int32_t status;       /* 0; -errno; CC_EFORMAT (file size != metapage + chunk, checked first as
                             CSChunkFile::Open does); CC_ECORRUPT (metapage header) */
    uint32_t table_state; /* CC_TABLE_* */
    uint32_t n_pages;
    uint32_t bad_pages;   /* pages whose bytes no longer match the (valid, current) table */
    int64_t first_bad;    /* -1: none */
} cc_integrity_result;

/* The integrity check of a batch of chunk files (the work of one
 * IntegrityService job step): every data page rehashed on the device (native
 * pread into pinned staging, cc_scan_files) and compared with the chunk's
 * table; a file that changes while it is read counts as stale.  Bad pages are
 * listed as (file index << 32 | page) in bad_list (the first bad_cap of them;
 * *n_bad = all).  Blocking, thread-safe. */
int cc_integrity_check(const char* const* chunk_paths, const char* const* table_paths, uint64_t n,
                       const cc_integrity_opts* opts, cc_integrity_result* res, uint64_t* bad_list, uint64_t bad_cap,
                       uint64_t* n_bad);

/* ------------------------------------------------------------------------
 * Diagnostics (new; no reference counterpart)
 * ------------------------------------------------------------------------ */
/* Copy the 163840-byte LDS image the page kernel loads into every CU (G tables
 * + per-lane final maps, DESIGN.md "LDS image") so host tests can replay the
 * kernel's arithmetic on the CPU.  Needs no GPU. */
int cc_lds_image(void* out, size_t bytes);

/* Read-only HBM probe: streams `bytes` (multiple of 4096, 16-byte aligned) from
 * d_buf with the page kernel's access style (nontemporal, grid-stride,
 * persistent blocks) and XOR-reduces into d_sink[0 .. 2*CUs*16).  What a pure
 * read achieves on THIS device: bench.py reports the page kernel against it
 * beside the 8 TB/s spec.  Enqueue only. */
int cc_hbm_read_probe_dev(const void* d_buf, uint64_t bytes, uint32_t* d_sink, void* stream);

/* Diagnostic (no reference counterpart): the page kernel over n_pages 4 KiB
 * pages with its CRC arithmetic replaced by a rotate-XOR -- the same schedule
 * (tiles, prefetch ring, dynamic tail), loads and 4-byte-per-page stores into
 * d_out, so its time is the ceiling cc_page_crc_dev is held to on this device.
 * d_out receives meaningless words.  Enqueue only. */
int cc_page_load_probe_dev(const void* d_pages, uint64_t n_pages, uint32_t* d_out, void* stream);

/* Diagnostic (no reference counterpart): the write log's page traffic alone,
 * the ceiling cc_apply_log_dev is held to on its access pattern.  One
 * descriptor per touched 4 KiB page of a log (host-built, e.g.
 * curve_amd.crc.log_probe_descs): the rows read from the source (covered by the
 * page's only piece; src_off = the source byte of page byte 0, mod 2^64) -- the
 * others from the page -- and the rows stored back.  Same grid and occupancy
 * as the write log's page pass, no table, no CRC.  It stores back the bytes it
 * loaded: run right after the log it describes was applied, it changes no
 * byte.  d_out[i] = an XOR of page i's words.  A descriptor naming a page past
 * the pool touches nothing (page 0 read, no store); source offsets are the
 * caller's to keep inside d_src.  Enqueue only. */
typedef struct cc_log_probe_desc {
    uint64_t page;
    uint64_t src_off;
    uint32_t covered_rows;
    uint32_t dirty_rows;
} cc_log_probe_desc;
int cc_apply_log_probe_dev(void* d_pool, uint64_t pool_bytes, const void* d_src, const cc_log_probe_desc* d_desc,
                           uint64_t n, uint32_t* d_out, void* stream);

/* Diagnostic (no reference counterpart): the read traffic of a list of 4 KiB
 * pages alone -- d_pages[i] = a page index of the pool, in list order (for a
 * batch of reads: each read's pages in turn) -- the ceiling cc_verify_reads_dev
 * is held to on its access pattern.  Verify-on-read's grid, occupancy and
 * schedule (a workgroup of 8 waves per CU, LDS unused; each wave an equal
 * contiguous share of the first 15/16 of the list, the rest in 32-page chunks
 * to whichever waves finish first), two pages in flight, no CRC, no stored-CRC
 * loads.  d_out[i] = an
 * XOR of page i's words.  An index past the pool reads page 0 instead (never
 * outside the pool).  Enqueue only. */
int cc_page_list_probe_dev(const void* d_pool, uint64_t pool_bytes, const uint64_t* d_pages, uint64_t n,
                           uint32_t* d_out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CURVE_CRC_H_ */
