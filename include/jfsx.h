/*
 * jfsx.h -- C-ABI of libjfsx.so, the MI355X block-transform engine for the
 * JuiceFS per-block data path (AEAD Seal/Open fused with CRC32C segment
 * checksums).  Plain C types only: this is the surface a cgo shim binds
 * (see INTEGRATION.md for the Go side).
 *
 * Reference interfaces each entry point replaces (JuiceFS 1.2.0,
 * /root/reference):
 *
 *   jfsx_seal_batch      dataEncryptor.Encrypt's aead.Seal          pkg/object/encrypt.go:164-194 (Seal at :192)
 *                        + checksum() on the same plaintext         pkg/chunk/disk_cache.go:1218-1231 (called :469)
 *   jfsx_open_batch      dataEncryptor.Decrypt's aead.Open          pkg/object/encrypt.go:196-216 (Open at :215)
 *                        + checksum()/verify of the plaintext       pkg/chunk/disk_cache.go:1219, :1315-1327
 *   jfsx_data_encrypt    dataEncryptor.Encrypt (object format)      pkg/object/encrypt.go:164-194
 *   jfsx_data_decrypt    dataEncryptor.Decrypt (object format)      pkg/object/encrypt.go:196-216
 *   jfsx_checksum        checksum(data) []byte                      pkg/chunk/disk_cache.go:1218-1231
 *   jfsx_crc32c_segments the CRC loop of cacheFile.ReadAt           pkg/chunk/disk_cache.go:1315-1327
 *   jfsx_cache_verify    cacheFile.ReadAt level logic + verify      pkg/chunk/disk_cache.go:1255-1329
 *   jfsx_object_crc32c   generateChecksum / checksumReader of the   pkg/object/checksum.go:31-82
 *   (+ JFSX_CRC_CT)      stored object, fused with Seal/Open        (s3.go:140-146,173-176)
 *   JFSX_AES256GCM /     NewDataEncryptor algo "aes256gcm-rsa" /    pkg/object/encrypt.go:142-162
 *   JFSX_CHACHA20P1305   "chacha20-rsa"
 *
 * RSA-OAEP key wrapping (encrypt.go:124-134) stays with the caller: the
 * engine takes the 32-byte data key and 12-byte nonce per block as inputs
 * (the reference draws both from crypto/rand, encrypt.go:165-180).
 *
 * Threading: a context may be used from several host threads; calls on one
 * context are serialised internally (one HIP stream per context).  Use one
 * context per GPU (per device ordinal) and per submitting thread for
 * concurrency.
 *
 * Return codes: 0 on success, negative errno-style values on batch-level
 * failure (JFSX_EINVAL, JFSX_ENODEV, JFSX_EIO, JFSX_ENOMEM).  Per-block
 * results are in jfsx_blk.status.
 */
#ifndef JFSX_H
#define JFSX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JFSX_ABI_VERSION 9

/* algorithms (encrypt.go:142-145) */
#define JFSX_AES256GCM 0     /* "aes256gcm-rsa" (also the "" default)   */
#define JFSX_CHACHA20P1305 1 /* "chacha20-rsa"                          */

/* CRC32C segment checksum mode, per 32 KiB segment of the PLAINTEXT
 * (csBlock = 32 KiB, disk_cache.go:1207).  CRC arrays are big-endian uint32
 * per segment, exactly the bytes checksum() returns (buffer.go:42-44,98-101);
 * a zero-length block has one zero CRC (4 bytes), as checksum() does. */
#define JFSX_CRC_NONE 0   /* no checksum                                  */
#define JFSX_CRC_GEN 1    /* write crc[] (level != none on cache write)   */
#define JFSX_CRC_VERIFY 2 /* compare against crc[] (cache read verify)    */
/* flag OR'ed into GEN/VERIFY: the segment CRCs cover the ciphertext C (seal:
 * output, open: input) instead of the plaintext -- the bytes the object store
 * checksums (pkg/object/checksum.go:31-53, s3.go:173-176); fold them into the
 * whole-object value with jfsx_object_crc32c. */
#define JFSX_CRC_CT 4
/* flag OR'ed into JFSX_CRC_GEN only: BOTH checksums in one call -- crc points
 * at 8*max(1,ceil(len/32K)) bytes, the plaintext segment CRCs (checksum() of
 * the block, as CRC_GEN) followed by the ciphertext segment CRCs (as
 * CRC_GEN|CRC_CT).  This is what an upload of one block to an S3-class store
 * with a disk cache needs: bcache.stage checksums the plaintext and the store's
 * Put checksums the sealed object (pkg/chunk/cached_store.go:439-451,
 * pkg/object/s3.go:173-176).  The ciphertext pass runs on the copy of the
 * block already in device memory, so it adds no host or PCIe traffic. */
#define JFSX_CRC_BOTH 8

/* where src/dst/crc pointers of a batch live */
#define JFSX_MEM_DEVICE 0 /* device memory (jfsx_alloc_device / hipMalloc) */
#define JFSX_MEM_HOST 1   /* host memory; staged through the engine          */
/* JFSX_MEM_HOST buffers may be page-locked (jfsx_alloc_pinned*, or memory the
 * HIP runtime knows as registered) or ordinary pageable memory (a Go-heap
 * slice, malloc).  Page-locked blocks are copied by DMA directly; the engine
 * copies a pageable block into pinned staging it owns on the calling thread
 * before the upload, and a pageable output out of it after the download, and
 * never keeps a pointer to caller memory past the call (cgo's rules). */

/* per-block status */
#define JFSX_OK 0
#define JFSX_ETAG 1 /* AEAD authentication failed (Go: cipher's errOpen)      */
#define JFSX_ECRC 2 /* "data checksum %d != expect %d" (disk_cache.go:1324)   */
#define JFSX_EOF 3  /* jfsx_cache_verify: short read (File.ReadAt's io.EOF)    */
#define JFSX_EFORMAT 4 /* malformed LZ4 block / zstd frame (the library's error) */
#define JFSX_EDSTSIZE 5 /* zstd: the frames decode to more than dst_cap bytes */

/* batch-level errors */
#define JFSX_EINVAL (-22)
#define JFSX_ENODEV (-19)
#define JFSX_EIO (-5)
#define JFSX_ENOMEM (-12)
#define JFSX_EAGAIN (-11) /* jfsx_wait: not finished within the timeout     */
#define JFSX_EMISFORMED (-74) /* "misformed ciphertext: %d %d" (encrypt.go:199-201) */

typedef struct jfsx_ctx jfsx_ctx;

/* One 4 MiB-class block.  For JFSX_MEM_DEVICE batches src/dst must be
 * 16-byte aligned; dst may equal src (in place, as aead.Seal(p[:0]...) and
 * aead.Open(ciphertext[:0]...) are).  Length limits are the ciphers' own
 * (JFSX_EINVAL beyond them, where Go's Seal panics and Open fails):
 *   AES-256-GCM        len <= (2^32 - 2) * 16 B  (32-bit block counter from 2;
 *                      crypto/cipher gcm.go gcmMaxPlaintext)
 *   ChaCha20-Poly1305  len <= 2^38 - 64 B        (x/crypto v0.19.0
 *                      chacha20poly1305.go: block counter from 1)
 * Open with a failed tag (status JFSX_ETAG) releases nothing: dst is zeroed,
 * as Go's in-place aead.Open (encrypt.go:215) clears out on a mismatch, and a
 * plaintext CRC_GEN array is zeroed too. */
typedef struct jfsx_blk {
    uint8_t key[32];      /* data key (encrypt.go:165)                        */
    uint8_t nonce[12];    /* nonce (encrypt.go:177)                           */
    uint32_t reserved;    /* must be 0                                        */
    const void *src;      /* seal: plaintext  / open: ciphertext (no tag)     */
    void *dst;            /* seal: ciphertext / open: plaintext               */
    uint64_t len;         /* bytes of src/dst                                 */
    uint8_t tag[16];      /* seal: out / open: in                             */
    uint8_t *crc;         /* GEN: out, VERIFY: in; 4*max(1,ceil(len/32K)) B   */
    int32_t status;       /* out: JFSX_OK / JFSX_ETAG / JFSX_ECRC             */
    int32_t crc_bad_seg;  /* out: first failing segment (VERIFY), else -1     */
    uint32_t crc_got;     /* out: CRC computed for crc_bad_seg                */
    uint32_t crc_expect;  /* out: CRC expected for crc_bad_seg                */
} jfsx_blk;

/* One checksum range: [data, data+len) is a segment-aligned window of a
 * cache block; crc[k] is the BE32 CRC of its k-th 32 KiB segment. */
typedef struct jfsx_range {
    const void *data;
    uint64_t len;
    uint8_t *crc;         /* GEN: out, VERIFY: in                             */
    int32_t status;       /* out: JFSX_OK / JFSX_ECRC                         */
    int32_t bad_seg;      /* out: first failing segment, -1 none              */
    uint32_t got, expect; /* out                                              */
} jfsx_range;

int jfsx_abi_version(void);
int jfsx_device_count(int *n);

/* Diagnostics for a batch-level JFSX_EIO / JFSX_ENOMEM: the HIP failure behind
 * it, as its hipError_t value and "name (text) at file:line in call", for the
 * calls made on ctx (from any thread, the aggregator's dispatchers and the
 * async queue's worker included) or, with ctx NULL, for the calling thread.
 * hip_error 0 and an empty msg when none was recorded; a newer failure
 * replaces an older one.  A sticky device fault (hipErrorIllegalAddress and
 * the like) leaves the context unusable: close it and fall back.  The Go shim
 * logs this text before it falls back to the CPU path. */
int jfsx_last_error(jfsx_ctx *ctx, int *hip_error, char *msg, size_t cap);

/* context = one GPU + one HIP stream + device workspace + pinned staging.
 * flags: 0, or JFSX_CTX_BITSLICE: AES-256-GCM computes the keystream of whole
 * 32 KiB segments with the bitsliced AES on the VALU instead of the T-table
 * AES in LDS (same bytes; a throughput trade-off). */
#define JFSX_CTX_BITSLICE 1u
int jfsx_ctx_open(int device, uint32_t flags, jfsx_ctx **out);
int jfsx_ctx_close(jfsx_ctx *ctx);
int jfsx_ctx_sync(jfsx_ctx *ctx);
/* returns the context's hipStream_t (as void*) for callers that order their
 * own copies against the engine's work */
void *jfsx_ctx_stream(jfsx_ctx *ctx);
/* kernel timing: when enabled, HIP events bracket the main transform kernel of
 * every batch on the context's stream; query returns the summed milliseconds
 * and the number of launches since the last reset */
int jfsx_ctx_set_timing(jfsx_ctx *ctx, int enable);
/* host-ingest pipeline slot size (default 256 MiB): JFSX_MEM_HOST batches are
 * streamed through 3 device staging slots of this size, H2D | transform | D2H
 * overlapped on three streams */
int jfsx_ctx_set_slot_bytes(jfsx_ctx *ctx, uint64_t bytes);
int jfsx_ctx_kernel_time(jfsx_ctx *ctx, double *ms_total, uint64_t *launches, int reset);

/* Engine counters for the shim's metrics hooks -- the byte / op counters the
 * reference keeps around the block path (cachedStore's Prometheus collectors,
 * pkg/chunk/cached_store.go:847-932: object request bytes and durations,
 * cache hits / misses / read bytes).  Per context, cumulative since open or the
 * last reset; a batch is counted when it returns 0.  bytes = plaintext
 * (AEAD), range (CRC) and input / output (codecs); *_fail = blocks whose
 * status was not JFSX_OK (tag, checksum, malformed, too small).  zstd_serial =
 * zstd objects the block-parallel decoder handed to the serial decoder (frame
 * shapes outside its fast path, or frames it rejects).  kernel_ms /
 * kernel_launches: the main-kernel time, counted only while
 * jfsx_ctx_set_timing is enabled. */
typedef struct jfsx_metrics {
    uint64_t seal_batches, seal_blocks, seal_bytes;
    uint64_t open_batches, open_blocks, open_bytes, open_fail;
    uint64_t crc_batches, crc_ranges, crc_bytes, crc_fail;
    uint64_t lz4c_blocks, lz4c_in, lz4c_out;
    uint64_t lz4d_blocks, lz4d_in, lz4d_out, lz4d_fail;
    uint64_t zstdc_blocks, zstdc_in, zstdc_out;
    uint64_t zstdd_blocks, zstdd_in, zstdd_out, zstdd_fail, zstd_serial;
    double kernel_ms;
    uint64_t kernel_launches;
} jfsx_metrics;
int jfsx_ctx_metrics(jfsx_ctx *ctx, jfsx_metrics *out, int reset);

/* memory helpers (engine-owned pinned staging, device buffers); pinned memory
 * is portable: any context of the process (any GPU) may stream from it.
 * Device buffers from jfsx_alloc_device are registered by address, so a
 * multi-device context can route a device-memory block to the GPU that owns
 * it (jfsx_mctx_seal_batch with JFSX_MEM_DEVICE). */
int jfsx_alloc_pinned(jfsx_ctx *ctx, size_t bytes, void **p);
int jfsx_free_pinned(jfsx_ctx *ctx, void *p);
int jfsx_alloc_device(jfsx_ctx *ctx, size_t bytes, void **p);
int jfsx_free_device(jfsx_ctx *ctx, void *p);

/* NUMA placement of pinned staging, so that at N GPUs on a multi-socket node
 * every GPU streams from memory on its own socket (the reference's uploaders
 * fill Go-heap pages wherever the scheduler ran them, pkg/chunk/page.go:33-60;
 * the shim copies them into this staging).
 *   jfsx_device_numa_node  host NUMA node closest to `device` (-1 unknown)
 *   jfsx_alloc_pinned_node pinned portable memory whose pages are bound to
 *                          `node` while they are allocated (-1: the node of the
 *                          context's device); where the node cannot be bound
 *                          (a cpuset without it) the default placement is used
 *   jfsx_host_numa_node    node of the pages of [p, p+bytes), sampled every
 *                          64 MiB: -1 unknown, -2 pages on more than one node
 * Free with jfsx_free_pinned. */
int jfsx_device_numa_node(int device, int *node);
int jfsx_alloc_pinned_node(jfsx_ctx *ctx, size_t bytes, int node, void **p);
int jfsx_host_numa_node(const void *p, size_t bytes, int *node);
int jfsx_memcpy_h2d(jfsx_ctx *ctx, void *dst, const void *src, size_t bytes);
int jfsx_memcpy_d2h(jfsx_ctx *ctx, void *dst, const void *src, size_t bytes);

/* Batched AEAD over blocks, fused with CRC32C segment checksums of the
 * plaintext.  mem = JFSX_MEM_DEVICE or JFSX_MEM_HOST.  Synchronous: returns
 * when tags, CRCs and statuses are written back into blks.
 * JFSX_MEM_HOST batches stream through the context's pipeline of 8 staging
 * slots (H2D | transform | D2H on three streams).  The pipeline is shared by
 * every thread calling on the context and never drains between calls: a call
 * enqueues its groups and then waits for its own groups only, so concurrent
 * callers (the aggregator's dispatchers, per-object shims) keep both copy
 * directions busy back to back.  Device batches hold the context for the
 * whole call. */
int jfsx_seal_batch(jfsx_ctx *ctx, int algo, int n, jfsx_blk *blks, int crc_mode, int mem);
int jfsx_open_batch(jfsx_ctx *ctx, int algo, int n, jfsx_blk *blks, int crc_mode, int mem);

/* CRC32C per 32 KiB segment over n ranges (cache-hit verify, none-cipher
 * volumes, staging re-read).  mode = JFSX_CRC_GEN or JFSX_CRC_VERIFY. */
int jfsx_crc32c_segments(jfsx_ctx *ctx, int n, jfsx_range *ranges, int mode, int mem);

/* Asynchronous variants: the batch is queued on the context's worker thread
 * (batches of one context run in submission order) and the call returns a
 * ticket at once.  blks/ranges and every buffer they name must stay valid
 * until jfsx_wait has returned for the ticket.  jfsx_wait returns the batch's
 * return code (as the synchronous call would) and retires the ticket;
 * timeout_ms < 0 waits without limit, 0 polls; JFSX_EAGAIN if the batch has
 * not finished in time (the ticket stays live).  jfsx_ctx_close runs the
 * queued batches before it releases the context. */
typedef uint64_t jfsx_ticket;
int jfsx_seal_batch_async(jfsx_ctx *ctx, int algo, int n, jfsx_blk *blks, int crc_mode, int mem, jfsx_ticket *t);
int jfsx_open_batch_async(jfsx_ctx *ctx, int algo, int n, jfsx_blk *blks, int crc_mode, int mem, jfsx_ticket *t);
int jfsx_crc32c_segments_async(jfsx_ctx *ctx, int n, jfsx_range *ranges, int mode, int mem, jfsx_ticket *t);
int jfsx_wait(jfsx_ctx *ctx, jfsx_ticket t, int timeout_ms);

/* Aggregator: per-block calls in the reference's shape --
 * one synchronous Encrypt / Decrypt / cache-read verify per goroutine
 * (encrypt.go:164-216, disk_cache.go:1315-1327) -- coalesced into batches.
 * jfsx_agg_seal / _open / _crc32c block the calling thread until its block
 * is done and return what a one-block batch would (per-block results in
 * blk->status or range->status).  Any number of threads may call at once.  A
 * dispatcher thread groups waiting requests with the same (op, algo, mode,
 * mem) and issues one batch when the group reaches max_blocks (0: 256) or
 * max_bytes (0: 1 GiB), or when the oldest request has waited window_us.  A
 * request the engine rejects (JFSX_EINVAL) fails alone: the batch is retried
 * one request at a time.  Free the aggregator before closing its context. */
typedef struct jfsx_agg jfsx_agg;
int jfsx_agg_new(jfsx_ctx *ctx, int max_blocks, uint64_t max_bytes, uint32_t window_us, jfsx_agg **out);
int jfsx_agg_free(jfsx_agg *agg);
int jfsx_agg_seal(jfsx_agg *agg, int algo, jfsx_blk *blk, int crc_mode, int mem);
int jfsx_agg_open(jfsx_agg *agg, int algo, jfsx_blk *blk, int crc_mode, int mem);
int jfsx_agg_crc32c(jfsx_agg *agg, jfsx_range *range, int mode, int mem);
/* requests taken, batches issued, requests those batches carried */
int jfsx_agg_stats(jfsx_agg *agg, uint64_t *calls, uint64_t *batches, uint64_t *blocks);
/* Dispatch: each context gets several dispatcher threads (4; the environment
 * variable JFSX_AGG_DISPATCHERS overrides, 1..32), so several batches of one
 * device are in flight at once (host batches pipeline, see jfsx_seal_batch).
 * A group waits for its window only while the engine is idle; while another
 * of the aggregator's batches is running, a free dispatcher takes what is
 * queued at once (the time spent queued behind the running batch is the
 * batching).  For per-object callers in host memory keep max_bytes near
 * 16 MiB, so that a 20-caller closed loop (max-uploads) is cut into several
 * batches in flight instead of one batch that all callers wait for. */

/* dataEncryptor.Encrypt / Decrypt (encrypt.go:164-216) through the
 * aggregator: the same object format and results as jfsx_data_encrypt /
 * jfsx_data_decrypt, with the Seal / Open issued as one aggregated request, so
 * the shim's per-object Encrypt from max-uploads goroutines batches. */
int jfsx_agg_data_encrypt(jfsx_agg *agg, int algo, const uint8_t key[32], const uint8_t nonce[12],
                          const uint8_t *wrapped, int wlen, const void *plaintext, uint64_t len, void *out,
                          uint64_t out_cap, uint64_t *out_len, uint32_t *obj_crc);
int jfsx_agg_data_decrypt(jfsx_agg *agg, int algo, const uint8_t key[32], const void *obj, uint64_t olen, void *out,
                          uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc, uint32_t *got_crc);
/* The same, and checksum() of the plaintext in the same pass (seg_crc,
 * nullable: 4*max(1,ceil(len/32K)) bytes, the cache file's trailer): the
 * block the reference touches twice -- wSlice.upload stages it in the disk
 * cache (bcache.stage -> checksum, disk_cache.go:433-483) and then uploads it
 * (store.upload -> Encrypt, cached_store.go:415-472); store.load decrypts it
 * and then caches it (bcache.cache -> checksum, cached_store.go:673-748) --
 * crosses PCIe once.  With obj_crc / expect_crc as well, both checksums come
 * out of the one call (JFSX_CRC_BOTH).  Decrypt: seg_crc is zeroed when the
 * call fails (tag or object checksum), as the plaintext is. */
int jfsx_agg_data_encrypt_ex(jfsx_agg *agg, int algo, const uint8_t key[32], const uint8_t nonce[12],
                             const uint8_t *wrapped, int wlen, const void *plaintext, uint64_t len, void *out,
                             uint64_t out_cap, uint64_t *out_len, uint32_t *obj_crc, uint8_t *seg_crc);
int jfsx_agg_data_decrypt_ex(jfsx_agg *agg, int algo, const uint8_t key[32], const void *obj, uint64_t olen,
                             void *out, uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc,
                             uint32_t *got_crc, uint8_t *seg_crc);

/* Multi-device context (SURVEY §8b jfsx_open_ctx(dev_mask), §8e): one
 * jfsx_ctx per selected GPU (bit d of dev_mask = device d; 0 = every visible
 * device).  Blocks are independent (own key, nonce, tag, CRCs), so the parts
 * of a batch run concurrently, one persistent worker thread per device; no
 * device-to-device traffic.  A JFSX_MEM_HOST batch is cut into one contiguous
 * run of blocks per device, balanced by bytes.  A JFSX_MEM_DEVICE batch is
 * routed by ownership: every block goes to the GPU whose memory holds its
 * src, dst and crc (buffers from jfsx_alloc_device on a member context, or any
 * device allocation); a block whose buffers span GPUs, or live on a GPU
 * outside the context, fails the batch with JFSX_EINVAL before anything runs.
 * Results land in blks exactly as with a single context.  A batch-level error
 * of any device is returned (the first one, in device order). */
typedef struct jfsx_mctx jfsx_mctx;
int jfsx_mctx_open(uint64_t dev_mask, uint32_t flags, jfsx_mctx **out);
int jfsx_mctx_close(jfsx_mctx *m);
int jfsx_mctx_ndev(jfsx_mctx *m);                 /* devices in the context   */
jfsx_ctx *jfsx_mctx_ctx(jfsx_mctx *m, int i);     /* i-th device's context    */
int jfsx_mctx_seal_batch(jfsx_mctx *m, int algo, int n, jfsx_blk *blks, int crc_mode, int mem);
int jfsx_mctx_open_batch(jfsx_mctx *m, int algo, int n, jfsx_blk *blks, int crc_mode, int mem);
int jfsx_mctx_crc32c_segments(jfsx_mctx *m, int n, jfsx_range *ranges, int mode, int mem);
/* Aggregator over every device of a multi-device context: one dispatcher
 * thread per device takes the next ready group from one shared queue, so the
 * per-block callers (≤ max-uploads upload goroutines, cached_store.go:371-472;
 * readers, :673-748) spread over all GPUs.  Same call semantics as jfsx_agg_new. */
int jfsx_agg_new_mctx(jfsx_mctx *m, int max_blocks, uint64_t max_bytes, uint32_t window_us, jfsx_agg **out);
/* batches issued by the aggregator's dispatcher for device slot i */
int jfsx_agg_dev_batches(jfsx_agg *agg, int i, uint64_t *batches);

/* checksum(data) on the GPU: out receives 4*max(1,ceil(len/32K)) bytes.
 * data and out are host memory. */
int jfsx_checksum(jfsx_ctx *ctx, const void *data, uint64_t len, uint8_t *out);

/* cacheFile.ReadAt verify (disk_cache.go:1255-1329) over an in-memory cache
 * file image: file = data(length) ‖ BE32 CRCs, level 0 none / 1 full /
 * 2 shrink / 3 extend (the level openCacheFile resolved).  Copies
 * [off, off+size) into out.  Returns 0 ok, JFSX_ECRC on mismatch (got,
 * expect, bad_seg filled), JFSX_EOF on a short read, <0 on argument errors.
 * *n_out is what Go's ReadAt returns as n.  file and out are host memory of
 * any alignment; the verified window is staged through a per-context pinned
 * arena (no per-call allocation). */
int jfsx_cache_verify(jfsx_ctx *ctx, const void *file, uint64_t file_size, uint64_t length, int level,
                      uint64_t off, uint64_t size, void *out, uint64_t *n_out, uint32_t *got,
                      uint32_t *expect, int64_t *bad_seg);

/* dataEncryptor.Encrypt with an already-wrapped key: writes
 * BE16(wlen) | 12 | wrapped | nonce | C | tag into out (host memory).
 * out_cap must be >= 3+wlen+12+len+16.  obj_crc (nullable) receives the
 * object-store checksum of the whole output, generateChecksum's value
 * (checksum.go:31-53), computed in the same pass as the Seal. */
int jfsx_data_encrypt(jfsx_ctx *ctx, int algo, const uint8_t key[32], const uint8_t nonce[12],
                      const uint8_t *wrapped, int wlen, const void *plaintext, uint64_t len, void *out,
                      uint64_t out_cap, uint64_t *out_len, uint32_t *obj_crc);
/* dataEncryptor.Decrypt after the key is unwrapped: parses the header
 * (JFSX_EMISFORMED if 3+klen+nlen >= olen), opens, and writes the plaintext
 * to out only when the tag verifies (returns JFSX_ETAG otherwise).  With
 * expect_crc non-null the object checksum is verified in the same pass
 * (checksumReader, checksum.go:55-82): on mismatch returns JFSX_ECRC with the
 * computed value in *got_crc ("verify checksum failed: %d != %d") and releases
 * no plaintext; the checksum failure takes precedence over JFSX_ETAG. */
int jfsx_data_decrypt(jfsx_ctx *ctx, int algo, const uint8_t key[32], const void *obj, uint64_t olen,
                      void *out, uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc,
                      uint32_t *got_crc);
/* the two above with checksum() of the plaintext in the same pass (seg_crc,
 * nullable; see jfsx_agg_data_encrypt_ex) */
int jfsx_data_encrypt_ex(jfsx_ctx *ctx, int algo, const uint8_t key[32], const uint8_t nonce[12],
                         const uint8_t *wrapped, int wlen, const void *plaintext, uint64_t len, void *out,
                         uint64_t out_cap, uint64_t *out_len, uint32_t *obj_crc, uint8_t *seg_crc);
int jfsx_data_decrypt_ex(jfsx_ctx *ctx, int algo, const uint8_t key[32], const void *obj, uint64_t olen,
                         void *out, uint64_t out_cap, uint64_t *out_len, const uint32_t *expect_crc,
                         uint32_t *got_crc, uint8_t *seg_crc);

/* crc32.Update(crc, MakeTable(Castagnoli), data) on the host (small spans:
 * object header and tag) */
uint32_t jfsx_crc32c_update(uint32_t crc, const void *data, uint64_t n);
/* CRC32C of A||B from crc(A), crc(B), len(B) (GF(2) shift by x^(8 len B)) */
uint32_t jfsx_crc32c_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
/* Batched RSA-OAEP key unwrap: replaces, per object,
 * rsaEncryptor.Decrypt = rsa.DecryptOAEP(sha256, rand, priv, wrapped,
 * label) (pkg/object/encrypt.go:124-134, called at :207-210) for every object
 * of a batch at once, on the GPU.  The key is given by its CRT components
 * (Go's Primes[0], Primes[1], Precomputed.Dp, Dq, Qinv), big-endian,
 * prime_bytes each; RSA-2048 (prime_bytes = 128) only.  ct: host memory, item
 * i at ct + i*ct_stride, ct_len[i] bytes.  msg_len[i] = message length, or -1
 * for the decryption error (Go's "crypto/rsa: decryption error"); up to
 * msg_stride bytes of each message are copied to msg + i*msg_stride. */
typedef struct jfsx_rsa_key jfsx_rsa_key;
int jfsx_rsa_key_new(jfsx_ctx *ctx, const uint8_t *p, const uint8_t *q, const uint8_t *dp, const uint8_t *dq,
                     const uint8_t *qinv, int prime_bytes, const uint8_t *label, int label_len, jfsx_rsa_key **out);
int jfsx_rsa_key_free(jfsx_rsa_key *key);
int jfsx_rsa_oaep_decrypt_batch(jfsx_ctx *ctx, const jfsx_rsa_key *key, int n, const uint8_t *ct, uint64_t ct_stride,
                                const uint32_t *ct_len, uint8_t *msg, uint64_t msg_stride, int32_t *msg_len);

/* object-store checksum of header || C || tag (checksum.go:31-53) from the
 * big-endian 32 KiB segment CRCs of C that a GEN|CT batch returned */
int jfsx_object_crc32c(const void *hdr, uint64_t hlen, const uint8_t *seg_crcs, uint64_t clen,
                       const uint8_t *tag, uint32_t *out);

/* LZ4 block stage: the "lz4" Compressor of pkg/compress
 * (compress.go:107-125) that cachedStore.upload runs before the object is
 * put (cached_store.go:371-392) and cachedStore.load after it is read
 * (:680-745).  Bytes are those of the LZ4 C library the reference binds
 * through github.com/hungys/go-lz4: jfsx_lz4_compress_batch writes what
 * LZ4_compress_default(src, dst, len, bound) writes; jfsx_lz4_decompress_batch
 * decodes as LZ4_decompress_safe(src, dst, len, cap) does (status
 * JFSX_EFORMAT where it returns < 0).  One zblk per block: compress needs
 * dst_cap >= jfsx_lz4_bound(src_len) (JFSX_EINVAL otherwise), as
 * cachedStore.upload's CompressBound-sized buffer; src_len <= 0x7E000000.
 * mem = JFSX_MEM_DEVICE or JFSX_MEM_HOST.  The empty-input error of
 * LZ4.Decompress ("decompress an empty input") is the caller's: a zero-length
 * src decodes as LZ4_decompress_safe does (JFSX_EFORMAT). */
typedef struct jfsx_zblk {
    const void *src;
    uint64_t src_len;
    void *dst;
    uint64_t dst_cap;
    uint64_t out_len;  /* out: bytes written to dst                      */
    int32_t status;    /* out: JFSX_OK / JFSX_EFORMAT (decompress)       */
    int32_t reserved;  /* zstd decompress, out: 0, or why the block-parallel
                          decoder handed the object to the serial one: 1 frame
                          shape / headers, 2 Huffman stream, 3 sequence stream,
                          4 sequence execution, 5 raw / RLE block, 6 last
                          literals, 7 content size, 8 content checksum */
} jfsx_zblk;
/* LZ4_compressBound: n + n/255 + 16 (0 for n > 0x7E000000) */
uint64_t jfsx_lz4_bound(uint64_t n);
int jfsx_lz4_compress_batch(jfsx_ctx *ctx, int n, jfsx_zblk *blks, int mem);
int jfsx_lz4_decompress_batch(jfsx_ctx *ctx, int n, jfsx_zblk *blks, int mem);
/* the same per block, through the aggregator (one synchronous call per
 * goroutine, as cachedStore.upload / load call Compress / Decompress), and
 * over a multi-device context (JFSX_MEM_HOST) */
int jfsx_agg_lz4_compress(jfsx_agg *agg, jfsx_zblk *blk, int mem);
int jfsx_agg_lz4_decompress(jfsx_agg *agg, jfsx_zblk *blk, int mem);
int jfsx_mctx_lz4_compress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem);
int jfsx_mctx_lz4_decompress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem);

/* Zstandard decompression (load side of "zstd" volumes):
 * ZStandard.Decompress of pkg/compress (compress.go:93-100,
 * github.com/DataDog/zstd v1.5.0 -> ZSTD_decompress), as cachedStore.load
 * calls it (cached_store.go:680-745).  Each zblk's src holds zstd frames
 * (concatenated frames and skippable frames allowed, as ZSTD_decompress);
 * out_len = decoded bytes; status JFSX_EFORMAT where ZSTD_decompress returns
 * an error (malformed frame, dictionary id, checksum mismatch, or output
 * larger than dst_cap); dst_cap < 2^31, src_len <= 0x7E000000 (JFSX_EINVAL
 * otherwise).  A frame that is well formed as far as it was decoded but does
 * not fit in dst_cap gets JFSX_EDSTSIZE (ZSTD_decompress's
 * dstSize_tooSmall): the caller can retry with the frame content size. */
int jfsx_zstd_decompress_batch(jfsx_ctx *ctx, int n, jfsx_zblk *blks, int mem);
/* per block through the aggregator, and over a multi-device context */
int jfsx_agg_zstd_decompress(jfsx_agg *agg, jfsx_zblk *blk, int mem);
int jfsx_mctx_zstd_decompress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem);

/* Zstandard compression (upload side of "zstd" volumes):
 * ZStandard.Compress of pkg/compress (compress.go:82-91,
 * zstd.CompressLevel(dst, src, 1) -> ZSTD_compress(dst, bound, src, n, 1)), as
 * cachedStore.upload calls it before the Put (cached_store.go:371-392, :387).
 * Each zblk's dst receives one level-1 frame, out_len bytes, byte for byte
 * what the zstd library's one-shot level-1 compressor writes (checked against
 * the system libzstd 1.4.8; see DESIGN.md for the 1.5.0 the reference pins).
 * dst_cap >= jfsx_zstd_bound(src_len) (JFSX_EINVAL otherwise), as upload's
 * CompressBound-sized buffer; src_len <= 0x7E000000. */
uint64_t jfsx_zstd_bound(uint64_t n); /* ZSTD_compressBound */
int jfsx_zstd_compress_batch(jfsx_ctx *ctx, int n, jfsx_zblk *blks, int mem);
int jfsx_agg_zstd_compress(jfsx_agg *agg, jfsx_zblk *blk, int mem);
int jfsx_mctx_zstd_compress_batch(jfsx_mctx *m, int n, jfsx_zblk *blks, int mem);

/* header helper: returns wrapped-key length and offset/size of the nonce so a
 * caller can unwrap the key first (encrypt.go:197-205) */
int jfsx_parse_header(const void *obj, uint64_t olen, int *klen, int *nlen);

/* synthetic input generator used by bench/tests: fills len bytes of device
 * memory with the SplitMix64 stream of (seed, block) (documented in
 * DESIGN.md; identical to oracle/jfs_oracle.c:orc_gen_block) */
int jfsx_gen_synthetic(jfsx_ctx *ctx, void *dst, uint64_t len, uint64_t seed, uint64_t block);
/* batched form: block i (global index block0 + i) is written at
 * dst + i*stride with lens[i] bytes (lens: host array), one launch for the
 * whole batch */
int jfsx_gen_synthetic_batch(jfsx_ctx *ctx, void *dst, uint64_t stride, int n, const uint64_t *lens, uint64_t seed,
                             uint64_t block0);
/* fills n keys (32 B) and nonces (12 B) with the same per-block stream as
 * orc_gen_key, host side */
void jfsx_gen_key(uint64_t seed, uint64_t block, uint8_t key[32], uint8_t nonce[12]);

/* PCIe probe on the streams the host-ingest ring uses (H2D stream, D2H
 * stream): `bytes` between engine-pinned host memory and device memory in
 * 8 chunks per direction, best of 3; out[0] H2D alone, out[1] D2H alone,
 * out[2] / out[3] H2D / D2H rate while both directions run at once (chunks
 * issued alternately, as the ring issues them), in GB/s.  The ring moves equal
 * bytes up and down, so min(out[2], out[3]) bounds a host-ingest seal. */
int jfsx_pcie_probe(jfsx_ctx *ctx, uint64_t bytes, double out[4]);

/* diagnostics: the lookup tables the kernels stage into LDS, built on the host
 * without a device (AES T0|T2 x32 replicated: 16384 dwords; CRC32C slice-by-16
 * and 1008/4032/1024/4096-byte shift tables: 8192 dwords; CRC lane/power constants: 192) */
int jfsx_debug_tables(uint32_t *aes, uint32_t *crc, uint32_t *crcx);

#ifdef __cplusplus
}
#endif
#endif /* JFSX_H */
