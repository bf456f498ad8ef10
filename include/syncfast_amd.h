/*
 * syncfast_amd.h -- C-ABI of the MI355X block-signature indexing path.
 *
 * Drop-in boundary for the hot path of syncfast's Index::index_file
 * (/root/reference/src/index.rs:610-659): file bytes -> one
 * (offset, size, SHA-1) row per block, plus the per-file blocks_hash
 * (src/index.rs:661-682).  The reference exposes no FFI of its own; the seam
 * it replaces is the loop at src/index.rs:621-647 that hands
 * (HashDigest, offset, size) tuples to Index::add_block (src/index.rs:387-408).
 * INTEGRATION.md shows the Rust `extern "C"` binding a maintainer would add.
 *
 * Conventions
 *  - Plain pointers and sizes only.  "d_" pointers are device (HBM) pointers
 *    on the current HIP device; `stream` is a hipStream_t passed as void*
 *    (NULL = the null stream).  Device entry points are asynchronous on
 *    `stream` and may be called from several host threads on different
 *    streams.
 *  - Return 0 on success, a negative errno-style SF_E* code otherwise; the
 *    Rust side maps them to Error::Io (src/lib.rs:25), as the reference
 *    propagates I/O errors with `?` (src/index.rs:615,630) and exposes no
 *    partial results.
 *  - Digests are the 20 bytes of sha1.digest().bytes() (big-endian SHA-1),
 *    exactly HashDigest's field (src/lib.rs:72-76), stored back to back:
 *    block i at byte 20*i.
 *  - Fixed tiling: block i = bytes [i*B, min((i+1)*B, len)).  No empty
 *    blocks: len == 0 gives 0 blocks, and there is no trailing empty block
 *    when len % B == 0 (the reference only emits a block on ChunkInput::End
 *    after data, src/index.rs:629-646).
 *  - blocks_hash of a file with no blocks is SHA1("") =
 *    da39a3ee5e6b4b0d3255bfef95601890afd80709.
 */
#ifndef SYNCFAST_AMD_H
#define SYNCFAST_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SF_HASH_DIGEST_LEN 20 /* HASH_DIGEST_LEN, src/lib.rs:72 */
#define SF_MAX_BLOCK_SIZE (32u << 20) /* fixed-tiling block size limit (32 MiB) */

#define SF_OK 0
#define SF_EIO (-5)      /* file read failed */
#define SF_EAGAIN (-11)  /* the file changed under the call (fd routes): cut it again and retry */
#define SF_ENOMEM (-12)  /* device, pinned or host allocation failed, or the system refused a thread */
#define SF_ENODEV (-19)  /* no HIP device, or a HIP runtime error */
#define SF_EINVAL (-22)  /* bad argument */
#define SF_ENOSPC (-28)  /* output capacity too small; *n_out holds the need */
#define SF_ERANGE (-34)  /* a block lies outside [0, len) */
#define SF_ETIMEDOUT (-110) /* kept for callers: no call returns it since round 6 (no kernel waits) */

/* One signature row: what index_file passes to add_block
 * (src/index.rs:636-642) and what FILE_BLOCK carries on the wire
 * (src/sync/ssh/proto.rs:162-166).  32 bytes. */
typedef struct sf_block_sig {
    uint64_t offset;
    uint32_t size;
    uint8_t sha1[SF_HASH_DIGEST_LEN];
} sf_block_sig;

/* A file inside one device buffer (many-file batch, BASELINE config 3). */
typedef struct sf_file_desc {
    uint64_t offset; /* byte offset of the file in the batch buffer */
    uint64_t len;    /* file length in bytes */
} sf_file_desc;

/* ------------------------------------------------------------ runtime */
const char *sf_version(void);
const char *sf_strerror(int code);
/* Number of visible HIP devices (0 on a machine without one). */
int sf_device_count(int *n);
int sf_set_device(int device);
/* The host-memory entry points (sf_index_buffer, sf_index_file) keep their
 * per-device streams, stage buffers and digest tables between calls (setting
 * them up costs ~8 ms per call).  This frees them; the next call sets them up
 * again.  Blocks while another thread is inside such a call. */
int sf_release_host_cache(void);

/* --------------------------------------- device-resident hot path ---- */

/* Scratch: calls that need device workspace on `stream` (an explicit list's
 * length sort, a batch's chain states, wire offsets, block-set slots) take it
 * stream-ordered from a memory pool of the library's own per device, which
 * keeps every freed block for later calls (it holds its peak use: at most
 * ~1 GiB, for a sort of 2^27 blocks) and reuses a block only on the stream
 * that freed it.  The device's default pool is not used: its blocks, given
 * back at every synchronisation and mapped again, made calls read wrong data
 * (DESIGN.md 3.4).  The caller's own allocations are not touched. */

/* Fixed tiling of d_data[0, len) into block_size-byte blocks; writes
 * ceil(len/block_size) digests to d_digests (20 B each).  Replaces the
 * chunk loop of src/index.rs:621-647 for fixed-size blocks.
 * SF_ENOSPC (with *n_blocks set) when cap_blocks is too small. */
int sf_index_device_fixed(const void *d_data, uint64_t len, uint32_t block_size,
                          void *d_digests, uint64_t cap_blocks, uint64_t *n_blocks,
                          void *stream);

/* Explicit block list: block i = d_data[d_offsets[i], d_offsets[i] + d_sizes[i]).
 * Used for content-defined boundaries (src/index.rs:622-625 produces them
 * in the reference), the reference KAT boundaries and ragged batches.
 * Blocks need not be sorted, aligned or disjoint.  A block outside
 * [0, len) is not read: its digest is zeroed and, if d_status != NULL,
 * *d_status (device int32, caller-initialised to 0) is set to SF_ERANGE. */
int sf_index_device_blocks(const void *d_data, uint64_t len, const uint64_t *d_offsets,
                           const uint32_t *d_sizes, uint64_t n_blocks, void *d_digests,
                           int *d_status, void *stream);

/* Opt-in weak checksum -- NOT part of the reference (SURVEY.md 8a row a8:
 * syncfast stores and sends no weak sum); north_star names an "Adler32-style"
 * weak sum beside the strong hash.  As sf_index_device_fixed /
 * sf_index_device_blocks, plus d_weak[i] = zlib Adler-32 (RFC 1950) of block
 * i's bytes, fused into the same pass over HBM (uint32 per block; 0 for an
 * out-of-range explicit block). */
int sf_index_device_fixed_weak(const void *d_data, uint64_t len, uint32_t block_size,
                               void *d_digests, uint32_t *d_weak, uint64_t cap_blocks,
                               uint64_t *n_blocks, void *stream);
int sf_index_device_blocks_weak(const void *d_data, uint64_t len, const uint64_t *d_offsets,
                                const uint32_t *d_sizes, uint64_t n_blocks, void *d_digests,
                                uint32_t *d_weak, int *d_status, void *stream);

/* Many-file batch: files[] (host array) describes n_files files inside
 * d_data[0, len).  Writes every file's fixed-size block digests, file after
 * file, to d_digests (cap_blocks rows) and, if d_file_hashes != NULL, each
 * file's blocks_hash (20 B per file, src/index.rs:661-682) computed on the
 * device.  first_block (host, n_files+1 entries, may be NULL) receives the
 * index of each file's first digest row; *n_blocks the total.  Asynchronous
 * on `stream` (ragged batches upload a small block table, stream-ordered).
 * Equal-size batches with d_file_hashes are hashed in two column halves, the
 * first half of every file's blocks_hash chain beside the second half's
 * blocks, then the chains' second half (the batch stream's last batch,
 * sf_index_device_batch_chained_cols): no wave waits for another, so no
 * bound and no timeout (round 6; until then one fused launch whose chain
 * lanes polled and, once, gave up).  d_status (device int32, may be NULL) is
 * accepted for source compatibility and is not written: no error of this
 * call is reported on the device.  (SF_BATCH_FUSED=0: the block kernel, then
 * a chain kernel.) */
int sf_index_device_batch(const void *d_data, uint64_t len, const sf_file_desc *files,
                          uint32_t n_files, uint32_t block_size, void *d_digests,
                          uint64_t cap_blocks, void *d_file_hashes, uint64_t *first_block,
                          uint64_t *n_blocks, int *d_status, void *stream);

/* Per-file blocks_hash (src/index.rs:661-682) of a batch of equal-size files
 * already hashed into d_digests (n_files files x blocks rows, blocks a
 * multiple of 4): part 0 = whole chains -> d_hashes (20 B per file);
 * part 1 = first half of every chain -> d_state (20 B per file);
 * part 2 = second half, resumed from d_state -> d_hashes. */
typedef struct sf_chain_job {
    const void *d_digests;
    uint32_t n_files;
    uint32_t part;
    uint64_t blocks;
    void *d_state;
    void *d_hashes;
} sf_chain_job;

/* Equal-size many-file batches as a stream (BASELINE config 3, batch after
 * batch, the shape of index_path over a large tree): ONE launch on `stream`
 * hashes every block of this batch -- n_files files of file_len bytes (a
 * multiple of block_size) back to back at d_data -- into d_digests
 * (file-major rows) and, in the same launch, up to two chain jobs of EARLIER
 * batches (digests and states written by earlier launches on the same
 * stream), so their blocks_hash latency hides behind this batch's blocks.
 * n_files = 0 runs only the jobs.  A batch of more than 2^31 blocks is
 * SF_EINVAL (one launch per batch; the other entry points split such inputs
 * into several launches themselves). */
int sf_index_device_batch_chained(const void *d_data, uint32_t n_files, uint64_t file_len,
                                  uint32_t block_size, void *d_digests, const sf_chain_job *jobs,
                                  uint32_t n_jobs, void *stream);

/* The same launch over block columns [col_lo, col_hi) of every file only
 * (rows f * (file_len / block_size) + col of d_digests; the other rows are
 * not written).  col_lo = 0, col_hi = file_len / block_size is
 * sf_index_device_batch_chained; any other range needs 64 | blocks per file,
 * 64 | col_lo, 64 | col_hi and col_lo < col_hi <= blocks per file, else
 * SF_EINVAL.  A stream's LAST batch in two column halves lets the first half
 * of its chains run inside the second launch (device.BatchStream.push_last). */
int sf_index_device_batch_chained_cols(const void *d_data, uint32_t n_files, uint64_t file_len,
                                       uint32_t block_size, uint64_t col_lo, uint64_t col_hi,
                                       void *d_digests, const sf_chain_job *jobs, uint32_t n_jobs,
                                       void *stream);

/* ------------------------------------ the receiving side of a sync ---- */

/* Block lookup of a sync destination.  For every FILE_BLOCK of an incoming
 * file, FsDestinationInner::sink (src/sync/fs.rs:461-476) asks its index
 * whether it holds that block: Index::get_block (src/index.rs:77-103), the
 * first row with that hash and present = 1, SQLite's (hash, rowid) index
 * order.  A block set is that question for a whole table at once: built on
 * the device from the destination's rows -- d_table, n_rows x 20-B digests in
 * rowid order (4-B aligned; the caller keeps it alive while the set is used),
 * d_present, one byte per row (non-zero = present; NULL = all present) --
 * then sf_block_set_lookup writes, for each of n_query digests at d_query,
 * the index of the first present row with that digest, or -1, to d_rows
 * (device int64).  Asynchronous on `stream`; n_rows <= 2^31.  Lookups only
 * read the set: any number may run at once, on any streams ordered after the
 * build.  sf_block_set_free releases the set (stream-ordered: after the
 * lookups on that stream). */
typedef struct sf_block_set sf_block_set;
int sf_block_set_build(const void *d_table, const uint8_t *d_present, uint64_t n_rows,
                       sf_block_set **out, void *stream);
int sf_block_set_lookup(const sf_block_set *set, const void *d_query, uint64_t n_query,
                        int64_t *d_rows, void *stream);
int sf_block_set_free(sf_block_set *set, void *stream);

/* The signature table as the reference's wire messages, on the device:
 * n_blocks FILE_BLOCK messages, "FILE_BLOCK\n" + 20 digest bytes + "\n" +
 * decimal block size + "\n" (write_message, src/sync/ssh/proto.rs:162-166),
 * what FsSource sends per block after FILE_START (src/sync/fs.rs:217-233).
 * Fixed tiling of a file_len-byte file.  *n_out = bytes written (the need,
 * with SF_ENOSPC, when cap is too small). */
int sf_wire_file_blocks_device(const void *d_digests, uint64_t n_blocks, uint32_t block_size,
                               uint64_t file_len, void *d_out, uint64_t cap, uint64_t *n_out,
                               void *stream);

/* The FILE_BLOCK run of an explicit block list -- the reference's default,
 * content-defined blocks, each with its own size -- built in HBM: message i =
 * "FILE_BLOCK\n" + digest i + "\n" + decimal d_sizes[i] + "\n"
 * (src/sync/ssh/proto.rs:162-166), back to back in list order.  The message
 * offsets come from a scan on the device; the total is read back, so the call
 * blocks until it is known.  *n_out = bytes (the need); SF_ENOSPC when cap is
 * too small or d_out is NULL (a query). */
int sf_wire_blocks_device(const void *d_digests, const uint32_t *d_sizes, uint64_t n_blocks,
                          void *d_out, uint64_t cap, uint64_t *n_out, void *stream);

/* The same FILE_BLOCK run written to a file descriptor (the SSH pipe of
 * src/sync/ssh/mod.rs, or a file), streamed: the device builds ~1M messages
 * at a time, each chunk comes back by DMA into pinned memory and is written
 * while the device builds the next.  d_digests may still be in production on
 * `stream` (the copy waits for it).  *n_written = bytes written.  Blocking. */
int sf_wire_file_blocks_fd(const void *d_digests, uint64_t n_blocks, uint32_t block_size,
                           uint64_t file_len, int fd, uint64_t *n_written, void *stream);

/* The explicit list's FILE_BLOCK run (sf_wire_blocks_device) streamed to a
 * file descriptor in chunks of messages, each built on the device, copied
 * back and written while the next is built.  *n_written = bytes written.
 * Blocking. */
int sf_wire_blocks_fd(const void *d_digests, const uint32_t *d_sizes, uint64_t n_blocks, int fd,
                      uint64_t *n_written, void *stream);

/* Deterministic synthetic input (bench / tests): bytes [start, start+len)
 * of the splitmix64 stream with this seed. */
int sf_fill_splitmix_device(void *d_out, uint64_t len, uint64_t seed, uint64_t start, void *stream);

/* ------------------------------------------------ host-memory entries */


/* End to end from host memory: H2D in pipelined chunks, fixed-tiling kernel,
 * D2H of the signature rows.  Blocking.  out has cap rows. */
int sf_index_buffer(const uint8_t *data, uint64_t len, uint32_t block_size,
                    sf_block_sig *out, uint64_t cap, uint64_t *n_out);

/* End to end from host memory with an explicit block list: block i =
 * data[offsets[i], offsets[i] + sizes[i]) -- the boundaries a chunker on the
 * host produced (the reference's default is cdchunking's ZPAQ,
 * src/index.rs:622-625: a Rust caller keeps that crate, runs it over the
 * file's bytes and hands the bytes + boundaries here).  Replaces the
 * Sha1::update / digest loop of src/index.rs:628-644 for every block.
 * Blocks must be in non-decreasing offset order (a chunker's output; they
 * may overlap and need not cover the buffer); sizes may be 0 (SHA-1 of no
 * bytes).  The list is checked before anything runs: SF_ERANGE if a block
 * passes len, SF_EINVAL if the offsets go backwards.  Stages of about
 * 256 MiB of whole blocks are copied (16 threads) into pinned buffers, moved
 * to HBM with their part of the list and hashed by the explicit-list kernel
 * while the next stage is copied.  out[i] = {offsets[i], sizes[i], digest};
 * blocks_hash (may be NULL) = SHA-1 over the digests in list order
 * (compute_blocks_hash, src/index.rs:661-682).  n_blocks rows; blocking. */
int sf_index_buffer_blocks(const uint8_t *data, uint64_t len, const uint64_t *offsets,
                           const uint32_t *sizes, uint64_t n_blocks, sf_block_sig *out,
                           uint8_t blocks_hash[SF_HASH_DIGEST_LEN]);

/* The same list over a regular file on disk: the caller's chunker streamed
 * the file once to find the boundaries (cdchunking's stream(file),
 * src/index.rs:625), and the library reads each ~256 MiB window again with
 * pread (16 threads) into the pinned stages -- the file is never held whole
 * in memory.  List checked against the file's size first (SF_ERANGE /
 * SF_EINVAL as above); SF_EIO if it cannot be opened or is not a regular
 * file; SF_EAGAIN if it changes while being read (stamps as in
 * sf_index_fd_blocks).  Rows in list order + blocks_hash; blocking.
 * The path is opened a second time here, after the chunker's open: a file
 * renamed over the path in between is hashed with the old file's
 * boundaries.  The drop-in splice uses sf_index_fd_blocks on the chunker's
 * own descriptor instead. */
int sf_index_file_blocks(const char *path, const uint64_t *offsets, const uint32_t *sizes,
                         uint64_t n_blocks, sf_block_sig *out, uint8_t blocks_hash[SF_HASH_DIGEST_LEN]);

/* What fstat says about an open file's contents: the identity of the bytes a
 * chunker read through that descriptor.  Two stamps match when dev, ino,
 * size and mtime are equal and, unless the link count changed, ctime too:
 * ctime moves on every write and cannot be set back by the writer (mtime
 * can), but it also moves when a link is added or removed -- a file renamed
 * over the path unlinks the open one, which changes nothing it holds.
 * Timestamps are only as fine as the filesystem's clock tick: a write within
 * the same tick as the stamp is not seen. */
typedef struct sf_file_stamp {
    uint64_t dev, ino, size, nlink;
    int64_t mtime_sec, mtime_nsec;
    int64_t ctime_sec, ctime_nsec;
} sf_file_stamp;

/* fstat(fd) as a stamp.  SF_EIO if fstat fails. */
int sf_file_stamp_fd(int fd, sf_file_stamp *out);

/* The explicit list over the regular file OPEN on fd -- the handle the caller's
 * chunker just streamed (index_file opens the file once and takes the mtime,
 * the boundaries and the bytes from that one handle, src/index.rs:615-625).
 * Reads with pread only (the descriptor's position is not used or moved), by
 * ~256 MiB windows as sf_index_file_blocks.  A rename over the path after the
 * open changes nothing: the descriptor still reads the file the chunker cut.
 * expect (may be NULL): the stamp taken before the chunker read the file
 * (sf_file_stamp_fd); if the file's stamp differs when the call starts, or
 * changes between then and the last window read (an in-place write, append
 * or truncation), the call returns SF_EAGAIN and the rows are not valid: the
 * caller takes a new stamp and cuts the file again.  SF_EINVAL if fd is not a
 * regular file (a pipe cannot be read twice: use sf_index_buffer_blocks);
 * SF_ERANGE / SF_EINVAL for the list as sf_index_file_blocks.  Blocking. */
int sf_index_fd_blocks(int fd, const sf_file_stamp *expect, const uint64_t *offsets, const uint32_t *sizes,
                       uint64_t n_blocks, sf_block_sig *out, uint8_t blocks_hash[SF_HASH_DIGEST_LEN]);

/* Fixed tiling of the regular file open on fd, [0, size at the call), through
 * the pread pipeline of sf_index_file, with the same stamp checks as
 * sf_index_fd_blocks (SF_EAGAIN: the file changed; the rows are not valid).
 * SF_ENOSPC with *n_out = the need when cap is too small (nothing is read).
 * SF_EINVAL if fd is not a regular file (use sf_index_fd).  Blocking. */
int sf_index_fd_fixed(int fd, const sf_file_stamp *expect, uint32_t block_size, sf_block_sig *out,
                      uint64_t cap, uint64_t *n_out, uint8_t blocks_hash[SF_HASH_DIGEST_LEN]);

/* End to end from a file on disk (the reference's input, src/index.rs:615):
 * pread into pinned buffers, overlapped H2D + kernel, D2H.  Writes the
 * rows and the file's blocks_hash.  Blocking.  A path that cannot seek (FIFO,
 * socket, character device) is read sequentially to EOF like File::open +
 * read (src/index.rs:615,625); its input is consumed, so when the rows
 * exceed cap the call returns SF_ENOSPC with *n_out = the need and the rows
 * are lost -- use sf_index_fd for such inputs. */
int sf_index_file(const char *path, uint32_t block_size, sf_block_sig *out, uint64_t cap,
                  uint64_t *n_out, uint8_t blocks_hash[SF_HASH_DIGEST_LEN]);

/* One shard of a file on disk: bytes [start, start+len) of a regular file
 * (start a multiple of block_size unless len == 0; the shard's last block
 * may be short only where the file ends), through the same pread pipeline
 * as sf_index_file.
 * Row offsets are FILE offsets, so the shards' rows concatenated in order
 * are the file's rows (src/index.rs:629-656).  No blocks_hash: it chains
 * over every digest of the file, so the rank that gathers the shards'
 * digests computes it (sf_blocks_hash).  SF_ERANGE if the range passes the
 * end of the file.  Blocking. */
int sf_index_file_range(const char *path, uint64_t start, uint64_t len, uint32_t block_size,
                        sf_block_sig *out, uint64_t cap, uint64_t *n_out);

/* Sequential input from an open file descriptor (pipe, FIFO, socket, or a
 * file read from its current position), read to EOF: the rows of its fixed
 * tiling, offsets from the first byte read, in a buffer the library
 * allocates and grows (*rows; release it with sf_free_rows), and its
 * blocks_hash.  Pinned double-buffered stages, each copied and hashed on
 * the device while the next is read.  Does not close fd.  Blocking. */
int sf_index_fd(int fd, uint32_t block_size, sf_block_sig **rows, uint64_t *n_out,
                uint8_t blocks_hash[SF_HASH_DIGEST_LEN]);
void sf_free_rows(sf_block_sig *rows);

/* Many files from disk: what index_path (src/index.rs:685-715) does by calling
 * index_file (src/index.rs:610-659) once per file, as ONE pipeline.  Fixed
 * tiling of every file.  Files are packed at 16-B aligned offsets into pinned
 * stages of about stage_bytes (0 = 256 MiB) by a pool of pread threads; each
 * stage is copied to HBM and hashed (blocks + every file's blocks_hash,
 * src/index.rs:661-682) while the next stage is read.  A file larger than a
 * stage goes through the one-file pipeline of sf_index_file.
 * out: the rows of file 0, then file 1, ... (offsets relative to each file);
 * first_row (n_files+1 entries): where each file's rows start;
 * blocks_hashes: 20 B per file.  *n_out = total rows (the need, with
 * SF_ENOSPC, checked before any file is read).  On SF_EIO (open, stat or a
 * short read: the file changed while being indexed) *bad_file (may be NULL)
 * is the index of the failing file.  Each stage's blocks and blocks_hash
 * chains go through sf_index_device_batch.  Blocking. */
int sf_index_files(const char *const *paths, uint32_t n_files, uint32_t block_size, uint64_t stage_bytes,
                   sf_block_sig *out, uint64_t cap, uint64_t *first_row, uint8_t *blocks_hashes,
                   uint64_t *n_out, uint32_t *bad_file);

/* Many files in the reference's default mode: what index_path
 * (src/index.rs:685-715) does with one index_file (src/index.rs:610-659) per
 * file, each file cut by the caller's chunker (cdchunking's ZPAQ,
 * src/index.rs:622-625) on its own open descriptor, as ONE pipeline.  File f
 * is the regular file open on fds[f]; stamps[f] (stamps may be NULL) its
 * sf_file_stamp_fd taken before the chunker read it; its list is block i =
 * [offsets[f][i], offsets[f][i] + sizes[f][i]) for i < n_blocks[f],
 * offset-ordered (a chunker's output).  The files are read again with pread
 * only (the descriptors' positions are not used or moved), by windows packed
 * into pinned stages of about stage_bytes (0 = 256 MiB; a window of one
 * larger block is a stage of its own) by a pool of reader threads; per stage
 * one H2D copy, one length-class sort + one explicit-list kernel launch over
 * every block of every file in it, one D2H, overlapped with the reading of
 * the next stage.  out: file 0's rows, then file 1's, ... (offsets relative
 * to each file); first_row (n_files + 1 entries): where each file's rows
 * start (written first, from n_blocks); blocks_hashes: 20 B per file,
 * compute_blocks_hash (src/index.rs:661-682) over its digests in list order
 * (SHA1("") for a file with no blocks).  SF_ENOSPC (nothing read) when cap <
 * first_row[n_files].  Each file succeeds or fails alone: file_status (may be
 * NULL, n_files entries) receives SF_OK or, for that file, SF_EAGAIN (its
 * stamp differs from stamps[f] at the call, or moved before its last window
 * was read: cut it again), SF_ERANGE / SF_EINVAL (its list: past the end of
 * the file / offsets going backwards), SF_EINVAL (fds[f] is not an open
 * regular file), SF_EIO (fstat or a read failed); a failed file's rows are not
 * valid and its blocks_hash is zeroed, every other file's are complete.  The
 * call returns SF_OK, or the first failing file's code with *bad_file (may be
 * NULL) = its index; a device error fails the whole call.  Blocking. */
int sf_index_fds_blocks(const int *fds, const sf_file_stamp *stamps, uint32_t n_files,
                        const uint64_t *const *offsets, const uint32_t *const *sizes, const uint64_t *n_blocks,
                        uint64_t stage_bytes, sf_block_sig *out, uint64_t cap, uint64_t *first_row,
                        uint8_t *blocks_hashes, int *file_status, uint32_t *bad_file);

/* -------------------------------- the caller's chunker, on N threads ---- */

/* A content-defined chunker of the caller's (cdchunking's ZPAQ with its
 * max_size cap, src/index.rs:622-625, on the Rust side), as three functions:
 *   create(ctx)       a fresh chunker: the state at a chunk's first byte;
 *   next(ch, p, n)    feeds p[0, n): the number of bytes up to and including
 *                     the next boundary, or 0 if the chunk goes on past p + n;
 *                     after a boundary the state is a fresh chunk's again;
 *   destroy(ch).
 * The chunker must restart at every boundary (its state after a boundary is a
 * fresh chunker's, which read_block relies on, src/sync/fs.rs:26-40): then
 * the boundaries are a function of where a chunk starts, which is what lets
 * sf_cut_fd cut one file on several threads and still return exactly the
 * sequential boundaries.  Called from the library's threads, one chunker
 * per thread at a time. */
typedef struct sf_chunker_ops {
    void *(*create)(void *ctx);
    size_t (*next)(void *chunker, const uint8_t *p, size_t n);
    void (*destroy)(void *chunker);
    void *ctx;
} sf_chunker_ops;

/* The boundaries of the regular file open on fd (pread only; the position is
 * not used), cut by `ops`, exactly as one chunker streaming the file from its
 * first byte would cut it (the loop of src/index.rs:629-647 without the
 * SHA-1).  With threads > 1 (0 = the library's reader count) the file is
 * split into up to `threads` segments of at least 4 MiB (a file under 8 MiB is
 * cut on one thread); a chunker starts
 * fresh at each segment's first byte and cuts speculatively; the segments are
 * then joined left to right: from the last boundary known to be right, the
 * file is cut again on one thread only until a boundary coincides with one of
 * the next segment's, after which (the chunker restarting at every boundary)
 * the two agree.  The result never depends on the thread count.  *offsets /
 * *sizes (n_blocks entries; allocated by the library, release both with
 * sf_free_cuts) are the blocks in file order; an empty file has none.
 * expect (may be NULL): the caller's sf_file_stamp_fd; the file's stamp is
 * compared with it at the start and with the one taken at the start after the
 * last read: SF_EAGAIN if it changed (cut it again).  SF_EINVAL if fd is not
 * a regular file or ops is incomplete, SF_EIO on a failed or short read,
 * SF_ENOMEM.  Host only (no device).  Blocking. */
int sf_cut_fd(int fd, const sf_file_stamp *expect, const sf_chunker_ops *ops, uint32_t threads,
              uint64_t **offsets, uint32_t **sizes, uint64_t *n_blocks);
void sf_free_cuts(void *p);

/* index_file (src/index.rs:610-659) in the default mode for one regular file
 * open on fd, with the caller's chunker on several threads: the boundaries
 * of sf_cut_fd (exactly the one-stream ones) and every block's SHA-1 and the
 * blocks_hash on the device, with the file read ONCE: each segment is read
 * into a pinned copy of the file by the thread that cuts it, copied to HBM
 * while the segments are cut and joined, and the joined list is hashed from
 * there -- by windows of up to 512 MiB, each ending at the last boundary
 * inside it (the next window starts there).  *rows (n_out entries, allocated by
 * the library, release with sf_free_rows) and blocks_hash as sf_index_fd_blocks
 * gives them.  expect / SF_EAGAIN / errors as sf_cut_fd.  Blocking. */
int sf_index_fd_cut(int fd, const sf_file_stamp *expect, const sf_chunker_ops *ops, uint32_t threads,
                    sf_block_sig **rows, uint64_t *n_out, uint8_t blocks_hash[SF_HASH_DIGEST_LEN]);

/* ------------------------------------------- one process, N devices ---- */

/* Contiguous, block-aligned shard `shard` of n_shards of a file_len-byte file:
 * bytes [*start, *start + *len).  Blocks are dealt as evenly as possible (the
 * first nblocks % n_shards shards get one more); a shard may be empty.  The
 * shards' rows concatenated in shard order are the file's rows.  The
 * partition every multi-device form below uses (and syncfast_amd.shard's
 * shard_range, one process per GPU). */
int sf_shard_range(uint64_t file_len, uint32_t block_size, uint32_t n_shards, uint32_t shard, uint64_t *start,
                   uint64_t *len);

/* index_file (src/index.rs:610-659) of one regular file on N devices of this
 * process: fixed tiling, shard r (sf_shard_range) read with pread from ONE
 * open of the file and hashed on device r by a host thread of its own (each
 * device on its own PCIe link, through the staged pipeline of sf_index_file),
 * rows written straight into out at the shard's first row; then blocks_hash
 * over every digest in order on the host (it chains over the whole file).
 * n_devices = 0: every visible device; devices 0 .. n_devices-1 are used.
 * The file is stamped at the open and again after the last read: SF_EAGAIN
 * if it changed (the rows are not valid).  SF_ENOSPC with *n_out = the need
 * when cap is too small (nothing read); SF_EINVAL if path is not a regular
 * file or n_devices exceeds the visible devices.  The calling thread's current
 * device is left as it was.  Blocking. */
int sf_index_file_multi(const char *path, uint32_t block_size, uint32_t n_devices, sf_block_sig *out, uint64_t cap,
                        uint64_t *n_out, uint8_t blocks_hash[SF_HASH_DIGEST_LEN]);

/* The device-resident form on N devices of this process, the gather over
 * xGMI inside the library: d_shards[r] (on device r) holds shard r
 * (sf_shard_range of file_len, block_size, n_devices) of one logical file;
 * each shard is hashed on its own device, on streams[r] (streams may be NULL:
 * each device's null stream), the root's straight into its rows of d_table
 * (device `root`, ceil(file_len / block_size) x 20 B), every other device's
 * into d_digests[r] (its own scratch, its shard's rows x 20 B) and from there
 * to its rows of d_table with RCCL (one communicator per device list,
 * ncclCommInitAll on first use, kept; grouped ncclSend / ncclRecv, since the
 * shards' row counts may differ by one).  Asynchronous: d_table is complete
 * once streams[root] has run past the call.  Devices 0 .. n_devices-1; the
 * caller's current device is left as it was.  SF_ENODEV if RCCL cannot be
 * loaded or a communicator not made. */
int sf_index_device_multi(uint32_t n_devices, const void *const *d_shards, uint64_t file_len, uint32_t block_size,
                          void *const *d_digests, uint32_t root, void *d_table, void *const *streams);

/* sf_index_device_multi with the exchange on streams of its own: shard r is
 * hashed on hash_streams[r] (NULL: each device's null stream) and sent -- and,
 * on the root, received -- on gather_streams[r], which first waits for device
 * r's hashing (an event the library records on hash_streams[r]; NULL
 * gather_streams: the hash streams, i.e. sf_index_device_multi).  A caller
 * indexing file after file (each file's table gathered to its owner, config
 * 4 of BASELINE.json over and over) can then hash file i+1 while file i's
 * tables are in flight: d_digests[r] may be written again, and d_table read,
 * once gather_streams[r] / gather_streams[root] have run past the call.
 * Errors as sf_index_device_multi. */
int sf_index_device_multi_ex(uint32_t n_devices, const void *const *d_shards, uint64_t file_len,
                             uint32_t block_size, void *const *d_digests, uint32_t root, void *d_table,
                             void *const *hash_streams, void *const *gather_streams);

/* compute_blocks_hash (src/index.rs:661-682) on the host: SHA-1 over the
 * n 20-byte digests in order.  Sequential by definition; runs on a host
 * core (SHA-NI when the CPU has it). */
int sf_blocks_hash(const uint8_t *digests, uint64_t n, uint8_t out[SF_HASH_DIGEST_LEN]);
int sf_blocks_hash_sigs(const sf_block_sig *sigs, uint64_t n, uint8_t out[SF_HASH_DIGEST_LEN]);

/* Host SHA-1 of an arbitrary byte range (the same function as the
 * reference's sha1 crate; used for blocks_hash and host-side checks). */
int sf_sha1_host(const uint8_t *data, uint64_t len, uint8_t out[SF_HASH_DIGEST_LEN]);

#ifdef __cplusplus
}
#endif

#endif /* SYNCFAST_AMD_H */
