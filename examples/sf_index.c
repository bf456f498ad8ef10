/* sf_index.c -- a plain-C consumer of the C-ABI (include/syncfast_amd.h).
 *
 * What the Rust side of syncfast would do through its extern "C" binding
 * (INTEGRATION.md), with no Python and no PyTorch: index each path given on
 * the command line with fixed-size blocks and print, per file, its rows as
 * "offset size sha1hex" and its blocks_hash -- the rows Index::index_file
 * inserts (src/index.rs:636-642) and the value compute_blocks_hash stores
 * (src/index.rs:649-682).  Regular files go through sf_index_file, anything
 * else (a FIFO, "-" for stdin) through sf_index_fd.
 *
 *   cc -O2 -I include examples/sf_index.c -L syncfast_amd/lib -lsyncfast_amd \
 *      -Wl,-rpath,$PWD/syncfast_amd/lib -o sf_index
 *   ./sf_index [-b block_size] [-m | -B | -s N] path...
 *     -m: all paths through one sf_index_files call; -B: each file from a host
 *     buffer (sf_index_buffer); -C: each file cut by a content-defined chunker
 *     on the host, its blocks hashed by sf_index_buffer_blocks (and again by
 *     sf_index_file_blocks, which must agree);
 *     -s N: each file as N sf_index_file_range shards;
 *     -X N: each file on N devices of this process (sf_index_file_multi; 0 =
 *     every visible device);
 *     -w N: N synthetic bytes hashed in HBM, their FILE_BLOCK run to stdout;
 *     -v N: the same bytes cut by the host chunker (-C), hashed as a list in
 *     HBM, the list's FILE_BLOCK run to stdout (sf_wire_blocks_fd);
 *     -L dst src: src's blocks looked up among dst's (sf_block_set_*);
 *     -Z: the drop-in's default splice: each file opened once, streamed
 *     through a boundary chunker (the stand-in of zpaq_standin.h in place of
 *     the cdchunking crate), its list hashed from the same descriptor
 *     (sf_index_fd_blocks); -T adds a timing line per file on stderr;
 *     -Z -M: the default mode over many files (index_path): the files cut by
 *     -j N chunker threads, every batch of ~-S MiB of cut files hashed by ONE
 *     sf_index_fds_blocks call while the threads cut the next batch; -q
 *     prints only the first and last file's rows (every file's blocks_hash);
 *     -P n: the whole run n times in one process (the first pays the
 *     library's stage allocations), a timing line per pass; -K MiB: a file
 *     of at least this size (default 64, configs[0]'s file; 0 = never) is
 *     indexed alone in its place through sf_index_fd_cut on the -j threads
 *     (cut in parallel, read once) instead of being cut on one thread.
 * Regular files (default mode) go through the same one-open form:
 * sf_file_stamp_fd + sf_index_fd_fixed on the open descriptor.
 */
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "syncfast_amd.h"
#include "zpaq_standin.h"

/* -w only: device memory for the device-resident entry points (what a Rust
 * binding would take from hip-sys). */
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

static void hex(const uint8_t *d, char out[41]) {
    static const char digits[] = "0123456789abcdef";
    for (int i = 0; i < 20; i++) {
        out[2 * i] = digits[d[i] >> 4];
        out[2 * i + 1] = digits[d[i] & 15];
    }
    out[40] = 0;
}

static int print_rows(const char *name, const sf_block_sig *rows, uint64_t n, const uint8_t bh[20]) {
    char h[41];
    printf("file %s blocks %llu\n", name, (unsigned long long)n);
    for (uint64_t i = 0; i < n; i++) {
        hex(rows[i].sha1, h);
        printf("%llu %u %s\n", (unsigned long long)rows[i].offset, rows[i].size, h);
    }
    hex(bh, h);
    printf("blocks_hash %s\n", h);
    return 0;
}

/* One open, as index_file (src/index.rs:615-625): the stamp (what the
 * caller would take the mtime from) and the bytes come from the same
 * descriptor; a file written while it is read gives SF_EAGAIN and is read
 * again, at most 3 times. */
static int index_one(const char *path, uint32_t bs) {
    uint8_t bh[20];
    struct stat sb;
    const int is_stdin = strcmp(path, "-") == 0;
    const int fd = is_stdin ? 0 : open(path, O_RDONLY);
    if (fd < 0) return SF_EIO;
    if (!is_stdin && fstat(fd, &sb) == 0 && S_ISREG(sb.st_mode)) {
        int rc = SF_EAGAIN;
        for (int attempt = 0; attempt < 3 && (rc == SF_EAGAIN || rc == SF_ENOSPC); attempt++) {
            sf_file_stamp st;
            uint64_t n = 0;
            if ((rc = sf_file_stamp_fd(fd, &st)) != SF_OK) break;
            const uint64_t cap = st.size ? (st.size + bs - 1) / bs : 0;
            sf_block_sig *rows = malloc((cap ? cap : 1) * sizeof(sf_block_sig));
            if (!rows) { rc = SF_ENOMEM; break; }
            rc = sf_index_fd_fixed(fd, &st, bs, rows, cap, &n, bh);
            if (rc == SF_OK) print_rows(path, rows, n, bh);
            free(rows);
        }
        close(fd);
        return rc;
    }
    sf_block_sig *rows = NULL;
    uint64_t n = 0;
    const int rc = sf_index_fd(fd, bs, &rows, &n, bh);
    if (!is_stdin) close(fd);
    if (rc == SF_OK) print_rows(path, rows, n, bh);
    sf_free_rows(rows);
    return rc;
}

/* -B: the file read into a host buffer, then sf_index_buffer (the in-place
 * page-locked route from 1 MiB, the staged copy below); -s N: the file as N
 * shards through sf_index_file_range, rows concatenated (the multi-GPU
 * layout on one device), blocks_hash over all digests with sf_blocks_hash. */
static int index_buffer_or_shards(const char *path, uint32_t bs, int shards) {
    struct stat sb;
    if (stat(path, &sb) != 0 || !S_ISREG(sb.st_mode)) return SF_EIO;
    const uint64_t len = (uint64_t)sb.st_size, nb = len ? (len + bs - 1) / bs : 0;
    sf_block_sig *rows = malloc((nb ? nb : 1) * sizeof(sf_block_sig));
    uint8_t *dig = malloc((nb ? nb : 1) * 20), bh[20];
    uint64_t n = 0;
    int rc = (rows && dig) ? SF_OK : SF_ENOMEM;
    if (rc == SF_OK && shards <= 0) {
        uint8_t *buf = malloc(len ? len : 1);
        FILE *f = fopen(path, "rb");
        if (!buf || !f || fread(buf, 1, len, f) != len) rc = SF_EIO;
        if (f) fclose(f);
        if (rc == SF_OK) rc = sf_index_buffer(buf, len, bs, rows, nb, &n);
        free(buf);
    } else if (rc == SF_OK) {
        for (int r = 0; r < shards && rc == SF_OK; r++) {  /* shard_range: blocks dealt evenly */
            const uint64_t per = nb / shards, extra = nb % shards;
            const uint64_t ur = (uint64_t)r;
            const uint64_t b0 = ur * per + (ur < extra ? ur : extra), cnt = per + (ur < extra ? 1 : 0);
            const uint64_t start = b0 * bs < len ? b0 * bs : len;
            const uint64_t end = (b0 + cnt) * bs < len ? (b0 + cnt) * bs : len;
            uint64_t got = 0;
            rc = sf_index_file_range(path, start, end - start, bs, rows + n, nb - n, &got);
            n += got;
        }
    }
    if (rc == SF_OK) {
        for (uint64_t i = 0; i < n; i++) memcpy(dig + 20 * i, rows[i].sha1, 20);
        rc = sf_blocks_hash(dig, n, bh);
    }
    if (rc == SF_OK) print_rows(path, rows, n, bh);
    free(rows);
    free(dig);
    return rc;
}

/* -X N: one file on N devices from this one process (sf_index_file_multi:
 * a host thread per device, shard rows at their row offsets, blocks_hash on
 * the host); the rows and blocks_hash are the one-device route's. */
static int index_multi(const char *path, uint32_t bs, int ndev) {
    struct stat sb;
    if (stat(path, &sb) != 0) return SF_EIO;
    uint64_t cap = sb.st_size ? ((uint64_t)sb.st_size + bs - 1) / bs : 0, n = 0;
    uint8_t bh[20];
    int rc = SF_ENOSPC;
    sf_block_sig *rows = NULL;
    for (int attempt = 0; attempt < 3 && rc == SF_ENOSPC; attempt++) { /* the file may grow meanwhile */
        free(rows);
        rows = malloc((cap ? cap : 1) * sizeof(sf_block_sig));
        if (!rows) return SF_ENOMEM;
        rc = sf_index_file_multi(path, bs, (uint32_t)ndev, rows, cap, &n, bh);
        if (rc == SF_ENOSPC) cap = n;
    }
    if (rc == SF_OK) print_rows(path, rows, n, bh);
    free(rows);
    return rc;
}

/* -C: content-defined blocks from C, the way the reference's default mode
 * drops in (INTEGRATION.md index_file_rows_cdc): a chunker on the host cuts
 * the file's bytes and sf_index_buffer_blocks hashes every block on the
 * device.  The chunker here is a stand-in (the reference's cdchunking ZPAQ
 * is Rust): a block ends after byte i when the little-endian word of bytes
 * i-3..i, times 2654435761 (mod 2^32), is below 2^19 (rate 2^-13, ~8 KiB
 * blocks), or when it reaches 32 KiB (src/index.rs:40-41). */
/* The stand-in chunker: (*offs, *sizes, *n) for buf[0, len), lists grown
 * with realloc (caller frees). */
static int cdc_cut(const uint8_t *buf, uint64_t len, uint64_t **offs_out, uint32_t **sizes_out, uint64_t *n_out) {
    uint64_t n = 0, cap = len / 4096 + 16;
    uint64_t *offs = malloc(cap * sizeof(uint64_t));
    uint32_t *sizes = malloc(cap * sizeof(uint32_t));
    int rc = (offs && sizes) ? SF_OK : SF_ENOMEM;
    for (uint64_t start = 0, i = 0; rc == SF_OK && i < len; i++) {
        const uint32_t w = i >= 3 ? (uint32_t)buf[i - 3] | (uint32_t)buf[i - 2] << 8 | (uint32_t)buf[i - 1] << 16 |
                                        (uint32_t)buf[i] << 24
                                  : 0xFFFFFFFFu;
        if ((uint32_t)(w * 2654435761u) < (1u << 19) || i + 1 - start == 32768 || i + 1 == len) {
            if (n == cap) {  /* the list grows as the chunker finds blocks */
                uint64_t *o2 = realloc(offs, 2 * cap * sizeof(uint64_t));
                if (o2) offs = o2;
                uint32_t *s2 = o2 ? realloc(sizes, 2 * cap * sizeof(uint32_t)) : NULL;
                if (s2) sizes = s2;
                if (!o2 || !s2) { rc = SF_ENOMEM; break; }
                cap *= 2;
            }
            offs[n] = start;
            sizes[n] = (uint32_t)(i + 1 - start);
            n++;
            start = i + 1;
        }
    }
    *offs_out = offs;
    *sizes_out = sizes;
    *n_out = n;
    return rc;
}

static int index_cdc(const char *path) {
    struct stat sb;
    if (stat(path, &sb) != 0 || !S_ISREG(sb.st_mode)) return SF_EIO;
    const uint64_t len = (uint64_t)sb.st_size;
    uint8_t *buf = malloc(len ? len : 1), bh[20];
    uint64_t n = 0, *offs = NULL;
    uint32_t *sizes = NULL;
    sf_block_sig *rows = NULL;
    int rc = buf ? SF_OK : SF_ENOMEM;
    FILE *f = rc == SF_OK ? fopen(path, "rb") : NULL;
    if (rc == SF_OK && (!f || fread(buf, 1, len, f) != len)) rc = SF_EIO;
    if (f) fclose(f);
    if (rc == SF_OK) rc = cdc_cut(buf, len, &offs, &sizes, &n);
    if (rc == SF_OK) rc = (rows = malloc((n ? n : 1) * sizeof(sf_block_sig))) ? SF_OK : SF_ENOMEM;
    if (rc == SF_OK) rc = sf_index_buffer_blocks(buf, len, offs, sizes, n, rows, bh);
    if (rc == SF_OK) {  /* the file form (pread windows) must give the same rows and blocks_hash */
        sf_block_sig *again = malloc((n ? n : 1) * sizeof(sf_block_sig));
        uint8_t bh2[20];
        rc = again ? sf_index_file_blocks(path, offs, sizes, n, again, bh2) : SF_ENOMEM;
        if (rc == SF_OK && (memcmp(bh, bh2, 20) != 0 || (n && memcmp(rows, again, n * sizeof(sf_block_sig)) != 0)))
            rc = SF_EIO;
        free(again);
    }
    if (rc == SF_OK) print_rows(path, rows, n, bh);
    free(buf);
    free(offs);
    free(sizes);
    free(rows);
    return rc;
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* -Z: the drop-in's default splice from C (INTEGRATION.md
 * index_file_rows_cdc): ONE open of the file and its stamp; the chunker
 * streams the open file (64 KiB reads, as Chunker::stream reads it,
 * src/index.rs:625) and only the (offset, size) list is kept; then
 * sf_index_fd_blocks hashes the list from the same descriptor, so a file
 * renamed over the path meanwhile changes nothing and one written in place
 * gives SF_EAGAIN: cut again, at most 3 times.  The chunker is the stand-in
 * of zpaq_standin.h (the crate's per-byte work, not its boundaries).  -T: one
 * line per file on stderr, {"zpaq_file": ..., "bytes", "blocks", "chunk_s",
 * "hash_s"}: the host chunker's time and the hashing call's. */
/* The stand-in chunker as sf_chunker_ops (sf_cut_fd calls it from the
 * library's threads, one chunker per thread). */
static void *zpaq_create(void *ctx) {
    (void)ctx;
    sf_zpaq *z = malloc(sizeof *z);
    if (z) sf_zpaq_init(z, 13, 32768); /* ZPAQ_BITS, MAX_BLOCK_SIZE: src/index.rs:40-41 */
    return z;
}
static size_t zpaq_next(void *ch, const uint8_t *p, size_t n) { return sf_zpaq_next(ch, p, n); }
static void zpaq_destroy(void *ch) { free(ch); }

/* -Z -p N: index_zpaq with the chunker on N threads: sf_index_fd_cut (the
 * file read once, cut by sf_cut_fd's segments and join -- the one-stream
 * boundaries whatever N -- and hashed from the copy already in HBM). */
static int index_zpaq_fused(const char *path, uint32_t threads, int timing) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return SF_EIO;
    const sf_chunker_ops ops = {zpaq_create, zpaq_next, zpaq_destroy, NULL};
    sf_block_sig *rows = NULL;
    uint64_t n = 0;
    uint8_t bh[20];
    int rc = SF_EAGAIN;
    double t = 0;
    for (int attempt = 0; attempt < 3 && rc == SF_EAGAIN; attempt++) { /* a file written meanwhile: again */
        sf_free_rows(rows);
        rows = NULL;
        const double t0 = now_s();
        rc = sf_index_fd_cut(fd, NULL, &ops, threads, &rows, &n, bh);
        t = now_s() - t0;
    }
    close(fd);
    if (rc == SF_OK) {
        print_rows(path, rows, n, bh);
        if (timing) {
            const uint64_t total = n ? rows[n - 1].offset + rows[n - 1].size : 0;
            fprintf(stderr, "{\"zpaq_file\": \"%s\", \"threads\": %u, \"bytes\": %llu, \"blocks\": %llu, "
                            "\"chunk_s\": 0, \"hash_s\": %.6f, \"fused\": 1}\n",
                    path, threads, (unsigned long long)total, (unsigned long long)n, t);
        }
    }
    sf_free_rows(rows);
    return rc;
}

/* -Z -p N -W: the same as two calls -- sf_cut_fd on N threads, then
 * sf_index_fd_blocks hashing the list from the descriptor (a second read). */
static int index_zpaq_parallel(const char *path, uint32_t threads, int timing) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return SF_EIO;
    const sf_chunker_ops ops = {zpaq_create, zpaq_next, zpaq_destroy, NULL};
    uint64_t *offs = NULL, n = 0;
    uint32_t *sizes = NULL;
    sf_block_sig *rows = NULL;
    uint8_t bh[20];
    double t_chunk = 0, t_hash = 0;
    int rc = SF_EAGAIN;
    for (int attempt = 0; attempt < 3 && rc == SF_EAGAIN; attempt++) { /* a file written meanwhile: again */
        sf_file_stamp st;
        if ((rc = sf_file_stamp_fd(fd, &st)) != SF_OK) break;
        sf_free_cuts(offs);
        sf_free_cuts(sizes);
        offs = NULL;
        sizes = NULL;
        const double t0 = now_s();
        rc = sf_cut_fd(fd, &st, &ops, threads, &offs, &sizes, &n);
        t_chunk = now_s() - t0;
        if (rc != SF_OK) continue;
        free(rows);
        if (!(rows = malloc((n ? n : 1) * sizeof(sf_block_sig)))) { rc = SF_ENOMEM; break; }
        const double t1 = now_s();
        rc = sf_index_fd_blocks(fd, &st, offs, sizes, n, rows, bh);
        t_hash = now_s() - t1;
    }
    close(fd);
    if (rc == SF_OK) {
        print_rows(path, rows, n, bh);
        if (timing) {
            uint64_t total = n ? offs[n - 1] + sizes[n - 1] : 0;
            fprintf(stderr, "{\"zpaq_file\": \"%s\", \"threads\": %u, \"bytes\": %llu, \"blocks\": %llu, "
                            "\"chunk_s\": %.6f, \"hash_s\": %.6f}\n",
                    path, threads, (unsigned long long)total, (unsigned long long)n, t_chunk, t_hash);
        }
    }
    sf_free_cuts(offs);
    sf_free_cuts(sizes);
    free(rows);
    return rc;
}

static int index_zpaq(const char *path, int timing) {
    enum { kRead = 1 << 16 };
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return SF_EIO;
    uint8_t *buf = malloc(kRead), bh[20];
    uint64_t n = 0, cap = 1024, total = 0, *offs = malloc(cap * sizeof(uint64_t));
    uint32_t *sizes = malloc(cap * sizeof(uint32_t));
    sf_block_sig *rows = NULL;
    double t_chunk = 0, t_hash = 0;
    int rc = (buf && offs && sizes) ? SF_EAGAIN : SF_ENOMEM;
    for (int attempt = 0; attempt < 3 && rc == SF_EAGAIN; attempt++) {
        sf_file_stamp st;
        if ((rc = sf_file_stamp_fd(fd, &st)) != SF_OK) break;
        if (lseek(fd, 0, SEEK_SET) != 0) { rc = SF_EIO; break; }
        const double t0 = now_s();
        sf_zpaq z;
        sf_zpaq_init(&z, 13, 32768); /* ZPAQ_BITS, MAX_BLOCK_SIZE: src/index.rs:40-41 */
        uint64_t start = 0;
        n = total = 0;
        for (int eof = 0; rc == SF_OK && !eof;) {
            const ssize_t r = read(fd, buf, kRead);
            if (r < 0 && errno == EINTR) continue;
            if (r < 0) { rc = SF_EIO; break; }
            uint64_t p = 0;
            for (;;) { /* boundaries in this read; at EOF the open chunk ends (ChunkInput::End after data) */
                const size_t k = r > 0 ? sf_zpaq_next(&z, buf + p, (size_t)((uint64_t)r - p)) : 0;
                eof = r == 0;
                if (k == 0 && !(eof && total > start)) break;
                const uint64_t end = k ? total + p + k : total;
                if (n == cap) {
                    uint64_t *o2 = realloc(offs, 2 * cap * sizeof(uint64_t));
                    if (o2) offs = o2;
                    uint32_t *s2 = o2 ? realloc(sizes, 2 * cap * sizeof(uint32_t)) : NULL;
                    if (s2) sizes = s2;
                    if (!o2 || !s2) { rc = SF_ENOMEM; break; }
                    cap *= 2;
                }
                offs[n] = start;
                sizes[n++] = (uint32_t)(end - start);
                start = end;
                if (!k) break;
                p += k;
            }
            total += r > 0 ? (uint64_t)r : 0;
        }
        t_chunk = now_s() - t0;
        if (rc != SF_OK) break;
        free(rows);
        if (!(rows = malloc((n ? n : 1) * sizeof(sf_block_sig)))) { rc = SF_ENOMEM; break; }
        const double t1 = now_s();
        rc = sf_index_fd_blocks(fd, &st, offs, sizes, n, rows, bh);
        t_hash = now_s() - t1;
    }
    close(fd);
    if (rc == SF_OK) {
        print_rows(path, rows, n, bh);
        if (timing)
            fprintf(stderr, "{\"zpaq_file\": \"%s\", \"bytes\": %llu, \"blocks\": %llu, \"chunk_s\": %.6f, \"hash_s\": %.6f}\n",
                    path, (unsigned long long)total, (unsigned long long)n, t_chunk, t_hash);
    }
    free(buf);
    free(offs);
    free(sizes);
    free(rows);
    return rc;
}

/* The stand-in chunker over an open file from its start (64 KiB reads, as
 * index_zpaq): the (offset, size) list, grown with realloc; *total = bytes
 * read.  SF_OK or SF_EIO / SF_ENOMEM. */
static int zpaq_cut_fd(int fd, uint8_t *buf, size_t bufsz, uint64_t **offs_io, uint32_t **sizes_io, uint64_t *cap_io,
                       uint64_t *n_out, uint64_t *total_out, double *read_s) {
    uint64_t *offs = *offs_io, cap = *cap_io, n = 0, total = 0, start = 0;
    uint32_t *sizes = *sizes_io;
    int rc = SF_OK;
    sf_zpaq z;
    sf_zpaq_init(&z, 13, 32768); /* ZPAQ_BITS, MAX_BLOCK_SIZE: src/index.rs:40-41 */
    for (int eof = 0; rc == SF_OK && !eof;) {
        const double t0 = now_s();
        const ssize_t r = pread(fd, buf, bufsz, (off_t)total);
        *read_s += now_s() - t0;
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) { rc = SF_EIO; break; }
        uint64_t p = 0;
        for (;;) {
            const size_t k = r > 0 ? sf_zpaq_next(&z, buf + p, (size_t)((uint64_t)r - p)) : 0;
            eof = r == 0;
            if (k == 0 && !(eof && total > start)) break;
            const uint64_t end = k ? total + p + k : total;
            if (n == cap) {
                const uint64_t c2 = cap ? 2 * cap : 1024;
                uint64_t *o2 = realloc(offs, c2 * sizeof(uint64_t));
                if (o2) offs = o2;
                uint32_t *s2 = o2 ? realloc(sizes, c2 * sizeof(uint32_t)) : NULL;
                if (s2) sizes = s2;
                if (!o2 || !s2) { rc = SF_ENOMEM; break; }
                cap = c2;
            }
            offs[n] = start;
            sizes[n++] = (uint32_t)(end - start);
            start = end;
            if (!k) break;
            p += k;
        }
        total += r > 0 ? (uint64_t)r : 0;
    }
    *offs_io = offs;
    *sizes_io = sizes;
    *cap_io = cap;
    *n_out = n;
    *total_out = total;
    return rc;
}

/* -Z -M: index_path's default mode from C.  Files are stat'ed and dealt into
 * batches of about batch_bytes; `threads` chunker threads take the files in
 * order (opening each once, stamping it, cutting it over the open descriptor)
 * but never more than one batch ahead of the hashing; the main thread hashes
 * each batch with ONE sf_index_fds_blocks on those descriptors as soon as all
 * its files are cut.  A file the call reports SF_EAGAIN for (written
 * meanwhile) is cut and hashed again alone through index_zpaq's retry loop.
 * -T: one JSON line on stderr with the wall time and its parts. */
typedef struct {
    const char *path;
    int fd, rc, large; /* large: opened and stamped only, cut + hashed by sf_index_fd_cut */
    sf_file_stamp st;
    uint64_t *offs, cap, n, bytes;
    uint32_t *sizes;
} cut_job;

typedef struct {
    cut_job *jobs;
    int n, threads;
    const int *batch_of;     /* file -> batch */
    int *batch_left;         /* files of each batch still being cut */
    int next, hashed;        /* next file to cut; the last batch hashed */
    double chunk_s, open_s, read_s; /* summed over threads: cutting (all of it), its open + stamp, its reads */
    pthread_mutex_t mu;
    pthread_cond_t cv;
} cut_pool;

static void *cut_worker(void *arg) {
    cut_pool *P = arg;
    enum { kRead = 1 << 16 };
    uint8_t *buf = malloc(kRead);
    for (;;) {
        pthread_mutex_lock(&P->mu);
        /* at most one batch ahead of the one being hashed (hashed + 1) */
        while (P->next < P->n && P->batch_of[P->next] > P->hashed + 2) pthread_cond_wait(&P->cv, &P->mu);
        const int k = P->next < P->n ? P->next++ : -1;
        pthread_mutex_unlock(&P->mu);
        if (k < 0) break;
        cut_job *j = &P->jobs[k];
        const double t0 = now_s();
        j->fd = open(j->path, O_RDONLY);
        j->rc = j->fd < 0 ? SF_EIO : !buf ? SF_ENOMEM : sf_file_stamp_fd(j->fd, &j->st);
        const double t1 = now_s();
        double rd = 0;
        if (j->rc == SF_OK && !j->large)
            j->rc = zpaq_cut_fd(j->fd, buf, kRead, &j->offs, &j->sizes, &j->cap, &j->n, &j->bytes, &rd);
        if (j->rc == SF_OK && !j->large && j->bytes != j->st.size) j->rc = SF_EAGAIN;  /* written while cut */
        const double dt = now_s() - t0;
        pthread_mutex_lock(&P->mu);
        P->chunk_s += dt;
        P->open_s += t1 - t0;
        P->read_s += rd;
        P->batch_left[P->batch_of[k]]--;
        pthread_cond_broadcast(&P->cv);
        pthread_mutex_unlock(&P->mu);
    }
    free(buf);
    return NULL;
}

typedef struct {
    char **paths;
    uint64_t *sizes;
    int n, next;
} stat_pool;

static void *stat_worker(void *arg) { /* the sizes for the batch plan, 64 files per take */
    stat_pool *S = arg;
    for (int k0; (k0 = __atomic_fetch_add(&S->next, 64, __ATOMIC_RELAXED)) < S->n;)
        for (int k = k0; k < S->n && k < k0 + 64; k++) {
            struct stat sb;
            S->sizes[k] = stat(S->paths[k], &sb) == 0 ? (uint64_t)sb.st_size : 0;
        }
    return NULL;
}

/* A large file of -Z -M, alone in its batch: cut on `threads` threads and
 * hashed from one read of the walk's open descriptor (sf_index_fd_cut), with
 * the stamp taken at that open; SF_EAGAIN (written meanwhile): again, alone,
 * from a new open (index_zpaq_fused's retries). */
static int index_zpaq_large(cut_job *j, int threads, int quiet, int edge, uint64_t *blocks, double *hash_s) {
    const sf_chunker_ops ops = {zpaq_create, zpaq_next, zpaq_destroy, NULL};
    sf_block_sig *rows = NULL;
    uint64_t n = 0;
    uint8_t bh[20];
    const double t0 = now_s();
    int rc = sf_index_fd_cut(j->fd, &j->st, &ops, (uint32_t)threads, &rows, &n, bh);
    *hash_s += now_s() - t0;
    if (rc == SF_EAGAIN) {
        close(j->fd);
        j->fd = -1;
        return index_zpaq_fused(j->path, (uint32_t)threads, 0);
    }
    if (rc == SF_OK) {
        j->bytes = j->st.size;
        *blocks += n;
        if (quiet == 2) { /* an untimed warm-up pass: no output */
        } else if (!quiet || edge) print_rows(j->path, rows, n, bh);
        else {
            char h[41];
            hex(bh, h);
            printf("file %s blocks %llu\nblocks_hash %s\n", j->path, (unsigned long long)n, h);
        }
    }
    sf_free_rows(rows);
    return rc;
}

static int index_zpaq_many(char **paths, int n, int threads, uint64_t batch_bytes, uint64_t stage_bytes, int timing,
                           int quiet, uint64_t large_bytes) {
    cut_job *jobs = calloc((size_t)(n ? n : 1), sizeof(cut_job));
    int *batch_of = malloc((size_t)(n ? n : 1) * sizeof(int)), nb = 0;
    int *batch_left = calloc((size_t)(n ? n : 1), sizeof(int)), *batch_first = calloc((size_t)n + 2, sizeof(int));
    if (!jobs || !batch_of || !batch_left || !batch_first) return SF_ENOMEM;
    const double t_start = now_s();
    uint64_t acc = 0, total_bytes = 0, total_blocks = 0;
    /* three batches' descriptors may be open at once (one hashed, one cut,
     * one waiting): a batch holds at most a quarter of the descriptor limit */
    struct rlimit rl;
    int max_files = 4096;
    if (getrlimit(RLIMIT_NOFILE, &rl) == 0 && rl.rlim_cur != RLIM_INFINITY && (int)(rl.rlim_cur / 4) < max_files)
        max_files = rl.rlim_cur / 4 > 16 ? (int)(rl.rlim_cur / 4) : 16;
    /* the files' sizes, stat'ed on the chunker threads (a stat can cost
     * ~100 us on some hosts: 10,000 files would be a second on one thread) */
    uint64_t *fsize = calloc((size_t)(n ? n : 1), sizeof(uint64_t));
    if (!fsize) return SF_ENOMEM;
    {
        stat_pool S = {paths, fsize, n, 0};
        pthread_t st[64];
        int ns = 0;
        for (int t = 1; t < threads && t < 64 && t * 256 < n; t++)
            if (pthread_create(&st[ns], NULL, stat_worker, &S) == 0) ns++;
        stat_worker(&S);
        for (int t = 0; t < ns; t++) pthread_join(st[t], NULL);
    }
    for (int k = 0; k < n; k++) { /* batches by size and descriptor count; a large file alone */
        jobs[k].path = paths[k];
        jobs[k].fd = -1;
        jobs[k].large = large_bytes && fsize[k] >= large_bytes;
        if (k == 0 || acc >= batch_bytes || k - batch_first[nb - 1] >= max_files || jobs[k].large ||
            jobs[k - 1].large) {
            batch_first[nb++] = k;
            acc = 0;
        }
        batch_of[k] = nb - 1;
        batch_left[nb - 1]++;
        acc += fsize[k];
    }
    batch_first[nb] = n;
    free(fsize);
    cut_pool P = {jobs, n, threads, batch_of, batch_left, 0, -1, 0.0, 0.0, 0.0, PTHREAD_MUTEX_INITIALIZER,
                  PTHREAD_COND_INITIALIZER};
    pthread_t *th = malloc((size_t)(threads > 0 ? threads : 1) * sizeof(pthread_t));
    int started = 0, rc = th ? SF_OK : SF_ENOMEM;
    for (int t = 0; rc == SF_OK && t < threads; t++)
        if (pthread_create(&th[t], NULL, cut_worker, &P) == 0) started++;
    if (started == 0) rc = SF_ENOMEM;
    double t_wait = 0, t_hash = 0;
    for (int b = 0; rc == SF_OK && b < nb; b++) {
        const int f0 = batch_first[b], m = batch_first[b + 1] - f0;
        const double tw = now_s();
        pthread_mutex_lock(&P.mu);
        while (batch_left[b] > 0) pthread_cond_wait(&P.cv, &P.mu);
        pthread_mutex_unlock(&P.mu);
        t_wait += now_s() - tw;
        if (m == 1 && jobs[f0].large) { /* the large file, in its place */
            cut_job *j = &jobs[f0];
            rc = j->rc != SF_OK ? j->rc : index_zpaq_large(j, threads, quiet, f0 == 0 || f0 == n - 1, &total_blocks,
                                                                  &t_hash);
            if (rc == SF_EAGAIN) { /* written between its open and its stamp check: once more, alone */
                if (j->fd >= 0) close(j->fd);
                j->fd = -1;
                rc = index_zpaq_fused(j->path, (uint32_t)threads, 0);
            }
            if (j->fd >= 0) close(j->fd);
            j->fd = -1;
            total_bytes += rc == SF_OK ? j->bytes : 0;
            pthread_mutex_lock(&P.mu);
            P.hashed = b;
            pthread_cond_broadcast(&P.cv);
            pthread_mutex_unlock(&P.mu);
            continue;
        }
        int *fds = malloc((size_t)m * sizeof(int)), *fst = malloc((size_t)m * sizeof(int));
        sf_file_stamp *sts = malloc((size_t)m * sizeof(sf_file_stamp));
        const uint64_t **po = malloc((size_t)m * sizeof(void *));
        const uint32_t **pz = malloc((size_t)m * sizeof(void *));
        uint64_t *cnt = malloc((size_t)m * sizeof(uint64_t)), *first = malloc(((size_t)m + 1) * sizeof(uint64_t));
        uint8_t *hashes = malloc((size_t)m * 20);
        uint64_t rows_n = 0;
        for (int k = 0; k < m; k++) rows_n += jobs[f0 + k].rc == SF_OK ? jobs[f0 + k].n : 0;
        sf_block_sig *rows = malloc((rows_n ? rows_n : 1) * sizeof(sf_block_sig));
        if (!fds || !fst || !sts || !po || !pz || !cnt || !first || !hashes || !rows) rc = SF_ENOMEM;
        for (int k = 0; rc == SF_OK && k < m; k++) {
            const cut_job *j = &jobs[f0 + k];
            if (j->rc != SF_OK && j->rc != SF_EAGAIN) { rc = j->rc; break; }
            fds[k] = j->rc == SF_OK ? j->fd : -1; /* a file written while cut: indexed again below */
            sts[k] = j->st;
            po[k] = j->offs;
            pz[k] = j->sizes;
            cnt[k] = j->rc == SF_OK ? j->n : 0;
        }
        uint32_t bad = 0;
        if (rc == SF_OK) {
            const double th0 = now_s();
            const int r = sf_index_fds_blocks(fds, sts, (uint32_t)m, po, pz, cnt, stage_bytes, rows, rows_n, first,
                                              hashes, fst, &bad);
            t_hash += now_s() - th0;
            if (r != SF_OK && !(r == fst[bad])) rc = r; /* a per-file failure is handled per file */
        }
        for (int k = 0; rc == SF_OK && k < m; k++) {
            cut_job *j = &jobs[f0 + k];
            if (j->rc == SF_EAGAIN || fst[k] == SF_EAGAIN) { /* written meanwhile: once more, alone */
                close(j->fd);
                j->fd = -1;
                if ((rc = index_zpaq(j->path, 0)) != SF_OK) break;
                continue;
            }
            if (fst[k] != SF_OK) { rc = fst[k]; break; }
            total_bytes += j->bytes;
            total_blocks += cnt[k];
            const int show = !quiet || f0 + k == 0 || f0 + k == n - 1;
            if (quiet == 2) { /* an untimed warm-up pass: no output */
            } else if (show) print_rows(j->path, rows + first[k], cnt[k], hashes + 20 * k);
            else {
                char h[41];
                hex(hashes + 20 * k, h);
                printf("file %s blocks %llu\nblocks_hash %s\n", j->path, (unsigned long long)cnt[k], h);
            }
        }
        for (int k = 0; k < m; k++) {
            cut_job *j = &jobs[f0 + k];
            if (j->fd >= 0) close(j->fd);
            j->fd = -1;
            free(j->offs);
            free(j->sizes);
            j->offs = NULL;
            j->sizes = NULL;
        }
        free(fds); free(fst); free(sts); free(po); free(pz); free(cnt); free(first); free(hashes); free(rows);
        pthread_mutex_lock(&P.mu);
        P.hashed = b;
        pthread_cond_broadcast(&P.cv);
        pthread_mutex_unlock(&P.mu);
    }
    pthread_mutex_lock(&P.mu);
    P.hashed = nb; /* on an error: release the workers */
    P.next = rc == SF_OK ? P.next : n;
    pthread_cond_broadcast(&P.cv);
    pthread_mutex_unlock(&P.mu);
    for (int t = 0; t < started; t++) pthread_join(th[t], NULL);
    for (int k = 0; k < n; k++) {
        if (jobs[k].fd >= 0) close(jobs[k].fd);
        free(jobs[k].offs);
        free(jobs[k].sizes);
    }
    const double wall = now_s() - t_start;
    if (timing && rc == SF_OK)
        fprintf(stderr,
                "{\"zpaq_many\": %d, \"threads\": %d, \"batches\": %d, \"bytes\": %llu, \"blocks\": %llu, "
                "\"wall_s\": %.6f, \"chunk_cpu_s\": %.6f, \"open_s\": %.6f, \"read_s\": %.6f, \"hash_call_s\": %.6f, "
                "\"wait_cut_s\": %.6f}\n",
                n, threads, nb, (unsigned long long)total_bytes, (unsigned long long)total_blocks, wall, P.chunk_s,
                P.open_s, P.read_s, t_hash, t_wait);
    free(th); free(jobs); free(batch_of); free(batch_left); free(batch_first);
    return rc;
}

/* -v N: the default mode's wire run from C: N synthetic bytes generated in
 * HBM, cut on the host by the stand-in chunker, hashed on the device as an
 * explicit list (sf_index_device_blocks), and the list's FILE_BLOCK run --
 * every block with its own size -- streamed to stdout (sf_wire_blocks_fd). */
static int wire_synthetic_cdc(uint64_t len) {
    void *d_data = NULL, *d_dig = NULL, *d_offs = NULL, *d_sizes = NULL;
    uint8_t *buf = malloc(len ? len : 1);
    uint64_t n = 0, *offs = NULL, written = 0;
    uint32_t *sizes = NULL;
    int rc = (buf && hipMalloc(&d_data, len ? len : 1) == hipSuccess) ? SF_OK : SF_ENOMEM;
    if (rc == SF_OK) rc = sf_fill_splitmix_device(d_data, len, 0x5EED0000ull, 0, NULL);
    if (rc == SF_OK && len && hipMemcpy(buf, d_data, len, hipMemcpyDeviceToHost) != hipSuccess) rc = SF_ENODEV;
    if (rc == SF_OK) rc = cdc_cut(buf, len, &offs, &sizes, &n);
    if (rc == SF_OK && (hipMalloc(&d_dig, n ? n * 20 : 20) != hipSuccess ||
                        hipMalloc(&d_offs, n ? n * 8 : 8) != hipSuccess || hipMalloc(&d_sizes, n ? n * 4 : 4) != hipSuccess))
        rc = SF_ENOMEM;
    if (rc == SF_OK && n &&
        (hipMemcpy(d_offs, offs, n * 8, hipMemcpyHostToDevice) != hipSuccess ||
         hipMemcpy(d_sizes, sizes, n * 4, hipMemcpyHostToDevice) != hipSuccess))
        rc = SF_ENODEV;
    if (rc == SF_OK) rc = sf_index_device_blocks(d_data, len, d_offs, d_sizes, n, d_dig, NULL, NULL);
    if (rc == SF_OK) rc = sf_wire_blocks_fd(d_dig, d_sizes, n, 1, &written, NULL);
    if (rc == SF_OK && n && written == 0) rc = SF_EIO;
    if (d_data) (void)hipFree(d_data);
    if (d_dig) (void)hipFree(d_dig);
    if (d_offs) (void)hipFree(d_offs);
    if (d_sizes) (void)hipFree(d_sizes);
    free(buf);
    free(offs);
    free(sizes);
    return rc;
}

/* -w N: the device-resident path and the wire stream from C: N bytes of the
 * splitmix64 stream (seed 0x5EED0000) generated in HBM
 * (sf_fill_splitmix_device), hashed there (sf_index_device_fixed), and the
 * file's FILE_BLOCK run (src/sync/ssh/proto.rs:162-166) streamed to stdout
 * (sf_wire_file_blocks_fd). */
static int wire_synthetic(uint64_t n, uint32_t bs) {
    const uint64_t nb = n ? (n + bs - 1) / bs : 0;
    void *d_data = NULL, *d_dig = NULL;
    uint64_t got = 0, written = 0;
    int rc = (hipMalloc(&d_data, n ? n : 1) == hipSuccess && hipMalloc(&d_dig, nb ? nb * 20 : 20) == hipSuccess)
                 ? SF_OK : SF_ENOMEM;
    if (rc == SF_OK) rc = sf_fill_splitmix_device(d_data, n, 0x5EED0000ull, 0, NULL);
    if (rc == SF_OK) rc = sf_index_device_fixed(d_data, n, bs, d_dig, nb, &got, NULL);
    if (rc == SF_OK) rc = sf_wire_file_blocks_fd(d_dig, nb, bs, n, 1, &written, NULL);
    if (rc == SF_OK && written == 0 && nb) rc = SF_EIO;
    if (d_data) (void)hipFree(d_data);
    if (d_dig) (void)hipFree(d_dig);
    return rc;
}

/* -L: the receiving side's lookup from C.  dst's rows are the destination's
 * index (digests in row order, all present); src's rows are the FILE_BLOCK
 * run it receives.  Each src block is looked up in a device block set built
 * from dst's digests (sf_block_set_*), as FsDestinationInner::sink asks
 * Index::get_block per block (src/sync/fs.rs:461-476): "i row" per src block,
 * row = dst row holding that digest first, or -1. */
static int lookup_blocks(const char *dst, const char *src, uint32_t bs) {
    sf_block_sig *rows[2] = {NULL, NULL};
    uint64_t n[2] = {0, 0};
    const char *paths[2] = {dst, src};
    uint8_t bh[20];
    int rc = SF_OK;
    for (int k = 0; k < 2 && rc == SF_OK; k++) {
        struct stat sb;
        if (stat(paths[k], &sb) != 0 || !S_ISREG(sb.st_mode)) { rc = SF_EIO; break; }
        const uint64_t cap = sb.st_size ? ((uint64_t)sb.st_size + bs - 1) / bs : 0;
        rows[k] = malloc((cap ? cap : 1) * sizeof(sf_block_sig));
        rc = rows[k] ? sf_index_file(paths[k], bs, rows[k], cap, &n[k], bh) : SF_ENOMEM;
    }
    uint8_t *h_dig[2] = {NULL, NULL};
    void *d_dig[2] = {NULL, NULL};
    int64_t *h_rows = NULL, *d_rows = NULL;
    sf_block_set *set = NULL;
    for (int k = 0; k < 2 && rc == SF_OK; k++) {  /* digests, 20 B apart, to the device */
        h_dig[k] = malloc(n[k] ? n[k] * 20 : 20);
        if (!h_dig[k]) { rc = SF_ENOMEM; break; }
        for (uint64_t i = 0; i < n[k]; i++) memcpy(h_dig[k] + 20 * i, rows[k][i].sha1, 20);
        if (hipMalloc(&d_dig[k], n[k] ? n[k] * 20 : 20) != hipSuccess ||
            hipMemcpy(d_dig[k], h_dig[k], n[k] * 20, hipMemcpyHostToDevice) != hipSuccess)
            rc = SF_ENOMEM;
    }
    if (rc == SF_OK) {
        h_rows = malloc((n[1] ? n[1] : 1) * sizeof(int64_t));
        rc = (h_rows && hipMalloc((void **)&d_rows, (n[1] ? n[1] : 1) * sizeof(int64_t)) == hipSuccess) ? SF_OK
                                                                                                       : SF_ENOMEM;
    }
    if (rc == SF_OK) rc = sf_block_set_build(d_dig[0], NULL, n[0], &set, NULL);
    if (rc == SF_OK) rc = sf_block_set_lookup(set, d_dig[1], n[1], d_rows, NULL);
    if (rc == SF_OK && hipMemcpy(h_rows, d_rows, n[1] * sizeof(int64_t), hipMemcpyDeviceToHost) != hipSuccess)
        rc = SF_ENODEV;
    if (rc == SF_OK)
        for (uint64_t i = 0; i < n[1]; i++) printf("%llu %lld\n", (unsigned long long)i, (long long)h_rows[i]);
    if (set) sf_block_set_free(set, NULL);
    (void)hipDeviceSynchronize();
    for (int k = 0; k < 2; k++) {
        if (d_dig[k]) (void)hipFree(d_dig[k]);
        free(h_dig[k]);
        free(rows[k]);
    }
    if (d_rows) (void)hipFree(d_rows);
    free(h_rows);
    return rc;
}

/* -m: every path through ONE sf_index_files call (index_path's pipeline,
 * src/index.rs:685-715), rows sized by a first call with cap 0. */
static int index_many(char **paths, int n, uint32_t bs) {
    uint64_t *first = malloc((n + 1) * sizeof(uint64_t)), need = 0;
    uint8_t *hashes = malloc((size_t)n * 20);
    uint32_t bad = 0;
    if (!first || !hashes) return SF_ENOMEM;
    int rc = sf_index_files((const char *const *)paths, (uint32_t)n, bs, 0, NULL, 0, first, hashes, &need, &bad);
    sf_block_sig *rows = NULL;
    if (rc == SF_ENOSPC || rc == SF_OK) {
        rows = malloc((need ? need : 1) * sizeof(sf_block_sig));
        rc = rows ? sf_index_files((const char *const *)paths, (uint32_t)n, bs, 0, rows, need, first, hashes, &need,
                                   &bad)
                  : SF_ENOMEM;
    }
    if (rc == SF_OK)
        for (int k = 0; k < n; k++) print_rows(paths[k], rows + first[k], first[k + 1] - first[k], hashes + 20 * k);
    else if (rc == SF_EIO)
        fprintf(stderr, "%s: %s\n", paths[bad], sf_strerror(rc));
    free(rows);
    free(first);
    free(hashes);
    return rc;
}

int main(int argc, char **argv) {
    uint32_t bs = 4096;
    int many = 0, buffer = 0, shards = 0, lookup = 0, cdc = 0, zpaq = 0, timing = 0, threads = 1, quiet = 0;
    int passes = 1, multi = -1, cut_threads = -1, two_calls = 0;
    uint64_t batch_mib = 256, stage_mib = 0, large_mib = 64;
    long long wire = -1, wire_cdc = -1;
    int i = 1;
    for (; i < argc; i++) {
        if (i + 1 < argc && strcmp(argv[i], "-b") == 0) bs = (uint32_t)strtoul(argv[++i], NULL, 10);
        else if (i + 1 < argc && strcmp(argv[i], "-s") == 0) shards = atoi(argv[++i]);
        else if (i + 1 < argc && strcmp(argv[i], "-w") == 0) wire = atoll(argv[++i]);
        else if (i + 1 < argc && strcmp(argv[i], "-v") == 0) wire_cdc = atoll(argv[++i]);
        else if (i + 1 < argc && strcmp(argv[i], "-j") == 0) threads = atoi(argv[++i]);
        else if (i + 1 < argc && strcmp(argv[i], "-X") == 0) multi = atoi(argv[++i]);
        else if (i + 1 < argc && strcmp(argv[i], "-p") == 0) cut_threads = atoi(argv[++i]);
        else if (strcmp(argv[i], "-W") == 0) two_calls = 1;
        else if (i + 1 < argc && strcmp(argv[i], "-S") == 0) batch_mib = strtoull(argv[++i], NULL, 10);
        else if (i + 1 < argc && strcmp(argv[i], "-G") == 0) stage_mib = strtoull(argv[++i], NULL, 10);
        else if (i + 1 < argc && strcmp(argv[i], "-K") == 0) large_mib = strtoull(argv[++i], NULL, 10);
        else if (strcmp(argv[i], "-M") == 0) many = 2;
        else if (strcmp(argv[i], "-q") == 0) quiet = 1;
        else if (i + 1 < argc && strcmp(argv[i], "-P") == 0) passes = atoi(argv[++i]);
        else if (strcmp(argv[i], "-m") == 0) many = 1;
        else if (strcmp(argv[i], "-L") == 0) lookup = 1;
        else if (strcmp(argv[i], "-B") == 0) buffer = 1;
        else if (strcmp(argv[i], "-C") == 0) cdc = 1;
        else if (strcmp(argv[i], "-Z") == 0) zpaq = 1;
        else if (strcmp(argv[i], "-T") == 0) timing = 1;
        else break;
    }
    if (i >= argc && wire < 0 && wire_cdc < 0) {
        fprintf(stderr, "usage: %s [-b block_size] [-m | -B | -C | -Z [-T] [-p cut_threads [-W]] [-M [-j threads] [-S batch_mib] [-G stage_mib] [-K large_mib] [-q] [-P passes]] | -s shards | -X devices] "
                        "path... | -w bytes | -v bytes | -L dst src\n",
                argv[0]);
        return 2;
    }
    int ndev = 0;
    sf_device_count(&ndev);
    if (ndev == 0) {
        fprintf(stderr, "%s: no HIP device (syncfast_amd has no CPU path)\n", argv[0]);
        return 1;
    }
    if (wire_cdc >= 0) {
        const int rc = wire_synthetic_cdc((uint64_t)wire_cdc);
        if (rc != SF_OK) fprintf(stderr, "wire: %s\n", sf_strerror(rc));
        sf_release_host_cache();
        return rc != SF_OK;
    }
    if (wire >= 0) {
        const int rc = wire_synthetic((uint64_t)wire, bs);
        if (rc != SF_OK) fprintf(stderr, "wire: %s\n", sf_strerror(rc));
        sf_release_host_cache();
        return rc != SF_OK;
    }
    int status = 0;
    if (lookup) {
        const int rc = i + 2 == argc ? lookup_blocks(argv[i], argv[i + 1], bs) : SF_EINVAL;
        if (rc != SF_OK) fprintf(stderr, "lookup: %s\n", sf_strerror(rc));
        sf_release_host_cache();
        return rc != SF_OK;
    }
    if (many == 2 && zpaq) {
        /* -P n: the whole pipeline n times in this process (the first pass
         * pays the library's stage allocations and first launches) */
        int rc = SF_OK;
        for (int pass = 0; pass < passes && rc == SF_OK; pass++)
            rc = index_zpaq_many(argv + i, argc - i, threads > 0 ? threads : 1, batch_mib << 20, stage_mib << 20, timing,
                                 pass + 1 < passes ? 2 : quiet, large_mib << 20);
        if (rc != SF_OK) fprintf(stderr, "zpaq many: %s\n", sf_strerror(rc));
        sf_release_host_cache();
        return rc != SF_OK;
    }
    if (many) {
        status = index_many(argv + i, argc - i, bs) != SF_OK;
        sf_release_host_cache();
        return status;
    }
    for (; i < argc; i++) {
        const int rc = multi >= 0 ? index_multi(argv[i], bs, multi)
                       : (zpaq && cut_threads >= 0 && two_calls) ? index_zpaq_parallel(argv[i], (uint32_t)cut_threads, timing)
                       : (zpaq && cut_threads >= 0) ? index_zpaq_fused(argv[i], (uint32_t)cut_threads, timing)
                       : zpaq  ? index_zpaq(argv[i], timing)
                       : cdc ? index_cdc(argv[i])
                       : (buffer || shards > 0) ? index_buffer_or_shards(argv[i], bs, buffer ? 0 : shards)
                                                : index_one(argv[i], bs);
        if (rc != SF_OK) {
            fprintf(stderr, "%s: %s\n", argv[i], sf_strerror(rc));
            status = 1;
        }
    }
    sf_release_host_cache();
    return status;
}
