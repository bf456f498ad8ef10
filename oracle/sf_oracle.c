/*
 * sf_oracle.c -- CPU restatement of syncfast's block-signature indexing path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product path in syncfast_amd/csrc/.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never links it
 * and never falls back to it.
 *
 * What it restates (reference @ v0.2.0, /root/reference):
 *   - SHA-1 per block: crate `sha1 0.6.0` (Cargo.lock:450-453), called as
 *     Sha1::new / update / digest().bytes() / reset at src/index.rs:628-644.
 *     Restated from FIPS 180-4 (standard SHA-1); pinned by the reference's
 *     own KATs src/lib.rs:184-195 (SHA1("test")) and src/index.rs:765-792
 *     (three block digests + blocks_hash), see tests/golden/.
 *   - The index_file loop, src/index.rs:621-647: every block gets
 *     (offset, size, SHA-1(bytes)), blocks in offset order, no empty blocks.
 *     Boundaries come from a fixed tiling (block_size) or an explicit list;
 *     the reference's own CDC boundaries (cdchunking 0.2.1 ZPAQ) are NOT
 *     restated here -- their recurrence is unpinned.
 *   - compute_blocks_hash, src/index.rs:661-682: SHA-1 over the
 *     concatenation of the raw 20-byte block digests in offset order.
 *   - Digest byte order: HashDigest(sha1.digest().bytes()), src/lib.rs:72-76,
 *     i.e. standard big-endian SHA-1 output.
 *   - The synthetic input generator used by bench.py and the tests
 *     (splitmix64 bytes) so CPU and GPU agree on inputs.
 *
 * Parity status: SHA-1 / blocks_hash pinned (reference KATs + hashlib
 * vectors); CDC boundaries unpinned.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

/* ---------------------------------------------------------------- SHA-1 */

typedef struct {
    uint32_t h[5];
    uint64_t total;       /* bytes fed so far */
    uint8_t buf[64];
    size_t nbuf;
} sfo_sha1_ctx;

static inline uint32_t rol32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void sfo_compress(uint32_t h[5], const uint8_t p[64]) {
    uint32_t w[80];
    for (int t = 0; t < 16; t++)
        w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) |
               ((uint32_t)p[4 * t + 2] << 8) | (uint32_t)p[4 * t + 3];
    for (int t = 16; t < 80; t++)
        w[t] = rol32(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int t = 0; t < 80; t++) {
        uint32_t f, k;
        if (t < 20) { f = (b & c) | (~b & d); k = 0x5A827999u; }
        else if (t < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
        else if (t < 60) { f = (b & c) | (b & d) | (c & d); k = 0x8F1BBCDCu; }
        else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
        uint32_t tmp = rol32(a, 5) + f + e + k + w[t];
        e = d; d = c; c = rol32(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
}

/* Sha1::new()  (src/index.rs:628) */
static void sfo_init(sfo_sha1_ctx *c) {
    c->h[0] = 0x67452301u; c->h[1] = 0xEFCDAB89u; c->h[2] = 0x98BADCFEu;
    c->h[3] = 0x10325476u; c->h[4] = 0xC3D2E1F0u;
    c->total = 0; c->nbuf = 0;
}

/* Sha1::update(d)  (src/index.rs:632) */
static void sfo_update(sfo_sha1_ctx *c, const uint8_t *d, size_t n) {
    c->total += n;
    if (c->nbuf) {
        size_t take = 64 - c->nbuf;
        if (take > n) take = n;
        memcpy(c->buf + c->nbuf, d, take);
        c->nbuf += take; d += take; n -= take;
        if (c->nbuf == 64) { sfo_compress(c->h, c->buf); c->nbuf = 0; }
    }
    while (n >= 64) { sfo_compress(c->h, d); d += 64; n -= 64; }
    if (n) { memcpy(c->buf, d, n); c->nbuf = n; }
}

/* sha1.digest().bytes()  (src/index.rs:636) -- big-endian output bytes */
static void sfo_final(sfo_sha1_ctx *c, uint8_t out[20]) {
    uint64_t bits = c->total * 8u;
    uint8_t pad[72];
    size_t padlen = (c->nbuf < 56) ? (56 - c->nbuf) : (120 - c->nbuf);
    memset(pad, 0, sizeof pad);
    pad[0] = 0x80;
    uint64_t keep = c->total;
    sfo_update(c, pad, padlen);
    uint8_t lenb[8];
    for (int i = 0; i < 8; i++) lenb[i] = (uint8_t)(bits >> (56 - 8 * i));
    sfo_update(c, lenb, 8);
    c->total = keep;
    for (int i = 0; i < 5; i++) {
        out[4 * i] = (uint8_t)(c->h[i] >> 24); out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->h[i] >> 8); out[4 * i + 3] = (uint8_t)c->h[i];
    }
}

void sfo_sha1(const uint8_t *data, uint64_t len, uint8_t out[20]) {
    sfo_sha1_ctx c;
    sfo_init(&c);
    sfo_update(&c, data, (size_t)len);
    sfo_final(&c, out);
}

/* ------------------------------------------------ index_file block loop */

/* Number of blocks of a fixed tiling: ceil(len / block_size), 0 for len 0.
 * (No trailing empty block when len % block_size == 0.) */
uint64_t sfo_num_blocks(uint64_t len, uint64_t block_size) {
    if (block_size == 0) return 0;
    return (len + block_size - 1) / block_size;
}

/* Restates src/index.rs:621-647 over a fixed tiling: for each block emit
 * (offset, size, SHA-1).  digests is nblocks*20 bytes, offsets/sizes may be
 * NULL.  Returns the block count. */
uint64_t sfo_index_fixed(const uint8_t *data, uint64_t len, uint64_t block_size,
                         uint64_t *offsets, uint32_t *sizes, uint8_t *digests) {
    uint64_t n = sfo_num_blocks(len, block_size);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t off = i * block_size;
        uint64_t sz = len - off < block_size ? len - off : block_size;
        if (offsets) offsets[i] = off;
        if (sizes) sizes[i] = (uint32_t)sz;
        sfo_sha1(data + off, sz, digests + 20 * i);
    }
    return n;
}

/* Same loop over an explicit boundary list (CDC output, KAT boundaries,
 * many-file batches).  Block i covers data[offsets[i], offsets[i]+sizes[i]). */
void sfo_index_blocks(const uint8_t *data, const uint64_t *offsets, const uint32_t *sizes,
                      uint64_t n, uint8_t *digests) {
    for (uint64_t i = 0; i < n; i++)
        sfo_sha1(data + offsets[i], sizes[i], digests + 20 * i);
}

/* compute_blocks_hash, src/index.rs:661-682: SHA-1 over d0 || d1 || ... */
void sfo_blocks_hash(const uint8_t *digests, uint64_t n, uint8_t out[20]) {
    sfo_sha1(digests, n * 20u, out);
}

/* ------------------------------------ opt-in weak sum (not in reference) */

/* zlib Adler-32 (RFC 1950 section 9) of one byte range: the checker for the
 * product's opt-in fused weak sum.  The reference computes no weak sum
 * (SURVEY.md 8a row a8); zlib.adler32 cross-checks this in tests/. */
uint32_t sfo_adler32(const uint8_t *data, uint64_t len) {
    uint64_t a = 1, b = 0;
    for (uint64_t i = 0; i < len; i++) {
        a += data[i];
        b += a;
        if ((i & 4095) == 4095) { a %= 65521u; b %= 65521u; }
    }
    return (uint32_t)(((b % 65521u) << 16) | (a % 65521u));
}

void sfo_adler_fixed(const uint8_t *data, uint64_t len, uint64_t block_size, uint32_t *out) {
    uint64_t n = sfo_num_blocks(len, block_size);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t off = i * block_size;
        out[i] = sfo_adler32(data + off, len - off < block_size ? len - off : block_size);
    }
}

void sfo_adler_blocks(const uint8_t *data, const uint64_t *offsets, const uint32_t *sizes, uint64_t n,
                      uint32_t *out) {
    for (uint64_t i = 0; i < n; i++) out[i] = sfo_adler32(data + offsets[i], sizes[i]);
}

/* ---------------------------------------- multi-threaded CPU baseline */

typedef struct {
    const uint8_t *data; uint64_t len, bs, first, last; uint8_t *dig;
} sfo_job;

static void *sfo_worker(void *p) {
    sfo_job *j = (sfo_job *)p;
    for (uint64_t i = j->first; i < j->last; i++) {
        uint64_t off = i * j->bs;
        uint64_t sz = j->len - off < j->bs ? j->len - off : j->bs;
        sfo_sha1(j->data + off, sz, j->dig + 20 * i);
    }
    return NULL;
}

/* Fixed tiling across `threads` pthreads (the "all host cores" column). */
uint64_t sfo_index_fixed_mt(const uint8_t *data, uint64_t len, uint64_t block_size,
                            uint8_t *digests, int threads) {
    uint64_t n = sfo_num_blocks(len, block_size);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t tid[256];
    int joined[256];
    sfo_job jobs[256];
    uint64_t per = (n + threads - 1) / threads;
    int nj = 0;
    for (int t = 0; t < threads; t++) {
        uint64_t a = (uint64_t)t * per, b = a + per > n ? n : a + per;
        if (a >= b) break;
        jobs[t] = (sfo_job){data, len, block_size, a, b, digests};
        joined[t] = pthread_create(&tid[t], NULL, sfo_worker, &jobs[t]) == 0;
        if (!joined[t]) sfo_worker(&jobs[t]);
        nj++;
    }
    for (int t = 0; t < nj; t++)
        if (joined[t]) pthread_join(tid[t], NULL);
    return n;
}

/* ------------------------------------------------- synthetic generator */

/* splitmix64 byte stream: 64-bit word i of a stream
 * with seed s is mix(s + (i+1) * 0x9E3779B97F4A7C15), stored little-endian.
 * fill writes bytes [start, start+len) of that stream. */
static inline uint64_t sfo_mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void sfo_fill_splitmix(uint8_t *out, uint64_t len, uint64_t seed, uint64_t start) {
    uint64_t p = start, end = start + len;
    while (p < end) {
        uint64_t wi = p >> 3;
        uint64_t w = sfo_mix(seed + (wi + 1) * 0x9E3779B97F4A7C15ull);
        for (unsigned b = (unsigned)(p & 7); b < 8 && p < end; b++, p++)
            out[p - start] = (uint8_t)(w >> (8 * b));
    }
}
