// host_sha1.cpp -- host-side SHA-1 for the sequential step of the path.
//
// compute_blocks_hash (/root/reference/src/index.rs:661-682) is ONE SHA-1 over
// a file's concatenated block digests: a Merkle-Damgard chain that cannot be
// split across lanes.  For a single large file it runs on a host core,
// overlapped with device work; for many files at once the device computes
// one file per lane instead (sf_index_device_batch).  This is a designed
// host stage, not a fallback of the block kernel.
//
// Uses the x86 SHA extensions (SHA-NI) when the CPU reports them, a portable
// scalar loop otherwise.
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "host_sha1.h"

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace sfh {

static inline uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void compress_scalar(uint32_t h[5], const uint8_t* p, size_t nblocks) {
  for (; nblocks; --nblocks, p += 64) {
    uint32_t w[80];
    for (int t = 0; t < 16; t++)
      w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) | ((uint32_t)p[4 * t + 2] << 8) |
             (uint32_t)p[4 * t + 3];
    for (int t = 16; t < 80; t++) w[t] = rol(w[t - 3] ^ w[t - 8] ^ w[t - 14] ^ w[t - 16], 1);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
    for (int t = 0; t < 80; t++) {
      uint32_t f, k;
      if (t < 20) { f = d ^ (b & (c ^ d)); k = 0x5A827999u; }
      else if (t < 40) { f = b ^ c ^ d; k = 0x6ED9EBA1u; }
      else if (t < 60) { f = (b & c) | (d & (b | c)); k = 0x8F1BBCDCu; }
      else { f = b ^ c ^ d; k = 0xCA62C1D6u; }
      uint32_t tmp = rol(a, 5) + f + e + k + w[t];
      e = d; d = c; c = rol(b, 30); b = a; a = tmp;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e;
  }
}

#if defined(__x86_64__)
// SHA-NI: 4 rounds per sha1rnds4.  Message group i (rounds 4i..4i+3) is
// W_i = msg2(msg1(W_{i-4}, W_{i-3}) ^ W_{i-2}, W_{i-1}); the E operand
// alternates between two registers.
__attribute__((target("sha,sse4.1,ssse3"))) static void compress_shani(uint32_t h[5], const uint8_t* p,
                                                                        size_t nblocks) {
  const __m128i bswap_mask = _mm_set_epi64x(0x0001020304050607ULL, 0x08090a0b0c0d0e0fULL);
  __m128i abcd = _mm_shuffle_epi32(_mm_loadu_si128((const __m128i*)h), 0x1B);
  __m128i e0 = _mm_set_epi32((int)h[4], 0, 0, 0);
  for (; nblocks; --nblocks, p += 64) {
    const __m128i abcd_save = abcd, e0_save = e0;
    __m128i w[4];
    for (int i = 0; i < 4; i++) w[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * i)), bswap_mask);
    __m128i e1;
    e0 = _mm_add_epi32(e0, w[0]);
    e1 = abcd;
    abcd = _mm_sha1rnds4_epu32(abcd, e0, 0);
#define SF_GROUP(i, F)                                                                               \
  do {                                                                                             \
    __m128i wi;                                                                                    \
    if ((i) < 4) wi = w[(i)];                                                                      \
    else {                                                                                         \
      wi = _mm_sha1msg2_epu32(_mm_xor_si128(_mm_sha1msg1_epu32(w[(i) & 3], w[((i) + 1) & 3]),    \
                                            w[((i) + 2) & 3]),                                     \
                              w[((i) + 3) & 3]);                                                   \
      w[(i) & 3] = wi;                                                                             \
    }                                                                                              \
    if ((i) & 1) { e1 = _mm_sha1nexte_epu32(e1, wi); e0 = abcd; abcd = _mm_sha1rnds4_epu32(abcd, e1, F); } \
    else { e0 = _mm_sha1nexte_epu32(e0, wi); e1 = abcd; abcd = _mm_sha1rnds4_epu32(abcd, e0, F); }          \
  } while (0)
    SF_GROUP(1, 0); SF_GROUP(2, 0); SF_GROUP(3, 0); SF_GROUP(4, 0);
    SF_GROUP(5, 1); SF_GROUP(6, 1); SF_GROUP(7, 1); SF_GROUP(8, 1); SF_GROUP(9, 1);
    SF_GROUP(10, 2); SF_GROUP(11, 2); SF_GROUP(12, 2); SF_GROUP(13, 2); SF_GROUP(14, 2);
    SF_GROUP(15, 3); SF_GROUP(16, 3); SF_GROUP(17, 3); SF_GROUP(18, 3); SF_GROUP(19, 3);
#undef SF_GROUP
    e0 = _mm_sha1nexte_epu32(e0, e0_save);
    abcd = _mm_add_epi32(abcd, abcd_save);
  }
  abcd = _mm_shuffle_epi32(abcd, 0x1B);
  _mm_storeu_si128((__m128i*)h, abcd);
  h[4] = (uint32_t)_mm_extract_epi32(e0, 3);
}
#endif

static bool have_shani() {
#if defined(__x86_64__)
  static int cached = -1;
  if (cached < 0) {
    __builtin_cpu_init();
    cached = (__builtin_cpu_supports("sha") && __builtin_cpu_supports("sse4.1")) ? 1 : 0;
  }
  return cached == 1;
#else
  return false;
#endif
}

static void compress(uint32_t h[5], const uint8_t* p, size_t nblocks, bool shani) {
#if defined(__x86_64__)
  if (shani) { compress_shani(h, p, nblocks); return; }
#endif
  (void)shani;
  compress_scalar(h, p, nblocks);
}

}  // namespace sfh

extern "C" void sf_host_sha1_impl(const uint8_t* data, uint64_t len, uint8_t out[20], int force_scalar) {
  using namespace sfh;
  const bool shani = !force_scalar && have_shani();
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  const uint64_t full = len / 64;
  if (full) compress(h, data, full, shani);
  uint8_t tail[128];
  const size_t rem = (size_t)(len - full * 64);
  memset(tail, 0, sizeof tail);
  if (rem) memcpy(tail, data + full * 64, rem);
  tail[rem] = 0x80;
  const size_t tblocks = rem < 56 ? 1 : 2;
  const uint64_t bits = len * 8u;
  for (int i = 0; i < 8; i++) tail[tblocks * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
  compress(h, tail, tblocks, shani);
  for (int i = 0; i < 5; i++) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}

extern "C" int sf_host_has_shani(void) { return sfh::have_shani() ? 1 : 0; }

// Streaming form (internal to the library, not in include/): the in-place
// host pipelines fold each stage's digests into a file's blocks_hash while the
// next stage is still on the PCIe link (src/index.rs:661-682 hashes the
// concatenated digests in order).
extern "C" void sf_host_sha1_begin(sf_host_sha1_stream* s) {
  static const uint32_t iv[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  memcpy(s->h, iv, sizeof iv);
  s->nbuf = 0;
  s->total = 0;
  s->shani = sfh::have_shani() ? 1 : 0;
}

extern "C" void sf_host_sha1_update(sf_host_sha1_stream* s, const uint8_t* p, uint64_t n) {
  s->total += n;
  if (s->nbuf) {
    const uint64_t take = std::min<uint64_t>(64 - s->nbuf, n);
    memcpy(s->buf + s->nbuf, p, take);
    s->nbuf += (uint32_t)take;
    p += take;
    n -= take;
    if (s->nbuf < 64) return;
    sfh::compress(s->h, s->buf, 1, s->shani);
    s->nbuf = 0;
  }
  const uint64_t full = n / 64;
  if (full) sfh::compress(s->h, p, full, s->shani);
  s->nbuf = (uint32_t)(n - full * 64);
  if (s->nbuf) memcpy(s->buf, p + full * 64, s->nbuf);
}

extern "C" void sf_host_sha1_final(sf_host_sha1_stream* s, uint8_t out[20]) {
  uint8_t tail[128];
  memset(tail, 0, sizeof tail);
  if (s->nbuf) memcpy(tail, s->buf, s->nbuf);
  tail[s->nbuf] = 0x80;
  const size_t tblocks = s->nbuf < 56 ? 1 : 2;
  const uint64_t bits = s->total * 8u;
  for (int i = 0; i < 8; i++) tail[tblocks * 64 - 1 - i] = (uint8_t)(bits >> (8 * i));
  sfh::compress(s->h, tail, tblocks, s->shani);
  for (int i = 0; i < 5; i++) {
    out[4 * i] = (uint8_t)(s->h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(s->h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(s->h[i] >> 8);
    out[4 * i + 3] = (uint8_t)s->h[i];
  }
}
