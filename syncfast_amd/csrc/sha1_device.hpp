// sha1_device.hpp -- SHA-1 building blocks for gfx950 (one lane = one message).
//
// The arithmetic is FIPS 180-4 SHA-1, the function the reference applies per
// block through the `sha1 0.6.0` crate (/root/reference/src/index.rs:628-644)
// and over the digest list in compute_blocks_hash (src/index.rs:661-682).
//
// Cost model (CDNA4): one 64-byte compression = 80 rounds x 5 VALU
// (v_alignbit rotl5, v_bitop3 f, 2 x v_add3, v_alignbit rotl30) + 64 x 3
// schedule ops (v_bitop3 xor3, v_xor, v_alignbit rotl1) + 16 v_perm byte swaps
// + 5 feed-forward adds ~= 613 VALU per 64 B (checked in the .s: make isa).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sf {

__device__ __forceinline__ uint32_t rotl(uint32_t x, uint32_t n) {
  return __builtin_amdgcn_alignbit(x, x, 32u - n);
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Three-input boolean functions as ONE v_bitop3_b32 (gfx950).  The immediate
// is the truth table over (S0=0xF0, S1=0xCC, S2=0xAA).  hipcc does not form
// v_bitop3 from a^b^c on its own (it emits two v_xor_b32), so spell it out.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t ch(uint32_t b, uint32_t c, uint32_t d) {  // (b & c) | (~b & d)
  return __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA);
}
__device__ __forceinline__ uint32_t maj(uint32_t b, uint32_t c, uint32_t d) {  // (b&c) | (b&d) | (c&d)
  return __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8);
}

struct Sha1 {
  uint32_t h0, h1, h2, h3, h4;
  __device__ __forceinline__ void init() {
    h0 = 0x67452301u; h1 = 0xEFCDAB89u; h2 = 0x98BADCFEu; h3 = 0x10325476u; h4 = 0xC3D2E1F0u;
  }
  // One compression over 16 big-endian message words (w is clobbered: it
  // holds the rolling 16-word schedule window).
  __device__ __forceinline__ void compress(uint32_t (&w)[16]) {
    uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
#pragma unroll
    for (int t = 0; t < 80; ++t) {
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        wt = rotl(xor3(w[(t + 13) & 15], w[(t + 8) & 15], w[(t + 2) & 15]) ^ w[t & 15], 1);
        w[t & 15] = wt;
      }
      uint32_t f, k;
      if (t < 20) { f = ch(b, c, d); k = 0x5A827999u; }
      else if (t < 40) { f = xor3(b, c, d); k = 0x6ED9EBA1u; }
      else if (t < 60) { f = maj(b, c, d); k = 0x8F1BBCDCu; }
      else { f = xor3(b, c, d); k = 0xCA62C1D6u; }
      const uint32_t tmp = rotl(a, 5) + f + e + k + wt;
      e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
    }
    h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
  }
  // Compression of a chunk whose message words are the same for every lane
  // (the padding-only chunk ending a message of a 64-B multiple length).
  // kw[t] = K_t + W_t is precomputed on the host and arrives as kernel
  // arguments (SGPRs), so each round costs 4 VALU (rotl5, f, add3, add) and
  // there is no per-lane message schedule.
  __device__ __forceinline__ void compress_uniform(const uint32_t (&kw)[80]) {
    uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
#pragma unroll
    for (int t = 0; t < 80; ++t) {
      uint32_t f;
      if (t < 20) f = ch(b, c, d);
      else if (t < 40) f = xor3(b, c, d);
      else if (t < 60) f = maj(b, c, d);
      else f = xor3(b, c, d);
      const uint32_t tmp = rotl(a, 5) + f + e + kw[t];
      e = d; d = c; c = rotl(b, 30); b = a; a = tmp;
    }
    h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
  }
  // Same bytes, stored write-through (sc1: global_store_dword ... sc1) so a
  // consumer on another XCD can read them after a drain + flag, without an
  // agent-scope release fence on this side.
  __device__ __forceinline__ void store_writethrough(uint8_t* out20) const {
    uint32_t* o = reinterpret_cast<uint32_t*>(out20);
    __hip_atomic_store(o + 0, bswap32(h0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(o + 1, bswap32(h1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(o + 2, bswap32(h2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(o + 3, bswap32(h3), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(o + 4, bswap32(h4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // Digest bytes in sha1.digest().bytes() order (big-endian), as 5 words
  // ready for a little-endian store.
  __device__ __forceinline__ void store(uint8_t* out20) const {
    uint32_t* o = reinterpret_cast<uint32_t*>(out20);
    o[0] = bswap32(h0); o[1] = bswap32(h1); o[2] = bswap32(h2); o[3] = bswap32(h3); o[4] = bswap32(h4);
  }
};

// Weak per-block checksum: zlib Adler-32 (RFC 1950 s.9), NOT computed by the
// reference (no table, message or call site carries a
// weak sum); north_star asks for an "Adler32-style" weak sum beside the strong
// hash, so the kernels can fuse one as an opt-in second output.
//   A = 1 + sum(x_i),  B = sum over i of A after byte i  (both mod 65521).
// Per 64-B chunk of bytes x_0..x_63 (memory order): A += S1, B += 64*A + S2
// with S1 = sum x_i, S2 = sum (64 - i) x_i -- two v_dot4_u32_u8 per word.
// Between chunks A and B stay partially reduced (65536 = 15 mod 65521):
// a <= 65550 and b <= 66720 hold after every chunk, so nothing overflows 32
// bits for any block length; fin() reduces exactly.
struct Adler {
  uint32_t a, b;
  __device__ __forceinline__ void init() { a = 1u; b = 0u; }
  __device__ __forceinline__ static uint32_t fold(uint32_t x) { return (x & 0xFFFFu) + (x >> 16) * 15u; }
  // 16 little-endian words = the chunk's 64 bytes in memory order.
  __device__ __forceinline__ void chunk(const uint32_t (&le)[16]) {
    uint32_t s1 = 0u, s2 = 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      // byte k of word j is x_{4j+k}: weight 64 - 4j - k
      const uint32_t wt = (uint32_t)(64 - 4 * j) | ((uint32_t)(63 - 4 * j) << 8) |
                          ((uint32_t)(62 - 4 * j) << 16) | ((uint32_t)(61 - 4 * j) << 24);
      s1 = __builtin_amdgcn_udot4(le[j], 0x01010101u, s1, false);
      s2 = __builtin_amdgcn_udot4(le[j], wt, s2, false);
    }
    b = fold(b + (a << 6) + s2);  // < 66720 + 64 * 65550 + 530400 before the fold
    a = fold(a + s1);
  }
  // One trailing byte (fewer than 64 follow the last chunk()).
  __device__ __forceinline__ void byte(uint32_t x) {
    a += x;
    b += a;
  }
  __device__ __forceinline__ uint32_t fin() const {
    uint32_t A = fold(a), B = fold(b);
    A = A >= 65521u ? A - 65521u : A;
    B = B >= 65521u ? B - 65521u : B;
    return (B << 16) | A;
  }
};

// ------------------------------------------------ message helpers
__device__ __forceinline__ uint32_t ld_u32_any(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

// Number of SHA-1 compressions for a message of `size` bytes.  (size + 8)
// wraps for size >= 2^32 - 8: the fixed tiling's blocks (<= 32 MiB) and the
// digest runs (< 2^32 - 16) use this form; explicit lists, whose sizes are
// any uint32, use n_chunks_wide.
__device__ __forceinline__ uint32_t n_chunks(uint32_t size) { return (size + 8u) / 64u + 1u; }
// The same count for any uint32 size: (size + 8) / 64 + 1 without the
// 32-bit wrap (2^26 + 1 for size = 2^32 - 1).
__device__ __forceinline__ uint32_t n_chunks_wide(uint32_t size) {
  return (size >> 6) + 1u + (((size & 63u) + 8u) >> 6);
}

// Chunk c (0-based) of the padded message of a block of `size` bytes that
// starts at p (global memory).  Reads only bytes [0, size) of the block.
__device__ __forceinline__ void build_tail_chunk(uint32_t (&w)[16], const uint8_t* p, uint32_t size,
                                                 uint32_t c, uint32_t nch) {
  const int64_t rem = (int64_t)size - (int64_t)c * 64;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int64_t v = rem - 4 * j;  // valid data bytes in word j
    uint32_t x = 0;
    const uint8_t* q = p + (uint64_t)c * 64 + 4 * j;
    if (v >= 4) {
      x = bswap32(ld_u32_any(q));
    } else if (v > 0) {
      uint32_t y = (uint32_t)q[0] << 24;
      if (v > 1) y |= (uint32_t)q[1] << 16;
      if (v > 2) y |= (uint32_t)q[2] << 8;
      x = y | (0x80u << (8 * (3 - (int)v)));
    } else if (v == 0) {
      x = 0x80000000u;
    }
    w[j] = x;
  }
  if (c == nch - 1) {
    w[14] = size >> 29;
    w[15] = size << 3;
  }
}

}  // namespace sf
