// sf_baseline.cpp -- CPU baseline with SHA-NI (TEST / BENCH INFRASTRUCTURE).
//
// bench.py's cpu_baseline_shani leg only: the fixed-tiling index_file loop
// (/root/reference/src/index.rs:621-647, one SHA-1 per block) on host cores,
// with the product's host SHA-1 (syncfast_amd/csrc/host_sha1.cpp, SHA-NI when
// the CPU has it) instead of the scalar C of sf_oracle.c.  It is the strongest
// CPU number for the same work, reported beside the scalar port that stands in
// for the reference's pure-Rust sha1 0.6 crate.  Never part of the product
// path; the product library has no CPU hashing of input blocks.
#include <stdint.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../syncfast_amd/csrc/host_sha1.h"
#include "../examples/zpaq_standin.h"

extern "C" {

int sfb_has_shani(void) { return sf_host_has_shani(); }

// digests: uint8[ceil(len/bs)][20]; threads >= 1 split the blocks evenly.
uint64_t sfb_index_fixed_shani(const uint8_t* data, uint64_t len, uint64_t bs, uint8_t* digests, int threads) {
  if (bs == 0) return 0;
  const uint64_t n = len ? (len + bs - 1) / bs : 0;
  auto run = [&](uint64_t b0, uint64_t b1) {
    for (uint64_t i = b0; i < b1; i++) {
      const uint64_t off = i * bs;
      sf_host_sha1_impl(data + off, std::min(bs, len - off), digests + 20 * i, 0);
    }
  };
  const uint64_t t = (uint64_t)std::max(1, threads);
  std::vector<std::thread> pool;
  const uint64_t per = (n + t - 1) / t;
  for (uint64_t k = 1; k < t && k * per < n; k++) pool.emplace_back(run, k * per, std::min(n, (k + 1) * per));
  run(0, std::min(n, per));
  for (auto& th : pool) th.join();
  return n;
}

// configs[0] stand-in (bench.py cpu_baseline's config1 block): the
// reference's default index_file loop over a buffer -- a ZPAQ-form chunker
// (examples/zpaq_standin.h: the crate's per-byte work, NOT its boundaries)
// with ZPAQ_BITS = 13 and MAX_BLOCK_SIZE = 32768 (/root/reference/src/
// index.rs:40-41).  sfb_zpaq_cut: the chunker alone, block sizes into
// sizes[0, cap) (the count is returned even past cap).  sfb_zpaq_index: the
// reference's single pass, each block SHA-1'd as it is cut
// (src/index.rs:629-647), scalar (the stand-in for the pure-Rust sha1 0.6
// crate) or SHA-NI; digests[0, cap).
uint64_t sfb_zpaq_cut(const uint8_t* data, uint64_t len, uint32_t* sizes, uint64_t cap) {
  sf_zpaq z;
  sf_zpaq_init(&z, 13, 32768);
  uint64_t n = 0, start = 0, p = 0;
  while (p < len) {
    const size_t k = sf_zpaq_next(&z, data + p, (size_t)(len - p));
    const uint64_t end = k ? p + k : len;
    if (n < cap) sizes[n] = (uint32_t)(end - start);
    n++;
    start = p = end;
  }
  return n;
}

uint64_t sfb_zpaq_index(const uint8_t* data, uint64_t len, uint8_t* digests, uint64_t cap, int shani) {
  sf_zpaq z;
  sf_zpaq_init(&z, 13, 32768);
  uint64_t n = 0, p = 0;
  while (p < len) {
    const size_t k = sf_zpaq_next(&z, data + p, (size_t)(len - p));
    const uint64_t end = k ? p + k : len;
    uint8_t d[20];
    sf_host_sha1_impl(data + p, end - p, n < cap ? digests + 20 * n : d, shani ? 0 : 1);
    n++;
    p = end;
  }
  return n;
}

}  // extern "C"
