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

}  // extern "C"
