// sf_chain.hpp -- per-file blocks_hash chain jobs (device side), shared by
// sf_kernels.hpp (chains inside block launches) and sf_chain.hip (chains
// alone, with a schedule-building helper wave).  The helper kernel lives in
// its own translation unit so that adding or changing it cannot change how
// the block kernels of sf_capi.hip are compiled.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sha1_device.hpp"

namespace sf {

// One per-file blocks_hash chain job (src/index.rs:661-682) of a batch of
// equal-size files: one lane per file over its run of run_len digest bytes,
// data chunks [lo, hi) (64-B units) of the run.  part 0 = the whole chain;
// part 1 = chunks [0, hi), the 5-word SHA-1 state saved to state[f]; part 2
// = resume from state[f], chunks [lo, end) + the padding chunk(s), hash to
// hashes[f].
struct ChainJob {
  const uint8_t* runs;
  uint8_t* state;
  uint8_t* hashes;
  uint32_t files, run_len, lo, hi, part, waves;  // waves = chain waves (64 files each)
};

constexpr int kChainDepth = 4;  // 64-B chunks in flight per chain lane

}  // namespace sf

namespace sfi {
// sha1_chain_helper_kernel over jobs j0 (its j0.waves chain waves first) and
// j1 on `stream`; SF_OK or the launch error.
int launch_chain_helper(const sf::ChainJob& j0, const sf::ChainJob& j1, hipStream_t stream);
}  // namespace sfi

namespace sf {
struct PadSchedule;
}

namespace sfi {
// sha1_fixed_chained_kernel<128> (sf_stream.hip): `bwaves` block waves of 64
// blocks (a column range: wpp of every file's wpf waves from poff) beside
// the chain waves of j0 and j1.
int launch_chained(const uint8_t* data, uint64_t len, uint32_t bs, uint64_t nblocks, uint8_t* digests,
                   const sf::PadSchedule& pad, const sf::ChainJob& j0, const sf::ChainJob& j1, uint64_t bwaves,
                   uint32_t wpf, uint32_t wpp, uint32_t poff, hipStream_t stream);
}  // namespace sfi
