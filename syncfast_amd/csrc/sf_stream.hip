// sf_stream.hip -- config 3 as a stream of batches:
// sha1_fixed_chained_kernel, one launch per batch hashing its blocks with
// the blocks_hash chains of earlier batches in its first workgroups.
//
// Its own translation unit: how its block part is compiled decides its rate
// (one compiled form of the same source ran 3 % slower than the plain kernel,
// another at its rate), so no change elsewhere may move it.  The measured
// form's machine code is recorded in profiles/r03/c3/chained_kernel.json.
#define SF_STREAM_TU 1  // the device functions of sf_kernels.hpp, not sf_capi.hip's kernels
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sf_internal.hpp"
#include "sf_kernels.hpp"

namespace sf {

// Equal-size many-file batches as a stream (BASELINE configs[2], batch after
// batch): ONE launch hashes every block of batch i (fixed_wave) and, in its
// first workgroups, up to two chain jobs of earlier batches (j0 then j1):
// with split chains, the second half of batch i-2's and the first half of
// batch i-1's.  Their digest tables and saved states were completed by
// earlier launches on the same stream, so no workgroup of this launch waits
// on another.  Halving each chain halves the latency it needs to hide: a
// chain lane beside the block waves runs ~3x slower than alone.
template <int TILE>
__global__ void __launch_bounds__(kThreads, 1)
sha1_fixed_chained_kernel(const uint8_t* __restrict__ data, uint64_t len, uint32_t bs, uint64_t nblocks,
                          uint8_t* __restrict__ digests, const PadSchedule pad, const ChainJob j0,
                          const ChainJob j1, const uint32_t wpf, const uint32_t wpp, const uint32_t poff) {
  // Chain waves are spread one per workgroup: workgroup g < C runs chain
  // wave g as its wave 0 (job 0's waves first) and block waves 3g..3g+2 as
  // its waves 1-3; the other workgroups run 4 block waves each.  So no CU
  // hosts more than one chain wave per workgroup, and the chains' scattered
  // digest loads are spread over C CUs instead of C/4.
  __shared__ uint4 smem[kWavesPerWG * 64 * (TILE / 16)];
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t C = j0.waves + j1.waves;  // chain waves
  const uint32_t g = blockIdx.x;
  uint64_t bw;
  if (g < C) {
    if (wid == 0) {
      if (g < j0.waves) chain_job(j0, g, smem);
      else chain_job(j1, g - j0.waves, smem);
      return;
    }
    bw = (uint64_t)g * 3 + (wid - 1);
  } else {
    bw = (uint64_t)C * 3 + (uint64_t)(g - C) * kWavesPerWG + wid;
  }
  // A column-range launch (wpp < wpf: every file's block waves [poff,
  // poff + wpp) of its wpf) maps its wave bw to the file's wave.
  if (wpp != wpf) bw = (uint64_t)((uint32_t)bw / wpp) * wpf + poff + (uint32_t)bw % wpp;
  fixed_wave<TILE, false>(data, len, bs, nblocks, digests, pad, nullptr, bw, smem + wid * 64 * (TILE / 16));
}

}  // namespace sf

namespace sfi {

int launch_chained(const uint8_t* data, uint64_t len, uint32_t bs, uint64_t nblocks, uint8_t* digests,
                   const sf::PadSchedule& pad, const sf::ChainJob& j0, const sf::ChainJob& j1, uint64_t bwaves,
                   uint32_t wpf, uint32_t wpp, uint32_t poff, hipStream_t stream) {
  // grid: C mixed workgroups (1 chain wave + 3 block waves), then 4 block
  // waves per workgroup for the rest
  const uint64_t C = j0.waves + j1.waves;
  const uint64_t rest = bwaves > 3 * C ? bwaves - 3 * C : 0;
  const unsigned grid = (unsigned)(C + ceil_div(rest, sf::kWavesPerWG));
  if (grid == 0) return SF_OK;
  sfi::clear_stale_error();
  hipLaunchKernelGGL(sf::sha1_fixed_chained_kernel<128>, dim3(grid), dim3(sf::kThreads), 0, stream, data, len, bs,
                     nblocks, digests, pad, j0, j1, wpf, wpp, poff);
  return hip_err(hipGetLastError());
}

}  // namespace sfi
