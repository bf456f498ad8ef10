// sf_sort.hip -- the processing order of an explicit block list for
// sha1_table_kernel: a stable counting sort of the
// blocks by their length class (8-bit by default; 9 and 10 bits for the
// SF_TABLE_CLASS_BITS A/B), descending (list order within a class), in three
// small kernels.  It replaces a general radix sort that
// spent ~45 us per call (key kernel, three buffer fills, histogram and
// onesweep passes) on what is one pass over 256 bins.
//
// Its own translation unit, so that it cannot change how sf_capi.hip's
// block kernels compile.
#define SF_STREAM_TU 1  // the device functions of sf_kernels.hpp only
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sf_internal.hpp"
#include "sf_kernels.hpp"
#include "../../include/syncfast_amd_test.h"

namespace sf {

constexpr int kSortThreads = 256;
// blocks per thread per tile: 1024-block tiles (2048: scatter 9.8 -> 7.7 us
// at 1024 on the 0.5 M-block CDC-like list, profiles/r04/s28)
constexpr int kSortRounds = 4;
constexpr uint32_t kSortTile = kSortThreads * kSortRounds;  // blocks per tile
constexpr uint32_t kSortBinsMax = 1024;                      // 8- to 10-bit class keys

__device__ __forceinline__ uint32_t class_key(uint32_t size, uint32_t mbits, uint32_t kmax) {
  const uint32_t k = length_class(n_chunks_wide(size), mbits);
  return k < kmax ? k : kmax;
}

// Inclusive scan of v over the 256 threads of the workgroup; *total = the sum.
__device__ __forceinline__ uint32_t block_scan256(uint32_t v, uint32_t* wsum, uint32_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const uint32_t o = (uint32_t)__shfl_up((int)v, m, 64);
    if (lane >= m) v += o;
  }
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  uint32_t before = 0;
#pragma unroll
  for (int i = 0; i < kSortThreads / 64; ++i)
    if (i < w) before += wsum[i];
  *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();  // wsum is reused by the next call
  return v + before;
}

// 1. Class histogram of every tile, bin-major: hist[bin * ntiles + tile].
// BINS: 256, 512 or 1024 classes (8-, 9- or 10-bit keys); each of the 256
// threads owns BINS / 256 of them.
template <uint32_t BINS>
__global__ void __launch_bounds__(kSortThreads)
class_hist_kernel(const uint32_t* __restrict__ sizes, uint64_t n, uint32_t mbits, uint32_t kmax,
                  uint32_t* __restrict__ hist, uint32_t ntiles) {
  constexpr uint32_t BPT = BINS / kSortThreads;
  __shared__ uint32_t h[BINS];
  const uint32_t tid = threadIdx.x, tile = blockIdx.x;
#pragma unroll
  for (uint32_t j = 0; j < BPT; ++j) h[tid * BPT + j] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)tile * kSortTile;
#pragma unroll
  for (int r = 0; r < kSortRounds; ++r) {
    const uint64_t i = base + (uint64_t)r * kSortThreads + tid;
    if (i < n) atomicAdd(&h[class_key(sizes[i], mbits, kmax)], 1u);
  }
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < BPT; ++j) hist[(uint64_t)(tid * BPT + j) * ntiles + tile] = h[tid * BPT + j];
}

// 2. Per bin (one workgroup each): exclusive prefix over the tiles, in
// place, and the bin's total.
__global__ void __launch_bounds__(kSortThreads)
class_scan_kernel(uint32_t* __restrict__ hist, uint32_t ntiles, uint32_t* __restrict__ totals) {
  __shared__ uint32_t wsum[kSortThreads / 64];
  uint32_t* col = hist + (uint64_t)blockIdx.x * ntiles;
  uint32_t carry = 0;
  for (uint32_t t0 = 0; t0 < ntiles; t0 += kSortThreads) {
    const uint32_t t = t0 + threadIdx.x;
    const uint32_t v = t < ntiles ? col[t] : 0u;
    uint32_t total;
    const uint32_t incl = block_scan256(v, wsum, &total);
    if (t < ntiles) col[t] = carry + incl - v;
    carry += total;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

// 3. Scatter: block i goes to order[pos], pos = (blocks of higher classes)
// + (blocks of its class in earlier tiles) + (its rank in its tile: earlier
// rounds, earlier waves of its round, lower lanes of its wave).
template <uint32_t BINS>
__global__ void __launch_bounds__(kSortThreads)
class_scatter_kernel(const uint32_t* __restrict__ sizes, uint64_t n, uint32_t mbits, uint32_t kmax,
                     const uint32_t* __restrict__ hist, const uint32_t* __restrict__ totals, uint32_t ntiles,
                     uint32_t* __restrict__ order) {
  constexpr int kWaves = kSortThreads / 64;
  constexpr uint32_t BPT = BINS / kSortThreads;
  constexpr int KBITS = BINS == 256 ? 8 : BINS == 512 ? 9 : 10;
  __shared__ uint32_t running[BINS];
  __shared__ uint32_t wcnt[kWaves][BINS];
  __shared__ uint32_t wsum[kWaves];
  const uint32_t tid = threadIdx.x, tile = blockIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  // classes in descending order: bin b starts after every bin above it;
  // thread t holds bins BINS - 1 - (t * BPT + j), j < BPT
  uint32_t tb = 0;
#pragma unroll
  for (uint32_t j = 0; j < BPT; ++j) tb += totals[BINS - 1 - (tid * BPT + j)];
  uint32_t all;
  uint32_t above = block_scan256(tb, wsum, &all) - tb;
#pragma unroll
  for (uint32_t j = 0; j < BPT; ++j) {
    const uint32_t b = BINS - 1 - (tid * BPT + j);
    running[b] = above + hist[(uint64_t)b * ntiles + tile];
    above += totals[b];
  }
#pragma unroll
  for (int i = 0; i < kWaves; ++i)
#pragma unroll
    for (uint32_t j = 0; j < BPT; ++j) wcnt[i][tid * BPT + j] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)tile * kSortTile;
  const uint64_t lt = (1ull << lane) - 1ull;  // lanes below this one
  for (int r = 0; r < kSortRounds; ++r) {
    const uint64_t i = base + (uint64_t)r * kSortThreads + tid;
    const bool valid = i < n;
    const uint32_t k = valid ? class_key(sizes[i], mbits, kmax) : 0u;
    // lanes of this wave holding the same key: AND of the key's bit-plane ballots
    uint64_t eq = __ballot(valid);
#pragma unroll
    for (int b = 0; b < KBITS; ++b) {
      const uint64_t m = __ballot((k >> b) & 1u);
      eq &= ((k >> b) & 1u) ? m : ~m;
    }
    const uint32_t lower = (uint32_t)__popcll(eq & lt);
    const bool leader = valid && lower == 0;
    if (leader) wcnt[w][k] = (uint32_t)__popcll(eq);
    __syncthreads();
    uint32_t pos = 0;
    if (valid) {
      pos = running[k] + lower;
      for (int v = 0; v < w; ++v) pos += wcnt[v][k];
    }
    __syncthreads();  // every lane has read running / wcnt
#pragma unroll
    for (uint32_t j = 0; j < BPT; ++j) {
      const uint32_t b = tid * BPT + j;
      uint32_t add = 0;
#pragma unroll
      for (int v = 0; v < kWaves; ++v) {
        add += wcnt[v][b];
        wcnt[v][b] = 0;
      }
      running[b] += add;
    }
    __syncthreads();
    if (valid) order[pos] = (uint32_t)i;
  }
}

}  // namespace sf

namespace sfi {

static uint32_t sort_bins(uint32_t kmax) { return kmax < 256 ? 256u : kmax < 512 ? 512u : 1024u; }

size_t class_order_workspace(uint64_t n, uint32_t kmax) {
  const uint64_t ntiles = (n + sf::kSortTile - 1) / sf::kSortTile, bins = sort_bins(kmax);
  return (size_t)(ntiles * bins + bins) * 4;
}

template <uint32_t BINS>
static void class_order_launch(const uint32_t* d_sizes, uint64_t n, uint32_t mbits, uint32_t kmax, uint32_t* hist,
                               uint32_t ntiles, uint32_t* d_order, hipStream_t s) {
  uint32_t* totals = hist + (uint64_t)ntiles * BINS;
  sfi::clear_stale_error();
  hipLaunchKernelGGL(sf::class_hist_kernel<BINS>, dim3(ntiles), dim3(sf::kSortThreads), 0, s, d_sizes, n, mbits, kmax,
                     hist, ntiles);
  hipLaunchKernelGGL(sf::class_scan_kernel, dim3(BINS), dim3(sf::kSortThreads), 0, s, hist, ntiles, totals);
  hipLaunchKernelGGL(sf::class_scatter_kernel<BINS>, dim3(ntiles), dim3(sf::kSortThreads), 0, s, d_sizes, n, mbits,
                     kmax, hist, totals, ntiles, d_order);
}

int class_order(const uint32_t* d_sizes, uint64_t n, uint32_t mbits, uint32_t kmax, void* d_ws, uint32_t* d_order,
                hipStream_t s) {
  if (n == 0) return SF_OK;
  if (n > 0xFFFFFFFFull || kmax >= sf::kSortBinsMax) return SF_EINVAL;
  const uint32_t ntiles = (uint32_t)((n + sf::kSortTile - 1) / sf::kSortTile);
  uint32_t* hist = static_cast<uint32_t*>(d_ws);
  if (kmax < 256)
    class_order_launch<256>(d_sizes, n, mbits, kmax, hist, ntiles, d_order, s);
  else if (kmax < 512)
    class_order_launch<512>(d_sizes, n, mbits, kmax, hist, ntiles, d_order, s);
  else
    class_order_launch<1024>(d_sizes, n, mbits, kmax, hist, ntiles, d_order, s);
  return hip_err(hipGetLastError());
}

}  // namespace sfi

extern "C" int sf_test_table_order_bits(const uint32_t* d_sizes, uint64_t n, uint32_t mbits, uint32_t* d_order,
                                        void* stream) {
  if (mbits < 1 || mbits > 6) return SF_EINVAL;
  if (n == 0) return SF_OK;
  if (!d_sizes || !d_order || n > 0xFFFFFFFFull) return SF_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  void* ws = nullptr;
  const uint32_t kmax = (16u << (mbits < 4 ? 4 : mbits)) - 1u;
  const int arc = sfi::stream_alloc(&ws, sfi::class_order_workspace(n, kmax), s);
  if (arc != SF_OK) return arc;
  const int rc = sfi::class_order(d_sizes, n, mbits, kmax, ws, d_order, s);
  sfi::stream_free(ws, s);
  return rc;
}

extern "C" int sf_test_table_order(const uint32_t* d_sizes, uint64_t n, uint32_t* d_order, void* stream) {
  return sf_test_table_order_bits(d_sizes, n, 4, d_order, stream);
}
