// sf_chain.hip -- blocks_hash chains alone on the device (a stream's finish
// launches): sha1_chain_helper_kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sf_chain.hpp"
#include "sf_internal.hpp"

namespace sf {

// A stream's chain jobs on an otherwise idle GPU (BatchStream's finish
// launches, sf_index_device_batch_chained_cols with no blocks).  A lone chain
// wave issues every instruction of its compressions itself, 613 VALU per
// chunk, and a wave alone on its SIMD issues at that SIMD's rate.  Here each
// chain wave (wave 0: 64 files) has a helper wave in its workgroup (wave 1,
// on another SIMD) that loads the chunks (kChainDepth ahead), builds each
// chunk's message schedule and adds the round constants, kw[t] = K_t + W_t,
// into one of two LDS buffers; the chain wave reads them (20 ds_read_b128)
// and runs only the 80 rounds.  One s_barrier per chunk hands a buffer over:
// the helper fills buffer (c+1)&1 while the chain reads buffer c&1.
constexpr int kHelperThreads = 128;
struct KwBuf {
  uint4 q[2][20][64];  // [buffer][4 rounds][lane]: 40 KiB
};

__device__ __forceinline__ void kw_from_words(uint32_t (&w)[16], uint4 (&kwq)[20]) {
  uint32_t kw[80];
#pragma unroll
  for (int t = 0; t < 80; ++t) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      wt = rotl(xor3(w[(t + 13) & 15], w[(t + 8) & 15], w[(t + 2) & 15]) ^ w[t & 15], 1);
      w[t & 15] = wt;
    }
    const uint32_t k = t < 20 ? 0x5A827999u : t < 40 ? 0x6ED9EBA1u : t < 60 ? 0x8F1BBCDCu : 0xCA62C1D6u;
    kw[t] = wt + k;
  }
#pragma unroll
  for (int i = 0; i < 20; ++i) kwq[i] = make_uint4(kw[4 * i], kw[4 * i + 1], kw[4 * i + 2], kw[4 * i + 3]);
}

__global__ void __launch_bounds__(kHelperThreads)
sha1_chain_helper_kernel(const ChainJob j0, const ChainJob j1) {
  __shared__ KwBuf sb;
  const ChainJob& j = blockIdx.x < j0.waves ? j0 : j1;
  const uint32_t wave = blockIdx.x < j0.waves ? blockIdx.x : blockIdx.x - j0.waves;
  const int lane = threadIdx.x & 63;
  const bool helper = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 1;
  const uint32_t f_raw = wave * 64 + lane;
  const bool valid = f_raw < j.files;
  const uint32_t f = valid ? f_raw : j.files - 1;  // spare lanes repeat the last file, store nothing
  const uint8_t* p = j.runs + (uint64_t)f * j.run_len;
  const uint32_t nch = n_chunks(j.run_len), data_ch = j.run_len / 64;
  const uint32_t n_data = j.hi - j.lo, n = n_data + (j.part != 1 ? nch - data_ch : 0u);  // uniform
  if (helper) {
    constexpr int D = kChainDepth;
    const uint4* q = reinterpret_cast<const uint4*>(p + (uint64_t)j.lo * 64);
    uint4 buf[D][4];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const uint32_t c = (uint32_t)k < n_data ? (uint32_t)k : (n_data ? n_data - 1 : 0u);
#pragma unroll
      for (int i = 0; i < 4; ++i) buf[k][i] = n_data ? q[(uint64_t)c * 4 + i] : make_uint4(0, 0, 0, 0);
    }
    for (uint32_t c0 = 0; c0 < n; c0 += D) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const uint32_t c = c0 + k;
        if (c < n) {
          uint32_t w[16];
          if (c < n_data) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              w[4 * i + 0] = bswap32(buf[k][i].x);
              w[4 * i + 1] = bswap32(buf[k][i].y);
              w[4 * i + 2] = bswap32(buf[k][i].z);
              w[4 * i + 3] = bswap32(buf[k][i].w);
            }
            const uint32_t nx = c + D < n_data ? c + D : n_data - 1;
#pragma unroll
            for (int i = 0; i < 4; ++i) buf[k][i] = q[(uint64_t)nx * 4 + i];
          } else {
            build_tail_chunk(w, p, j.run_len, data_ch + (c - n_data), nch);
          }
          uint4 kwq[20];
          kw_from_words(w, kwq);
#pragma unroll
          for (int i = 0; i < 20; ++i) sb.q[c & 1][i][lane] = kwq[i];
          __syncthreads();
        }
      }
    }
    return;
  }
  Sha1 st;
  if (j.part == 2) {
    const uint32_t* sv = reinterpret_cast<const uint32_t*>(j.state + (uint64_t)f * 20);
    st.h0 = sv[0]; st.h1 = sv[1]; st.h2 = sv[2]; st.h3 = sv[3]; st.h4 = sv[4];
  } else {
    st.init();
  }
  for (uint32_t c = 0; c < n; ++c) {
    __syncthreads();  // the helper filled buffer c & 1
    uint32_t kw[80];
#pragma unroll
    for (int i = 0; i < 20; ++i) {
      const uint4 v = sb.q[c & 1][i][lane];
      kw[4 * i] = v.x; kw[4 * i + 1] = v.y; kw[4 * i + 2] = v.z; kw[4 * i + 3] = v.w;
    }
    st.compress_uniform(kw);
  }
  if (!valid) return;
  if (j.part == 1) {
    uint32_t* sv = reinterpret_cast<uint32_t*>(j.state + (uint64_t)f * 20);
    sv[0] = st.h0; sv[1] = st.h1; sv[2] = st.h2; sv[3] = st.h3; sv[4] = st.h4;
  } else {
    st.store(j.hashes + (uint64_t)f * 20);
  }
}

}  // namespace sf

namespace sfi {

int launch_chain_helper(const sf::ChainJob& j0, const sf::ChainJob& j1, hipStream_t stream) {
  const unsigned grid = j0.waves + j1.waves;
  if (grid == 0) return SF_OK;
  sfi::clear_stale_error();
  hipLaunchKernelGGL(sf::sha1_chain_helper_kernel, dim3(grid), dim3(sf::kHelperThreads), 0, stream, j0, j1);
  return hip_err(hipGetLastError());
}

}  // namespace sfi
