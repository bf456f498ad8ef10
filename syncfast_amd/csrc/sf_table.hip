// sf_table.hip -- the explicit-list kernel, sha1_table_kernel (DESIGN.md
// section 3.4), in its own translation unit, so that a change to it cannot
// move how the fixed kernel (sf_capi.hip) compiles, and its compiler options
// can differ from the fixed kernel's.
#define SF_STREAM_TU 1  // the device functions of sf_kernels.hpp only
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "sf_internal.hpp"
#include "sf_kernels.hpp"

#ifdef SF_WAVE_TRACE
// Diagnostic build: the per-wave trace buffer (8 uint32 per wave) the next
// plain launches write; NULL turns tracing off.
static uint32_t* g_trace = nullptr;
extern "C" int sf_trace_set(void* d_trace) {
  g_trace = static_cast<uint32_t*>(d_trace);
  return 0;
}
#endif

namespace sfi {

#ifndef SF_TABLE_WPS
#define SF_TABLE_WPS SF_TABLE_LB  // waves per SIMD of a persistent launch (A/B builds with SF_TABLE_PERSIST=1)
#endif

int launch_table_kernel(bool weak_form, unsigned grid, const uint8_t* d_data, uint64_t len,
                        const uint64_t* d_offsets, const uint32_t* d_sizes, uint64_t nblocks, uint8_t* d_digests,
                        int* d_status, uint32_t* weak, const uint32_t* order, uint32_t* next_group, unsigned cus,
                        hipStream_t stream) {
  (void)grid;  // the caller's grid assumes 4-wave workgroups: sized here for SF_TABLE_WG
  const uint64_t ngroups = (nblocks + 63) / 64;
  grid = (unsigned)((ngroups + SF_TABLE_WG - 1) / SF_TABLE_WG);
#if SF_TABLE_PERSIST
  // persistent (A/B): SF_TABLE_WPS waves per SIMD (SF_TABLE_WPS 2/SIMD: SF_TABLE_LB 3 code)
  if (next_group) grid = (unsigned)std::min<uint64_t>(grid, (uint64_t)SF_TABLE_WPS * cus * 4 / SF_TABLE_WG);
#else
  next_group = nullptr;
  (void)cus;
#endif
  if (weak_form)
    hipLaunchKernelGGL((sf::sha1_table_kernel<128, true>), dim3(grid), dim3(64 * SF_TABLE_WG), 0, stream, d_data, len,
                       d_offsets, d_sizes, nblocks, d_digests, d_status, weak, order, next_group);
  else
#ifdef SF_WAVE_TRACE
    hipLaunchKernelGGL((sf::sha1_table_kernel<128, false>), dim3(grid), dim3(64 * SF_TABLE_WG), 0, stream, d_data, len,
                       d_offsets, d_sizes, nblocks, d_digests, d_status, g_trace, order, next_group);
#else
    hipLaunchKernelGGL((sf::sha1_table_kernel<128, false>), dim3(grid), dim3(64 * SF_TABLE_WG), 0, stream, d_data, len,
                       d_offsets, d_sizes, nblocks, d_digests, d_status, nullptr, order, next_group);
#endif
  return hip_err(hipGetLastError());
}

}  // namespace sfi
