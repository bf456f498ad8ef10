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

namespace sfi {

int launch_table_kernel(bool weak_form, const uint8_t* d_data, uint64_t len, const uint64_t* d_offsets,
                        const uint32_t* d_sizes, uint64_t nblocks, uint8_t* d_digests, int* d_status, uint32_t* weak,
                        const uint32_t* order, hipStream_t stream) {
  const uint64_t ngroups = (nblocks + 63) / 64;
  const unsigned grid = (unsigned)((ngroups + sf::kTableWG - 1) / sf::kTableWG);
  sfi::clear_stale_error();
  if (weak_form)
    hipLaunchKernelGGL((sf::sha1_table_kernel<128, true>), dim3(grid), dim3(64 * sf::kTableWG), 0, stream, d_data, len,
                       d_offsets, d_sizes, nblocks, d_digests, d_status, weak, order);
  else
    hipLaunchKernelGGL((sf::sha1_table_kernel<128, false>), dim3(grid), dim3(64 * sf::kTableWG), 0, stream, d_data, len,
                       d_offsets, d_sizes, nblocks, d_digests, d_status, nullptr, order);
  return hip_err(hipGetLastError());
}

}  // namespace sfi
