// sf_table.hip -- the explicit-list kernel, sha1_table_kernel (DESIGN.md
// section 3.4), in its own translation unit: its rate on content-defined
// lists depends on how it is compiled, so it is built apart from the fixed
// kernel (sf_capi.hip) and its machine code is pinned by a measurement.
#define SF_STREAM_TU 1  // the device functions of sf_kernels.hpp only
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sf_internal.hpp"
#include "sf_kernels.hpp"

namespace sfi {

int launch_table_kernel(bool weak_form, unsigned grid, const uint8_t* d_data, uint64_t len,
                        const uint64_t* d_offsets, const uint32_t* d_sizes, uint64_t nblocks, uint8_t* d_digests,
                        int* d_status, uint32_t* weak, const uint32_t* order, uint64_t work, uint64_t lane_slots,
                        hipStream_t stream) {
  if (weak_form)
    hipLaunchKernelGGL((sf::sha1_table_kernel<128, true>), dim3(grid), dim3(sf::kThreads), 0, stream, d_data, len,
                       d_offsets, d_sizes, nblocks, d_digests, d_status, weak, order, work, lane_slots);
  else
    hipLaunchKernelGGL((sf::sha1_table_kernel<128, false>), dim3(grid), dim3(sf::kThreads), 0, stream, d_data, len,
                       d_offsets, d_sizes, nblocks, d_digests, d_status, nullptr, order, work, lane_slots);
  return hip_err(hipGetLastError());
}

}  // namespace sfi
