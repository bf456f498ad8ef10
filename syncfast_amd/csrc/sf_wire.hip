// sf_wire.hip -- the FILE_BLOCK run of an explicit block list, built on the
// device (its own translation unit: the SHA-1 kernels' code object in
// sf_capi.hip stays as it is).
//
// The reference's source streams one FILE_BLOCK message per block after
// FILE_START (src/sync/fs.rs:217-233, written by write_message,
// src/sync/ssh/proto.rs:162-166): "FILE_BLOCK\n" + the 20 raw digest bytes +
// "\n" + the block's size in decimal + "\n".  With the reference's default,
// content-defined blocks every size differs, so message i starts at the sum
// of the earlier messages' lengths (33 + digits(size)): one pass writes the
// lengths, a rocprim inclusive scan turns them into end offsets, and one
// thread per message writes it at its place.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <rocprim/device/device_scan.hpp>

#include "sf_internal.hpp"

namespace {

__device__ __forceinline__ uint32_t digits10(uint32_t v) {
  uint32_t d = 1;
  while (v >= 10) { v /= 10; ++d; }
  return d;
}

__global__ void __launch_bounds__(256) wire_len_kernel(const uint32_t* __restrict__ sizes, uint64_t n,
                                                       uint64_t* __restrict__ lens) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) lens[i] = 33u + digits10(sizes[i]);  // 11 + 20 + 1 + digits + 1
}

// Message i goes to out + ends[i] - base - its length (base: the end offset
// of the message before the first one written, so a chunk of a longer run
// lands at the start of its own buffer).
__global__ void __launch_bounds__(256) wire_blocks_kernel(const uint8_t* __restrict__ digests,
                                                          const uint32_t* __restrict__ sizes,
                                                          const uint64_t* __restrict__ ends, uint64_t n,
                                                          uint64_t base, uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t v = sizes[i];
  const uint32_t nd = digits10(v);
  uint8_t* o = out + (ends[i] - base) - (33u + nd);
  const char tag[11] = {'F', 'I', 'L', 'E', '_', 'B', 'L', 'O', 'C', 'K', '\n'};
#pragma unroll
  for (int k = 0; k < 11; ++k) o[k] = (uint8_t)tag[k];
  const uint8_t* d = digests + i * 20;
#pragma unroll
  for (int k = 0; k < 20; ++k) o[11 + k] = d[k];
  o[31] = '\n';
  for (int k = (int)nd - 1; k >= 0; --k) { o[32 + k] = (uint8_t)('0' + v % 10); v /= 10; }
  o[32 + nd] = '\n';
}

// out[k] = ends[min((k + 1) * per, n) - 1]: the end offset of chunk k
__global__ void __launch_bounds__(256) wire_chunk_ends_kernel(const uint64_t* __restrict__ ends, uint64_t n,
                                                              uint64_t per, uint64_t nchunks,
                                                              uint64_t* __restrict__ out) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k < nchunks) out[k] = ends[std::min((k + 1) * per, n) - 1];
}

constexpr uint64_t kWireMaxPerLaunch = 1ull << 30;  // messages per launch (grid x stays far below 2^31)

}  // namespace

namespace sfi {

// The end offset of every message of the run (inclusive scan of the
// lengths), in stream-ordered scratch the caller frees with stream_free on
// `s`.
int wire_plan(const uint32_t* d_sizes, uint64_t n, uint64_t** d_ends, hipStream_t s) {
  *d_ends = nullptr;
  size_t tmp = 0;
  uint64_t* nul = nullptr;
  if (rocprim::inclusive_scan(nullptr, tmp, nul, nul, (size_t)n, rocprim::plus<uint64_t>(), s) != hipSuccess) {
    (void)hipGetLastError();
    return SF_ENODEV;
  }
  const size_t lb = (n * 8 + 255) & ~(size_t)255;
  uint8_t* ws = nullptr;  // ends first (returned), then lengths and the scan's temporary
  {
    const int arc = stream_alloc(reinterpret_cast<void**>(&ws), 2 * lb + tmp + 8, s);
    if (arc != SF_OK) return arc;
  }
  uint64_t* ends = reinterpret_cast<uint64_t*>(ws);
  uint64_t* lens = reinterpret_cast<uint64_t*>(ws + lb);
  int rc = SF_OK;
  // pieces of at most 2^30 messages per launch: a grid past 2^32 work-items
  // is not launched whole
  for (uint64_t first = 0; first < n && rc == SF_OK; first += kWireMaxPerLaunch) {
    const uint64_t cnt = std::min(kWireMaxPerLaunch, n - first);
    sfi::clear_stale_error();
    hipLaunchKernelGGL(wire_len_kernel, dim3((unsigned)ceil_div(cnt, 256)), dim3(256), 0, s, d_sizes + first, cnt,
                       lens + first);
    rc = hip_err(hipGetLastError());
  }
  if (rc == SF_OK &&
      rocprim::inclusive_scan(ws + 2 * lb, tmp, lens, ends, (size_t)n, rocprim::plus<uint64_t>(), s) != hipSuccess) {
    (void)hipGetLastError();
    rc = SF_ENODEV;
  }
  if (rc != SF_OK) {
    stream_free(ws, s);
    return rc;
  }
  *d_ends = ends;
  return SF_OK;
}

// d_chunk_ends[k] = end offset of chunk k (chunks of `per` messages).
int wire_chunk_ends(const uint64_t* d_ends, uint64_t n, uint64_t per, uint64_t* d_chunk_ends, hipStream_t s) {
  const uint64_t nchunks = ceil_div(n, per);
  sfi::clear_stale_error();
  hipLaunchKernelGGL(wire_chunk_ends_kernel, dim3((unsigned)ceil_div(nchunks, 256)), dim3(256), 0, s, d_ends, n, per,
                     nchunks, d_chunk_ends);
  return hip_err(hipGetLastError());
}

// Messages [first, first + cnt) of a planned run, written from the start of
// d_out (base = the end offset of message first - 1, 0 for the first).
int wire_build(const uint8_t* d_digests, const uint32_t* d_sizes, const uint64_t* d_ends, uint64_t first,
               uint64_t cnt, uint64_t base, uint8_t* d_out, hipStream_t s) {
  for (uint64_t a = 0; a < cnt; a += kWireMaxPerLaunch) {
    const uint64_t m = std::min(kWireMaxPerLaunch, cnt - a);
    sfi::clear_stale_error();
    hipLaunchKernelGGL(wire_blocks_kernel, dim3((unsigned)ceil_div(m, 256)), dim3(256), 0, s,
                       d_digests + (first + a) * 20, d_sizes + first + a, d_ends + first + a, m, base, d_out);
    const int rc = hip_err(hipGetLastError());
    if (rc != SF_OK) return rc;
  }
  return SF_OK;
}

}  // namespace sfi

extern "C" {

int sf_wire_blocks_device(const void* d_digests, const uint32_t* d_sizes, uint64_t n_blocks, void* d_out,
                          uint64_t cap, uint64_t* n_out, void* stream) {
  using sfi::ceil_div;
  if (n_out) *n_out = 0;
  if (n_blocks == 0) return SF_OK;
  if (!d_sizes) return SF_EINVAL;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  uint64_t* ends = nullptr;
  int rc = sfi::wire_plan(d_sizes, n_blocks, &ends, s);
  if (rc != SF_OK) return rc;
  uint64_t total = 0;
  do {
    // the need is the last end offset: read back (this call blocks here)
    if (hipMemcpyAsync(&total, ends + n_blocks - 1, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      rc = SF_ENODEV;
      break;
    }
    if (n_out) *n_out = total;
    if (total > cap || !d_out) { rc = SF_ENOSPC; break; }
    if (!d_digests) { rc = SF_EINVAL; break; }
    rc = sfi::wire_build(static_cast<const uint8_t*>(d_digests), d_sizes, ends, 0, n_blocks, 0,
                         static_cast<uint8_t*>(d_out), s);
  } while (0);
  sfi::stream_free(ends, s);
  return rc;
}

}  // extern "C"
