// sf_litmus.hip -- test hook sf_test_xcd_litmus (include/syncfast_amd_test.h):
// the cross-XCD counter read that round 5's fused many-file launch's
// blocks_hash lanes polled (sha1_staged_kernel, removed in round 6), in
// isolation.  Its own translation unit, so it cannot change how the product
// kernels compile.
//
// One launch of kLitmusWGs one-wave workgroups, lane 0 of each doing the work:
//   * workgroup 0 (the reader) reads the counter once with the form under
//     test -- mode 0: a relaxed agent-scope atomic load (`global_load ... sc1`,
//     round 5's poll); mode 1: an agent-scope atomic add of an opaque zero
//     -- which puts the counter's line in its XCD's L2 for mode 0 if loads
//     allocate there, then publishes its XCD id;
//   * every other workgroup on ANOTHER XCD adds 1 to the counter once the
//     reader says go; workgroups on the reader's XCD never touch the counter's
//     line (a same-XCD atomic would drop it from that L2);
//   * after every add has returned, the reader reads the counter again with
//     the same form, then with the add of an opaque zero.
// A stale form returns the first value on its second read although every add
// is done.  Every hand-shake word lives on a line of its own and is only ever
// touched by atomic read-modify-writes; every wait is bounded (status 1).
#include <hip/hip_runtime.h>

#include "sf_internal.hpp"
#include "../../include/syncfast_amd_test.h"

namespace {

constexpr int kLitmusWGs = 64;
constexpr uint32_t kSpinLimit = 1u << 22;

// word layout (uint32 index): each 32-word group is one 128-B line
enum : int {
  W_COUNTER = 0,     // the counter under test, alone on its line
  W_READER_XCC = 32,  // reader's XCD id + 1 (0 = not yet published)
  W_REGISTERED = 64,  // workgroups other than the reader that saw the id
  W_ADDERS = 96,      // of those, the ones on another XCD
  W_GO = 128,         // 1 once the reader has seen every registration
  W_DONE = 160,       // adds that have returned
  W_RESULT = 192,     // results (sf_test_xcd_litmus's out[8])
  W_WORDS = 224
};

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xF;
}

__device__ __forceinline__ uint32_t rmw_read(uint32_t* p) {
  uint32_t zero;
  asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
  return __hip_atomic_fetch_add(p, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t read_form(uint32_t* p, int mode) {
  return mode == 0 ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : rmw_read(p);
}

// Waits until rmw_read(p) >= want; false if the bound ran out.
__device__ __forceinline__ bool wait_at_least(uint32_t* p, uint32_t want) {
  for (uint32_t spins = 0; spins < kSpinLimit; ++spins) {
    if (rmw_read(p) >= want) return true;
    __builtin_amdgcn_s_sleep(2);
  }
  return false;
}

__global__ void __launch_bounds__(64) xcd_litmus_kernel(uint32_t* __restrict__ w, int mode) {
  if (threadIdx.x != 0) return;
  const uint32_t me = xcc_id();
  if (blockIdx.x == 0) {
    uint32_t* r = w + W_RESULT;
    const uint32_t v0 = read_form(w + W_COUNTER, mode);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    (void)__hip_atomic_exchange(w + W_READER_XCC, me + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t status = 0, adders = 0, v1 = 0, fresh = 0;
    if (!wait_at_least(w + W_REGISTERED, kLitmusWGs - 1)) {
      status = 1;
    } else {
      adders = rmw_read(w + W_ADDERS);
      (void)__hip_atomic_exchange(w + W_GO, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!wait_at_least(w + W_DONE, adders)) status = 1;
      v1 = read_form(w + W_COUNTER, mode);
      fresh = rmw_read(w + W_COUNTER);
    }
    // plain vector stores: the host reads them after the launch
    r[0] = status;
    r[1] = me;
    r[2] = adders;
    r[3] = v0;
    r[4] = v1;
    r[5] = fresh;
    r[6] = (uint32_t)mode;
    r[7] = 0;
    return;
  }
  // every other workgroup: learn the reader's XCD, register, add if on another
  if (!wait_at_least(w + W_READER_XCC, 1)) return;  // the reader's wait then runs out too
  const uint32_t reader = rmw_read(w + W_READER_XCC) - 1;
  const bool adder = me != reader;
  if (adder) (void)__hip_atomic_fetch_add(w + W_ADDERS, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the adder count must land before the registration the reader waits on
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  (void)__hip_atomic_fetch_add(w + W_REGISTERED, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!adder) return;
  if (!wait_at_least(w + W_GO, 1)) return;
  (void)__hip_atomic_fetch_add(w + W_COUNTER, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the add is complete (vmcnt counts writes and atomics on gfx9) before DONE moves
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  (void)__hip_atomic_fetch_add(w + W_DONE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

extern "C" int sf_test_xcd_litmus(int mode, uint32_t out[8]) {
  if ((mode != 0 && mode != 1) || !out) return SF_EINVAL;
  uint32_t* w = nullptr;
  SF_HIP(hipMalloc(reinterpret_cast<void**>(&w), W_WORDS * sizeof(uint32_t)));
  int rc = SF_OK;
  if (hipMemset(w, 0, W_WORDS * sizeof(uint32_t)) != hipSuccess) rc = SF_ENODEV;
  if (rc == SF_OK) {
    sfi::clear_stale_error();
    hipLaunchKernelGGL(xcd_litmus_kernel, dim3(kLitmusWGs), dim3(64), 0, nullptr, w, mode);
    rc = sfi::hip_err(hipGetLastError());
  }
  if (rc == SF_OK && hipMemcpy(out, w + W_RESULT, 8 * sizeof(uint32_t), hipMemcpyDeviceToHost) != hipSuccess)
    rc = SF_ENODEV;
  (void)hipFree(w);
  return rc;
}
