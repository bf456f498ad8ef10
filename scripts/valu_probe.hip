// valu_probe.hip -- per-instruction VALU throughput on gfx950 (MI355X).
// Each lane runs 8 independent dependency chains of one instruction type;
// reports wave-instructions per SIMD per cycle (s_memtime cycles) and
// per second, at W waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 2048
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t r0 = threadIdx.x ^ seed, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 11, r5 = r0 * 13, r6 = r0 * 17, r7 = r0 * 19;
  uint32_t s = seed | 1;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; i++) {
#define STEP(r) \
    if (OP == 0) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(r1)); \
    if (OP == 1) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(r)); \
    if (OP == 2) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r) : "v"(r2), "s"(s)); \
    if (OP == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r) : "v"(r2), "v"(r3)); \
    if (OP == 4) asm volatile("v_perm_b32 %0, 0, %0, %1" : "+v"(r) : "s"(s)); \
    if (OP == 5) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(r1)); \
    if (OP == 6) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(r) : "v"(r1), "v"(r2)); \
    if (OP == 7) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(r) : "v"(r1), "v"(r2));
    STEP(r0) STEP(r1) STEP(r2) STEP(r3) STEP(r4) STEP(r5) STEP(r6) STEP(r7)
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 256 + threadIdx.x] = r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
int run(const char* name, int waves_per_simd, uint32_t* out, uint64_t* cyc, uint64_t* hcyc) {
  int nblk = 256 * waves_per_simd;  // 256 CUs x (4 waves per block = 1 per SIMD) x W
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipLaunchKernelGGL(k<OP>, dim3(nblk), dim3(256), 0, 0, out, cyc, 1u);
  CHK(hipDeviceSynchronize());
  hipEventRecord(a);
  hipLaunchKernelGGL(k<OP>, dim3(nblk), dim3(256), 0, 0, out, cyc, 3u);
  hipEventRecord(b);
  CHK(hipDeviceSynchronize());
  float ms; hipEventElapsedTime(&ms, a, b);
  CHK(hipMemcpy(hcyc, cyc, nblk * 4 * 8, hipMemcpyDeviceToHost));
  double avg = 0; for (int i = 0; i < nblk * 4; i++) avg += hcyc[i]; avg /= nblk * 4;
  double winstr = (double)nblk * 4 * ITERS * 8;  // wave-instructions
  double per_simd_per_s = winstr / 1024 / (ms * 1e-3);
  // cycles per wave-instruction per SIMD, from the wave's own cycle count
  double cyc_per_inst = avg / (ITERS * 8.0) / waves_per_simd;
  printf("%-10s W=%d  %.3f ms  %.3e winst/SIMD/s (=%.2f cyc @2.4GHz)  s_memtime: %.2f cyc/inst/SIMD\n",
         name, waves_per_simd, ms, per_simd_per_s, 2.4e9 / per_simd_per_s, cyc_per_inst);
  return 0;
}

int main() {
  uint32_t* out; uint64_t* cyc; uint64_t* hcyc = (uint64_t*)malloc(256 * 8 * 4 * 8);
  CHK(hipMalloc(&out, 256 * 8 * 256 * 4)); CHK(hipMalloc(&cyc, 256 * 8 * 4 * 8));
  for (int w : {1, 2, 4, 8}) {
    run<0>("xor", w, out, cyc, hcyc); run<1>("alignbit", w, out, cyc, hcyc); run<2>("add3", w, out, cyc, hcyc);
    run<3>("bitop3", w, out, cyc, hcyc); run<4>("perm", w, out, cyc, hcyc); run<5>("add_u32", w, out, cyc, hcyc);
    run<6>("fma_f32", w, out, cyc, hcyc); run<7>("bfi", w, out, cyc, hcyc);
  }
  return 0;
}
