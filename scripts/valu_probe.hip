// valu_probe.hip -- per-instruction VALU throughput on gfx950 (MI355X).
// Each lane runs 8 independent dependency chains of one instruction type;
// reports wave-instructions per SIMD per cycle (s_memtime cycles) and
// per second, at W waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 8192
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint64_t* cyc, uint32_t seed) {
  uint32_t r0 = threadIdx.x ^ seed, r1 = r0 * 3, r2 = r0 * 5, r3 = r0 * 7, r4 = r0 * 11, r5 = r0 * 13, r6 = r0 * 17, r7 = r0 * 19;
  uint32_t s = seed | 1;
  // per-lane non-trivial operands that never collapse to 0 (a random-data
  // proxy: toggling activity affects the clock)
  uint32_t vk = 0x9E3779B9u * (threadIdx.x + 1), vsel = 0x00010203u + (threadIdx.x & 0), vsh = 27 + (threadIdx.x & 0);
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
    if (OP == 7) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(r) : "v"(r1), "v"(r2)); \
    if (OP == 8) asm volatile("v_lshlrev_b32 %0, 5, %0" : "+v"(r)); \
    if (OP == 9) asm volatile("v_or_b32 %0, %0, %1" : "+v"(r) : "v"(r1)); \
    if (OP == 10) asm volatile("v_lshl_or_b32 %0, %0, 5, %1" : "+v"(r) : "v"(r1)); \
    if (OP == 11) asm volatile("v_lshl_add_u32 %0, %0, 5, %1" : "+v"(r) : "v"(r1)); \
    if (OP == 12) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(r) : "v"(r1), "v"(r2)); \
    if (OP == 13) asm volatile("v_add_u32 %0, %1, %0" : "+v"(r) : "s"(s)); \
    if (OP == 14) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(r) : "v"(r1)); \
    if (OP == 15) asm volatile("v_alignbyte_b32 %0, %0, %0, 1" : "+v"(r)); \
    if (OP == 16) asm volatile("v_lshrrev_b32 %0, 27, %0" : "+v"(r)); \
    if (OP == 17) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(r) : "s"(s)); \
    if (OP == 18) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(r) : "v"(r1) : "vcc"); \
    if (OP == 19) asm volatile("v_pk_lshlrev_b16 %0, 1, %0" : "+v"(r)); \
    if (OP == 20) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r) : "v"(r2), "s"(s)); \
    if (OP == 21) asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(r1)); \
    if (OP == 22) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(r) : "v"(r1), "v"(r2)); \
    if (OP == 23) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r) : "v"(r2), "v"(vk)); \
    if (OP == 24) asm volatile("v_perm_b32 %0, %0, %0, %1" : "+v"(r) : "v"(vsel)); \
    if (OP == 25) asm volatile("v_alignbit_b32 %0, %0, %0, %1" : "+v"(r) : "v"(vsh)); \
    if (OP == 26) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(r) : "v"(vsh)); \
    if (OP == 27) asm volatile("v_add_u32 %0, %0, %1" : "+v"(r) : "v"(vk)); \
    if (OP == 28) asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(r) : "v"(vsh)); \
    if (OP == 29) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r) : "v"(vk)); \
    if (OP == 30) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(r) : "v"(vk), "v"(vsel)); \
    if (OP == 31) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r) : "v"(vk), "v"(vsel)); \
    if (OP == 32) asm volatile("v_alignbit_b32 %0, %0, %1, 27" : "+v"(r) : "v"(vk));
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
  for (int w : {8}) {
    run<23>("add3_vvv", w, out, cyc, hcyc); run<24>("perm_vvv", w, out, cyc, hcyc); run<25>("alignbit_vsh", w, out, cyc, hcyc);
    run<26>("lshl_vsh", w, out, cyc, hcyc); run<27>("add_vk", w, out, cyc, hcyc); run<28>("lshr_vsh", w, out, cyc, hcyc);
    run<29>("xor_vk", w, out, cyc, hcyc); run<30>("bitop3_vk", w, out, cyc, hcyc); run<31>("add3_vk", w, out, cyc, hcyc);
    run<32>("alignbit_2src", w, out, cyc, hcyc);
  }
  for (int w : {8}) {
    run<0>("xor", w, out, cyc, hcyc); run<1>("alignbit", w, out, cyc, hcyc); run<2>("add3", w, out, cyc, hcyc);
    run<3>("bitop3", w, out, cyc, hcyc); run<4>("perm", w, out, cyc, hcyc); run<5>("add_u32", w, out, cyc, hcyc);
    run<6>("fma_f32", w, out, cyc, hcyc); run<7>("bfi", w, out, cyc, hcyc);
    run<8>("lshlrev", w, out, cyc, hcyc); run<9>("or", w, out, cyc, hcyc); run<10>("lshl_or", w, out, cyc, hcyc);
    run<11>("lshl_add", w, out, cyc, hcyc); run<12>("or3", w, out, cyc, hcyc); run<13>("add_sgpr", w, out, cyc, hcyc);
    run<14>("pk_add_u16", w, out, cyc, hcyc); run<15>("alignbyte", w, out, cyc, hcyc); run<16>("lshrrev", w, out, cyc, hcyc);
    run<17>("xor_sgpr", w, out, cyc, hcyc); run<18>("add_co", w, out, cyc, hcyc); run<19>("pk_lshl16", w, out, cyc, hcyc);
    run<20>("bitop3_sgpr", w, out, cyc, hcyc); run<21>("mov", w, out, cyc, hcyc); run<22>("and_or", w, out, cyc, hcyc);
  }
  return 0;
}
