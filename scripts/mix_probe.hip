// mix_probe.hip -- do full-rate (v_xor/v_add) and half-rate (v_alignbit /
// v_add3) VALU ops add up in issue cycles, or overlap?  8 waves/SIMD, 8
// independent chains per lane, random-looking per-lane data.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define ITERS 4096
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int P>
__global__ void __launch_bounds__(256) k(uint32_t* out, uint32_t seed) {
  uint32_t r[8];
  for (int i = 0; i < 8; i++) r[i] = (threadIdx.x + i * 7919u) * 0x9E3779B9u ^ seed;
  uint32_t v1 = threadIdx.x * 0x85EBCA6Bu + seed, v2 = threadIdx.x * 0xC2B2AE35u;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (P == 0) { asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(v1)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(v2)); }
      if (P == 1) { asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(r[i])); asm volatile("v_alignbit_b32 %0, %0, %0, 5" : "+v"(r[i])); }
      if (P == 2) { asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(v1)); asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(r[i])); }
      if (P == 3) { asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(v1)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(v2)); }
      if (P == 4) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(v1), "v"(v2)); }
      if (P == 5) { asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(r[i]) : "v"(v1), "v"(v2)); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(v1)); }
      if (P == 6) { asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(r[i])); asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(v1)); asm volatile("v_add_u32 %0, %0, %1" : "+v"(r[i]) : "v"(v2)); }
    }
  }
  uint32_t x = 0;
  for (int i = 0; i < 8; i++) x ^= r[i];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int P>
void run(const char* name, int ninstr_per_step, uint32_t* out) {
  const int W = 8, nblk = 256 * W;
  hipLaunchKernelGGL(k<P>, dim3(nblk), dim3(256), 0, 0, out, 1u);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  for (int rep = 0; rep < 5; rep++) hipLaunchKernelGGL(k<P>, dim3(nblk), dim3(256), 0, 0, out, 3u + rep);
  (void)hipEventRecord(b); (void)hipDeviceSynchronize();
  float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 5;
  double winst = (double)nblk * 4 * ITERS * 8 * ninstr_per_step;
  printf("%-28s %.3f ms  %.3f ns per wave-instr per SIMD\n", name, ms, ms * 1e6 / (winst / 1024));
}

int main() {
  uint32_t* out; CHK(hipMalloc(&out, 256 * 8 * 256 * 4));
  for (int rep = 0; rep < 2; rep++) {
    run<0>("xor,xor (fast,fast)", 2, out);
    run<1>("alignbit,alignbit (slow,slow)", 2, out);
    run<2>("xor,alignbit (fast,slow)", 2, out);
    run<3>("add,add (fast,fast)", 2, out);
    run<4>("add3 (slow)", 1, out);
    run<5>("add3,xor (slow,fast)", 2, out);
    run<6>("alignbit,xor,add (s,f,f)", 3, out);
  }
  return 0;
}
