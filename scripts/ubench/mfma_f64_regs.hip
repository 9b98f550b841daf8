// Micro-benchmark: v_mfma_f64_16x16x4_f64 rate with accumulators in VGPRs vs AGPRs and with
// one or two waves per SIMD (inline asm pins the register classes).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));

template <bool AGPR, int WPS>
__global__ __launch_bounds__(256 * WPS, WPS) void kern(const double* in, double* out, int iters) {
  const int l = threadIdx.x;
  double a = in[l & 63], b = in[(l + 7) & 63];
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (AGPR) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c0) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c1) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c2) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+a"(c3) : "v"(a), "v"(b));
      } else {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c2) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c3) : "v"(a), "v"(b));
      }
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(a));
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + l] = s[0] + s[1] + s[2] + s[3];
}

template <bool AGPR, int WPS>
void run(const double* in, double* out, int cus) {
  const int iters = 4096 / WPS;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((kern<AGPR, WPS>), dim3(cus), dim3(256 * WPS), 0, 0, in, out, iters);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((kern<AGPR, WPS>), dim3(cus), dim3(256 * WPS), 0, 0, in, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = 5.0 * cus * 4 * WPS * (double)iters * 32;
  printf("acc in %s, %d wave(s)/SIMD: %.3f ms  %.1f TFLOP/s  %.1f cyc/MFMA/SIMD @2.4GHz\n", AGPR ? "AGPR" : "VGPR",
         WPS, ms, mfmas * 2048 / (ms * 1e-3) / 1e12, ms * 1e-3 / 5 * 2.4e9 / (WPS * iters * 32.0));
}

int main() {
  int dev; (void)hipGetDevice(&dev);
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, dev);
  double *in, *out;
  (void)hipMalloc(&in, 64 * sizeof(double));
  (void)hipMalloc(&out, p.multiProcessorCount * 512 * sizeof(double));
  double h[64]; for (int i = 0; i < 64; ++i) h[i] = 1.0 + 1e-3 * i;
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  run<true, 1>(in, out, p.multiProcessorCount); run<false, 1>(in, out, p.multiProcessorCount);
  run<true, 2>(in, out, p.multiProcessorCount); run<false, 2>(in, out, p.multiProcessorCount);
  return 0;
}
