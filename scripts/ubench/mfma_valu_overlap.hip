// Micro-benchmark: does f64 VALU work of one wave overlap f64 MFMAs of another wave on the
// same SIMD?  2 waves per SIMD; wave parity selects MFMA-only / VALU-only / both.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));

// MODE 0: every wave MFMA; 1: every wave VALU f64 FMA; 2: even waves MFMA, odd waves VALU;
// 3: odd waves int32/LDS-address VALU (v_add_u32 chain), even MFMA
template <int MODE>
__global__ __launch_bounds__(512, 2) void kern(const double* in, double* out, int iters) {
  const int l = threadIdx.x, w = l >> 6;
  double a = in[l & 63], b = in[(l + 7) & 63];
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double v0 = a, v1 = b, v2 = a + b, v3 = a - b, v4 = a * 2, v5 = b * 2, v6 = a * 3, v7 = b * 3;
  int i0 = l, i1 = l * 3, i2 = l * 5, i3 = l * 7;
  const bool do_mfma = MODE == 0 || ((MODE == 2 || MODE == 3) && (w & 1) == 0);
  const bool do_valu = MODE == 1 || (MODE == 2 && (w & 1) == 1);
  const bool do_int = MODE == 3 && (w & 1) == 1;
  if (do_mfma) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c1) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c2) : "v"(a), "v"(b));
        asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(c3) : "v"(a), "v"(b));
      }
    }
  }
  if (do_valu) {   // 32 MFMAs' worth of time at 1 f64 FMA per 4 cycles would be 32*65/4 = 520 FMAs
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 64; ++u) {
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v0) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v1) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v2) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v3) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v4) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v5) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v6) : "v"(a), "v"(b));
        asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v7) : "v"(a), "v"(b));
      }
    }
  }
  if (do_int) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int u = 0; u < 128; ++u) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(i0) : "v"(i1));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(i1) : "v"(i2));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(i2) : "v"(i3));
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(i3) : "v"(i0));
      }
    }
  }
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" : "+v"(a));
  d4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * blockDim.x + l] = s[0] + s[1] + s[2] + s[3] + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + i0 + i1 + i2 + i3;
}

template <int MODE>
void run(const double* in, double* out, int cus, const char* name) {
  const int iters = 2048;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  hipLaunchKernelGGL((kern<MODE>), dim3(cus), dim3(512), 0, 0, in, out, iters);
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((kern<MODE>), dim3(cus), dim3(512), 0, 0, in, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  printf("%-40s %.3f ms per launch\n", name, ms / 5);
}

int main() {
  int dev; (void)hipGetDevice(&dev);
  hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, dev);
  double *in, *out;
  (void)hipMalloc(&in, 64 * sizeof(double));
  (void)hipMalloc(&out, p.multiProcessorCount * 512 * sizeof(double));
  double h[64]; for (int i = 0; i < 64; ++i) h[i] = 1.0 + 1e-6 * i;
  (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const int c = p.multiProcessorCount;
  run<0>(in, out, c, "all waves MFMA (2/SIMD)");
  run<1>(in, out, c, "all waves f64 FMA (2/SIMD)");
  run<2>(in, out, c, "even MFMA + odd f64 FMA");
  run<3>(in, out, c, "even MFMA + odd int32 add");
  return 0;
}
