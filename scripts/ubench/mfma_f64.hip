// Micro-benchmark: v_mfma_f64_16x16x4_f64 throughput vs number of independent accumulator
// chains, one wave per SIMD on every CU; plus MFMA + independent f64 VALU co-issue.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int K, int VALU>
__global__ __launch_bounds__(256, 1) void kern(const double* in, double* out, int iters,
                                                unsigned long long* clk) {
  const int l = threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  double a = in[l & 63], b = in[(l + 7) & 63];
  d4 acc[K];
#pragma unroll
  for (int k = 0; k < K; ++k) acc[k] = (d4){0.0, 0.0, 0.0, 0.0};
  double v0 = a, v1 = b, v2 = a + b, v3 = a - b;
  for (int it = 0; it < iters; it += 32) {
#pragma unroll
    for (int u = 0; u < 32; ++u)
#pragma unroll
    for (int k = 0; k < K; ++k) {
      acc[k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[k], 0, 0, 0);
#pragma unroll
      for (int v = 0; v < VALU; ++v) {
        v0 = __builtin_fma(v0, a, b); v1 = __builtin_fma(v1, b, a);
        v2 = __builtin_fma(v2, a, v0); v3 = __builtin_fma(v3, b, v1);
      }
    }
  }
  double s = v0 + v1 + v2 + v3;
#pragma unroll
  for (int k = 0; k < K; ++k) s += acc[k][0] + acc[k][1] + acc[k][2] + acc[k][3];
  out[blockIdx.x * blockDim.x + l] = s;
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (l == 0) { clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }
}

template <int K, int VALU>
void run(const double* in, double* out, int cus, unsigned long long* clk) {
  const int iters = 131072 / K;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((kern<K, VALU>), dim3(cus), dim3(256), 0, 0, in, out, iters, clk);
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((kern<K, VALU>), dim3(cus), dim3(256), 0, 0, in, out, iters, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double mfmas = 5.0 * cus * 4 * (double)iters * K;   // per-SIMD instruction count x SIMDs
  const double tflops = mfmas * 2048 / (ms * 1e-3) / 1e12;
  unsigned long long h[2];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / (double)h[1] * 0.1;   // s_memrealtime ticks at 100 MHz
  printf("K=%d VALU_per_mfma=%d: %.3f ms  %.1f TFLOP/s (f64 MFMA)  in-kernel clock %.2f GHz  shader cycles/mfma %.1f\n", K,
         4 * VALU, ms, tflops, ghz, (double)h[0] / (iters * K));
}

int main() {
  int dev; hipGetDevice(&dev);
  hipDeviceProp_t p; hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount;
  double *in, *out;
  hipMalloc(&in, 64 * sizeof(double));
  hipMalloc(&out, cus * 256 * sizeof(double));
  unsigned long long* clk;
  hipMalloc(&clk, cus * 2 * sizeof(unsigned long long));
  double h[64]; for (int i = 0; i < 64; ++i) h[i] = 1.0 + 1e-3 * i;
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  printf("CUs=%d clock=%d kHz\n", cus, p.clockRate);
  run<1, 0>(in, out, cus, clk); run<2, 0>(in, out, cus, clk); run<4, 0>(in, out, cus, clk); run<8, 0>(in, out, cus, clk);
  run<2, 1>(in, out, cus, clk); run<2, 2>(in, out, cus, clk); run<4, 1>(in, out, cus, clk); run<4, 2>(in, out, cus, clk);
  run<4, 4>(in, out, cus, clk);
  return 0;
}
