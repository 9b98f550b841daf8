// Micro-benchmark: the LU panel's pivot-column loop (bo_lu.hip panel_columns) on one workgroup,
// clocks per column, with parts of the column step left out (ABL bits, see panel_columns).
//   hipcc -O3 --offload-arch=gfx950 -I include -I bayesopt_smart_amd/csrc scripts/ubench/lu_panel_ubench.hip
#include "bo_lu.hip"
#include <stdio.h>

template <int NW, int RPL, int ABL>
__global__ __launch_bounds__(512) void ub(const double* __restrict__ A, int R, int reps, long long* clk) {
  __shared__ StripLds L;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave >= NW) return;
  long long tot = 0;
  for (int it = 0; it < reps; ++it) {
    double v[RPL][LB];
#pragma unroll
    for (int r = 0; r < RPL; ++r) {
      const int o = wave * 64 * RPL + 64 * r + lane;
#pragma unroll
      for (int c = 0; c < LB; ++c) v[r][c] = o < R ? A[(long long)c * R + o] : 0.0;
    }
    __syncthreads();
    const long long t0 = clock64();
    const bool sing = panel_columns<NW, RPL, ABL>(L, v, (long long)wave * 64 * RPL, 64, 0, R, 0);
    __syncthreads();
    tot += clock64() - t0;
    double s = sing ? 1.0 : 0.0;
#pragma unroll
    for (int r = 0; r < RPL; ++r)
#pragma unroll
      for (int c = 0; c < LB; ++c) s += v[r][c];
    if (s == 12345.678) clk[1] = 1;                    // keep the results live
  }
  if (threadIdx.x == 0) clk[0] = tot;
}

template <int NW, int RPL, int ABL>
void run(const double* A, int R, long long* clk, const char* name) {
  const int reps = 20;
  hipLaunchKernelGGL((ub<NW, RPL, ABL>), dim3(1), dim3(512), 0, 0, A, R, reps, clk);
  hipLaunchKernelGGL((ub<NW, RPL, ABL>), dim3(1), dim3(512), 0, 0, A, R, reps, clk);
  long long h[2];
  (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  printf("NW %d RPL %d rows %4d abl %2d %-28s %6.0f clocks per column\n", NW, RPL, R, ABL, name,
         (double)h[0] / reps / LB);
}

int main() {
  const int R = 512;
  double* h = (double*)malloc(sizeof(double) * R * LB);
  unsigned s = 12345;
  for (int i = 0; i < R * LB; ++i) { s = s * 1664525u + 1013904223u; h[i] = (s >> 8) * (1.0 / 16777216.0) - 0.5; }
  double* A;
  long long* clk;
  (void)hipMalloc(&A, sizeof(double) * R * LB);
  (void)hipMalloc(&clk, 64);
  (void)hipMemcpy(A, h, sizeof(double) * R * LB, hipMemcpyHostToDevice);
#define ALL(NW, RPL, RR)                                              \
  run<NW, RPL, 0>(A, RR, clk, "library default");                     \
  run<NW, RPL, 512>(A, RR, clk, "row-branch update");                 \
  run<NW, RPL, 768>(A, RR, clk, "next search ahead of the update");   \
  run<NW, RPL, 520>(A, RR, clk, "no update");                         \
  run<NW, RPL, 513>(A, RR, clk, "no barrier");                        \
  run<NW, RPL, 575>(A, RR, clk, "all of them out");
  ALL(8, 1, 512)
  ALL(4, 2, 512)
  ALL(4, 1, 256)
  ALL(8, 2, 512)
  ALL(8, 4, 512)
  return 0;
}
