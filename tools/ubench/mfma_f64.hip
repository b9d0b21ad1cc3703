// Microbenchmark + layout check for v_mfma_f64_16x16x4_f64 on gfx950 (design input for the
// GEMM-form drag loop).  Prints the measured layout check and TFLOP/s for
// MFMA f64 and v_fma_f64.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void k_layout(const double* A, const double* B, double* D) {
  const int l = threadIdx.x;
  const double a = A[(l & 15) * 4 + (l >> 4)];   // A[i=l&15][k=l>>4], A is 16x4 row-major
  const double b = B[(l >> 4) * 16 + (l & 15)];  // B[k=l>>4][j=l&15], B is 4x16 row-major
  d4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(((l >> 4) + 4 * r) * 16) + (l & 15)] = acc[r];   // row=(l>>4)+4r, col=l&15
}

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma_rate(double* out, int iters, double x) {
  d4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = d4{0, 0, 0, 0};
  double a = x + threadIdx.x, b = x - threadIdx.x;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  }
  double s = 0;
  for (int j = 0; j < NACC; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  if (s == 12345.678) out[0] = s;
}

__global__ __launch_bounds__(256) void k_fma_rate(double* out, int iters, double x) {
  double v[8];
  for (int j = 0; j < 8; ++j) v[j] = x + j + threadIdx.x;
  const double m = 1.0000001, c = 1e-9;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = fma(v[j], m, c);
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += v[j];
  if (s == 12345.678) out[0] = s;
}

int main() {
  // layout check with exact small integers, asymmetric B
  std::vector<double> A(64), B(64), D(256), R(256, 0.0);
  for (int i = 0; i < 16; ++i) for (int k = 0; k < 4; ++k) A[i * 4 + k] = i * 7 + k * 3 + 1;
  for (int k = 0; k < 4; ++k) for (int j = 0; j < 16; ++j) B[k * 16 + j] = k * 11 - j * 2 + 5;
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) for (int k = 0; k < 4; ++k) R[i * 16 + j] += A[i * 4 + k] * B[k * 16 + j];
  double *dA, *dB, *dD, *dO;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 2048); hipMalloc(&dO, 64);
  hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int e = 0; e < 256; ++e) bad += D[e] != R[e];
  printf("layout check: %d mismatches of 256\n", bad);

  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int grid = 256 * 8, iters = 4000;
  float ms;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma_rate<4>, dim3(grid), dim3(256), 0, 0, dO, iters, 1.0);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    double fl = (double)grid * 4 * iters * 4 * 2048.0;
    printf("mfma_f64_16x16x4 (4 acc/wave, %d waves): %.3f ms  %.1f TFLOP/s  %.1f cycles/MFMA/SIMD at 2.4 GHz\n", grid * 4, ms,
           fl / ms / 1e9, (ms * 1e-3 * 2.4e9) / ((double)grid * 4 * iters * 4 / 1024.0));
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma_rate<1>, dim3(grid), dim3(256), 0, 0, dO, iters, 1.0);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    fl = (double)grid * 4 * iters * 1 * 2048.0;
    printf("mfma_f64_16x16x4 (1 acc/wave, dependent chain): %.3f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_fma_rate, dim3(grid), dim3(256), 0, 0, dO, iters, 1.0);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    fl = (double)grid * 256 * iters * 8 * 2.0;
    printf("v_fma_f64 (8 chains/lane): %.3f ms  %.1f TFLOP/s\n", ms, fl / ms / 1e9);
  }
  return 0;
}
