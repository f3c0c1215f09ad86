// MFMA-only power/clock microbenchmark (no memory traffic in the loop): the same number of bf16 MACs issued as
// v_mfma_f32_16x16x32_bf16 (8 K MACs per instruction) or v_mfma_f32_32x32x16_bf16 (16 K MACs per instruction,
// half the operand register reads per MAC), on random or zero operand bits. 4 waves per CU-quarter (one per
// SIMD per block, 2 blocks per CU), independent accumulator chains, 4 rotating operand sets.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

template <int BIG>
__global__ void __launch_bounds__(256) mfma_loop(const bf16x8_t* ops, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8_t a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = ops[(i * 2) * 64 + lane];
    b[i] = ops[(i * 2 + 1) * 64 + lane];
  }
  float s = 0.f;
  if constexpr (BIG) {
    f32x16_t c[4] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          c[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[(i + j) & 3], b[i], c[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += c[j][r];
  } else {
    f32x4_t c[8] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[(i + j) & 3], b[i], c[j], 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += c[j][r];
  }
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

static unsigned short f2bf(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  return (unsigned short)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 512, n_ops = 8 * 64 * 8;   // 8 operand regs x 64 lanes x 8 bf16
  std::vector<unsigned short> rnd(n_ops), zero(n_ops, 0);
  srand(1);
  for (auto& v : rnd) v = f2bf((float)rand() / (float)RAND_MAX * 2.f - 1.f);
  bf16x8_t *d_rnd, *d_zero;
  float* d_out;
  if (hipMalloc(&d_rnd, n_ops * 2) != hipSuccess || hipMalloc(&d_zero, n_ops * 2) != hipSuccess ||
      hipMalloc(&d_out, blocks * 256 * 4) != hipSuccess) return 1;
  (void)hipMemcpy(d_rnd, rnd.data(), n_ops * 2, hipMemcpyHostToDevice);
  (void)hipMemcpy(d_zero, zero.data(), n_ops * 2, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  // equal MACs: small = 32 MFMAs x 8 K per iteration, big = 16 MFMAs x 16 K per iteration
  const int iters = 4000;
  const double macs = (double)blocks * 4 * iters * 32 * 8192;
  for (int rep = 0; rep < 2; ++rep)
    for (int big = 0; big < 2; ++big)
      for (int z = 0; z < 2; ++z) {
        const bf16x8_t* src = z ? d_zero : d_rnd;
        auto launch = [&] {
          if (big) hipLaunchKernelGGL(mfma_loop<1>, dim3(blocks), dim3(256), 0, 0, src, d_out, iters);
          else hipLaunchKernelGGL(mfma_loop<0>, dim3(blocks), dim3(256), 0, 0, src, d_out, iters);
        };
        for (int i = 0; i < 3; ++i) launch();
        (void)hipEventRecord(e0);
        for (int i = 0; i < 10; ++i) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 10;
        printf("blocks %d rep %d %s %s: %.3f ms  %.0f TFLOP/s\n", blocks, rep, big ? "32x32x16" : "16x16x32", z ? "zeros " : "random",
               ms, 2 * macs / (ms * 1e-3) / 1e12);
      }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
