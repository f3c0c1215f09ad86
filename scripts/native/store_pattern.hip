// Store-pattern microbenchmark for the conv2d output (NCHW bf16 [100][64][106][106], 144 MB): each block walks
// row groups of R output rows; per group, wave w writes the R*OW-element run of planes oc = w + 4j (j < 16) as
// 8-byte pieces (the full-row conv kernel's store pattern, no compute). R = 4 is the production kernel's group.
// Compared with a plain contiguous 8-B-per-lane write of the same bytes. Prints one line per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
constexpr int N = 100, OC = 64, OH = 106, OW = 106;

__global__ void __launch_bounds__(256) groups_kernel(unsigned short* out, int R) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int gpi = (OH + R - 1) / R, ngroups = N * gpi;
  const long long OHW = (long long)OH * OW;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(N * OC * OHW * 2), 0x00020000);
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int n = g / gpi, oh0 = (g % gpi) * R;
    const int rows = min(R, OH - oh0), n4 = rows * OW / 4;
    const int base = (int)(((long long)n * OC * OHW + (long long)oh0 * OW) * 2);
    for (int j = 0; j < 16; ++j) {
      const int oc = wave + 4 * j;
      for (int q = lane; q < n4; q += 64)
        __builtin_amdgcn_raw_buffer_store_b64(u32x2_t{(unsigned)q, (unsigned)g},
                                              rs, base + (int)(oc * OHW * 2) + 8 * q, 0, 0);
    }
  }
}

__global__ void __launch_bounds__(256) contig_kernel(unsigned long long* out, long long n8) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) out[i] = i;
}

int main() {
  const long long bytes = (long long)N * OC * OH * OW * 2;
  unsigned short* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto timeit = [&](auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    float best = 1e9f;
    for (int r = 0; r < 5; ++r) {
      (void)hipEventRecord(e0);
      for (int i = 0; i < 20; ++i) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      best = ms / 20 < best ? ms / 20 : best;
    }
    return best * 1e3f;
  };
  const float tc = timeit([&] { hipLaunchKernelGGL(contig_kernel, dim3(2048), dim3(256), 0, 0, (unsigned long long*)d, bytes / 8); });
  printf("contiguous: %.1f us  %.2f TB/s\n", tc, bytes / (tc * 1e-6) / 1e12);
  for (int R : {2, 4, 8, 16, 32}) {
    for (int blocks : {256, 512}) {
      const float t = timeit([&] { hipLaunchKernelGGL(groups_kernel, dim3(blocks), dim3(256), 0, 0, d, R); });
      printf("groups R=%2d blocks=%d: %.1f us  %.2f TB/s\n", R, blocks, t, bytes / (t * 1e-6) / 1e12);
    }
  }
  (void)hipFree(d);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
