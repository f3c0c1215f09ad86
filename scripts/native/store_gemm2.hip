// Store-pattern microbenchmark for the FF output GEMM's epilogue (C f32 [1000][14588], ldc 14592, 58 MB): one
// workgroup of 512 threads per 256x256 tile (4 x 57 = 228 tiles, one wave of tiles as in the 8-phase kernel),
// each wave writing 32 full 1-KiB tile rows with 16-B lane stores — the store stream of the GEMM's epilogue with
// no main loop and no LDS staging. Compared with a contiguous write of the same bytes, the same tiles written as
// bf16, and with the tile order/grid varied. Prints one line per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));
constexpr int M = 1000, N = 14588, LDC = 14592;

// ELEM = 4 (f32) or 2 (bf16); ROWMAJOR: wave w writes rows w, w+8, ... (interleaved) instead of a 32-row block
template <int ELEM, bool INTERLEAVE>
__global__ void __launch_bounds__(512) tile_kernel(char* out, int tiles_n) {
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)((long long)M * LDC * ELEM), 0x00020000);
  constexpr int LANE_COLS = 16 / ELEM;            // columns per 16-B lane store
  constexpr int ROW_PASSES = 256 / (64 * LANE_COLS);   // f32: 1 pass of 64 lanes covers 256 cols; bf16: 0.5
  for (int i = 0; i < 32; ++i) {
    const int r = INTERLEAVE ? i * 8 + wave : wave * 32 + i;
    const int row = tm * 256 + r;
    if constexpr (ELEM == 4) {
      const int col = tn * 256 + lane * 4;
      const int off = (row < M && col < N) ? (row * LDC + col) * 4 : 0x7ffffff0;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{(unsigned)row, (unsigned)col, 1u, 2u}, rs, off, 0, 0);
    } else {
      // bf16: a row is 32 lanes x 16 B; lanes 32-63 write the row 16 further down, 16 instructions per wave
      if (i >= 16) continue;
      const int rr = (INTERLEAVE ? i * 8 + wave : wave * 32 + i) + (lane >> 5) * (INTERLEAVE ? 128 : 16);
      const int row2 = tm * 256 + rr;
      const int col = tn * 256 + (lane & 31) * 8;
      const int off = (row2 < M && col < N) ? (row2 * LDC + col) * 2 : 0x7ffffff0;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{(unsigned)row2, (unsigned)col, 1u, 2u}, rs, off, 0, 0);
    }
    (void)ROW_PASSES;
  }
}

// Direct register -> global stores in the 8-phase kernel's transposed accumulator layout (no LDS staging):
// wave (wr, wc) owns rows wr*128 + i*16 + (lane & 15), columns wc*64 + j*16 + 4*(lane >> 4) .. +3 of the tile;
// one 16-B store per (i, j): an instruction writes 16 rows x 64 B
__global__ void __launch_bounds__(512) direct_kernel(char* out, int tiles_n) {
  const int tm = blockIdx.x / tiles_n, tn = blockIdx.x % tiles_n;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, wr = wave >> 2, wc = wave & 3;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)((long long)M * LDC * 4), 0x00020000);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = tm * 256 + wr * 128 + i * 16 + (lane & 15);
      const int col = tn * 256 + wc * 64 + j * 16 + 4 * (lane >> 4);
      const int off = (row < M && col < N) ? (row * LDC + col) * 4 : 0x7ffffff0;
      __builtin_amdgcn_raw_buffer_store_b128(u32x4_t{(unsigned)row, (unsigned)col, 1u, 2u}, rs, off, 0, 0);
    }
}

__global__ void __launch_bounds__(256) contig_kernel(u32x4_t* out, long long n16) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n16; i += (long long)gridDim.x * 256)
    out[i] = u32x4_t{(unsigned)i, 0u, 1u, 2u};
}

int main() {
  const long long bytes = (long long)M * LDC * 4;
  char* d = nullptr;
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
  const int tiles_n = (N + 255) / 256, tiles = 4 * tiles_n;
  const float tc = timeit([&] { hipLaunchKernelGGL(contig_kernel, dim3(2048), dim3(256), 0, 0, (u32x4_t*)d, bytes / 16); });
  printf("contiguous f32 58 MB: %.1f us  %.2f TB/s\n", tc, bytes / (tc * 1e-6) / 1e12);
  const float t1 = timeit([&] { hipLaunchKernelGGL((tile_kernel<4, false>), dim3(tiles), dim3(512), 0, 0, d, tiles_n); });
  printf("tiles f32 (wave = 32-row block): %.1f us  %.2f TB/s\n", t1, (double)M * N * 4 / (t1 * 1e-6) / 1e12);
  const float t2 = timeit([&] { hipLaunchKernelGGL((tile_kernel<4, true>), dim3(tiles), dim3(512), 0, 0, d, tiles_n); });
  printf("tiles f32 (waves interleaved by row): %.1f us  %.2f TB/s\n", t2, (double)M * N * 4 / (t2 * 1e-6) / 1e12);
  const float t3 = timeit([&] { hipLaunchKernelGGL((tile_kernel<2, false>), dim3(tiles), dim3(512), 0, 0, d, tiles_n); });
  printf("tiles bf16 (half the bytes, half the instructions): %.1f us  %.2f TB/s\n", t3, (double)M * N * 2 / (t3 * 1e-6) / 1e12);
  const float t4 = timeit([&] { hipLaunchKernelGGL(direct_kernel, dim3(tiles), dim3(512), 0, 0, d, tiles_n); });
  printf("tiles f32 direct from the MFMA layout (16 rows x 64 B per instruction): %.1f us  %.2f TB/s\n", t4,
         (double)M * N * 4 / (t4 * 1e-6) / 1e12);
  (void)hipFree(d);
  return 0;
}
