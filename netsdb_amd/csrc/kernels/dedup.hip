// Model-deduplication kernels (reference: src/deduplication — TensorBlockIndex matching of identical
// FFMatrixBlocks; model-inference/deduplication/indexing). One HBM pass per operation:
//  * block_hash    — order-aware 64-bit content hash of every fixed-size block:
//                    h(block) = mix64( sum_j mix64(w_j * 0x100000001B3 + j) )  over the block's 32-bit
//                    words w_j (wrapping u64 arithmetic). The kernel writes the per-(block, split) partial
//                    sums; the host-side wrapper adds the S partials and applies the final mix (both
//                    wrap mod 2^64, so the result is bit-identical to the torch reference on any device).
//  * block_maxdiff — max |pool[cand[b]] - blks[b]| per block without gathering the candidate blocks
//                    (content verification of a hash hit); per-(block, split) partials again.
//  * block_simcount — approximate-dedup similarity (indexing/deduplicator.py): the number of elements of
//                    candidate pool[cand[b]] within fp of ONE query block, over the valid h x w corner of
//                    the br x bc blocks (padded edge blocks compare only their real part).
// Blocks are streamed with 16-B loads; S workgroups per block so a launch has >> 256 workgroups even
// for a few hundred 2-MB word2vec blocks.
#include "common.h"
#include <algorithm>

namespace nsdb {

typedef unsigned int u32x4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned long long mix64u(unsigned long long x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// data: nblocks x words (u32), words % 4 == 0, 16-B aligned. grid (S, nblocks), 256 threads.
__global__ void __launch_bounds__(256) block_hash_kernel(const unsigned int* __restrict__ data, long long words,
                                                         unsigned long long* __restrict__ partial) {
  const int b = blockIdx.y, s = blockIdx.x, S = gridDim.x;
  const long long q = words / 4;                          // uint4 per block
  const long long per = (q + S - 1) / S;
  const long long q0 = (long long)s * per, q1 = q0 + per < q ? q0 + per : q;
  const u32x4v* p = reinterpret_cast<const u32x4v*>(data + (long long)b * words);
  unsigned long long acc = 0;
  for (long long i = q0 + threadIdx.x; i < q1; i += blockDim.x) {
    const u32x4v v = __builtin_nontemporal_load(p + i);
    const unsigned long long j = (unsigned long long)i * 4;
    acc += mix64u((unsigned long long)v.x * 0x100000001B3ull + j);
    acc += mix64u((unsigned long long)v.y * 0x100000001B3ull + j + 1);
    acc += mix64u((unsigned long long)v.z * 0x100000001B3ull + j + 2);
    acc += mix64u((unsigned long long)v.w * 0x100000001B3ull + j + 3);
  }
  // wave reduce (64 lanes) then across the 4 waves through LDS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  __shared__ unsigned long long red[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[(long long)b * S + s] = red[0] + red[1] + red[2] + red[3];
}

template <typename T> __device__ __forceinline__ float to_f(T v);
template <> __device__ __forceinline__ float to_f<float>(float v) { return v; }
template <> __device__ __forceinline__ float to_f<unsigned short>(unsigned short v) { return bf16_to_f32(v); }

// pool: [*, elems] T, cand: [nblocks] i64 (valid rows of pool), blks: [nblocks, elems] T.
// grid (S, nblocks); elems * sizeof(T) % 16 == 0.
template <typename T>
__global__ void __launch_bounds__(256) block_maxdiff_kernel(const T* __restrict__ pool, const long long* __restrict__ cand,
                                                            const T* __restrict__ blks, long long elems,
                                                            float* __restrict__ partial) {
  constexpr int V = 16 / sizeof(T);
  const int b = blockIdx.y, s = blockIdx.x, S = gridDim.x;
  const long long q = elems / V, per = (q + S - 1) / S;
  const long long q0 = (long long)s * per, q1 = q0 + per < q ? q0 + per : q;
  const u32x4v* pa = reinterpret_cast<const u32x4v*>(pool + cand[b] * elems);
  const u32x4v* pb = reinterpret_cast<const u32x4v*>(blks + (long long)b * elems);
  float m = 0.f;
  for (long long i = q0 + threadIdx.x; i < q1; i += blockDim.x) {
    u32x4v va = pa[i], vb = __builtin_nontemporal_load(pb + i);
    const T* ea = reinterpret_cast<const T*>(&va);
    const T* eb = reinterpret_cast<const T*>(&vb);
#pragma unroll
    for (int k = 0; k < V; ++k) m = fmaxf(m, fabsf(to_f<T>(ea[k]) - to_f<T>(eb[k])));
  }
  m = wave_reduce_max(m);
  __shared__ float red[4];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) partial[(long long)b * S + s] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// pool: [*, elems] T, cand: [nblocks] i64, query: [elems] T; elems = br * bc; counts the elements e of the
// h x w corner (row e / bc < h, column e % bc < w) with |pool[cand[b]][e] - query[e]| <= fp.
// grid (S, nblocks); elems * sizeof(T) % 16 == 0.
template <typename T>
__global__ void __launch_bounds__(256) block_simcount_kernel(const T* __restrict__ pool, const long long* __restrict__ cand,
                                                             const T* __restrict__ query, long long elems, int bc,
                                                             long long valid_end, int w, float fp,
                                                             unsigned* __restrict__ partial) {
  constexpr int V = 16 / sizeof(T);
  const int b = blockIdx.y, s = blockIdx.x, S = gridDim.x;
  const long long q = elems / V, per = (q + S - 1) / S;
  const long long q0 = (long long)s * per, q1 = q0 + per < q ? q0 + per : q;
  const u32x4v* pa = reinterpret_cast<const u32x4v*>(pool + cand[b] * elems);
  const u32x4v* pq = reinterpret_cast<const u32x4v*>(query);
  unsigned cnt = 0;
  for (long long i = q0 + threadIdx.x; i < q1; i += blockDim.x) {
    const u32x4v va = __builtin_nontemporal_load(pa + i), vq = pq[i];
    const T* ea = reinterpret_cast<const T*>(&va);
    const T* eq = reinterpret_cast<const T*>(&vq);
    const long long e0 = i * V;
    int col = (int)(e0 % bc);
#pragma unroll
    for (int k = 0; k < V; ++k) {
      const bool valid = (e0 + k) < valid_end && col < w;
      cnt += (valid && fabsf(to_f<T>(ea[k]) - to_f<T>(eq[k])) <= fp) ? 1u : 0u;
      col = col + 1 == bc ? 0 : col + 1;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  __shared__ unsigned red[4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wv] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) partial[(long long)b * S + s] = red[0] + red[1] + red[2] + red[3];
}

}  // namespace nsdb

extern "C" {

// splits per block: enough workgroups to cover the chip (>= 2048 total) but >= 64 KiB per workgroup
int nsdb_dedup_splits(long long nblocks, long long bytes_per_block) {
  long long s = (2048 + nblocks - 1) / std::max(1LL, nblocks);
  s = std::min(s, std::max(1LL, bytes_per_block / 65536));
  return (int)std::max(1LL, std::min(s, 1024LL));
}

int nsdb_block_hash(const void* data, long long nblocks, long long words, int S, unsigned long long* partial,
                    hipStream_t st) {
  if (nblocks <= 0) return 0;
  if (words % 4 || nblocks > 65535 || S <= 0) return -1;
  hipLaunchKernelGGL(nsdb::block_hash_kernel, dim3(S, (unsigned)nblocks), dim3(256), 0, st,
                     (const unsigned int*)data, words, partial);
  return (int)hipGetLastError();
}

int nsdb_block_maxdiff(const void* pool, const long long* cand, const void* blks, long long nblocks, long long elems,
                       int is_f32, int S, float* partial, hipStream_t st) {
  if (nblocks <= 0) return 0;
  if ((elems * (is_f32 ? 4 : 2)) % 16 || nblocks > 65535 || S <= 0) return -1;
  if (is_f32)
    hipLaunchKernelGGL(nsdb::block_maxdiff_kernel<float>, dim3(S, (unsigned)nblocks), dim3(256), 0, st,
                       (const float*)pool, cand, (const float*)blks, elems, partial);
  else
    hipLaunchKernelGGL(nsdb::block_maxdiff_kernel<unsigned short>, dim3(S, (unsigned)nblocks), dim3(256), 0, st,
                       (const unsigned short*)pool, cand, (const unsigned short*)blks, elems, partial);
  return (int)hipGetLastError();
}

int nsdb_block_simcount(const void* pool, const long long* cand, const void* query, long long nblocks, long long elems,
                        int bc, int h, int w, float fp, int is_f32, int S, unsigned* partial, hipStream_t st) {
  if (nblocks <= 0) return 0;
  if ((elems * (is_f32 ? 4 : 2)) % 16 || nblocks > 65535 || S <= 0 || bc <= 0) return -1;
  const long long valid_end = (long long)h * bc;
  if (is_f32)
    hipLaunchKernelGGL(nsdb::block_simcount_kernel<float>, dim3(S, (unsigned)nblocks), dim3(256), 0, st,
                       (const float*)pool, cand, (const float*)query, elems, bc, valid_end, w, fp, partial);
  else
    hipLaunchKernelGGL(nsdb::block_simcount_kernel<unsigned short>, dim3(S, (unsigned)nblocks), dim3(256), 0, st,
                       (const unsigned short*)pool, cand, (const unsigned short*)query, elems, bc, valid_end, w, fp,
                       partial);
  return (int)hipGetLastError();
}

}  // extern "C"
