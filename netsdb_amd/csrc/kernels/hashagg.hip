// Device hash table for exact group-by on 64-bit keys (execution/kernels.py group_ids). The reference groups
// records through C++ hash maps on the CPU (src/queryExecution aggregation processors, PDBMap inside pages);
// here one launch inserts a whole key column into an open-addressing table in HBM and records each row's slot:
//
//  * nsdb_hash_group_insert — linear probing over a power-of-two table (load factor <= 1/2). Each workgroup
//    keeps a 1024-entry LDS cache of key -> slot, so a low-cardinality column (TPC-H flags, dates, nations:
//    millions of rows on a handful of keys) resolves almost every row in LDS instead of sending millions of
//    accesses to the same few table words. A global probe reads the slot with a device-coherent load and only
//    issues the 64-bit compare-and-swap when the slot is empty; the slots live in the memory-side coherence
//    domain (agent-scope atomics), which is what makes the table consistent across the 8 XCDs' private L2s.
//    A filled slot never changes, so a stale read can only be "empty", which the CAS then corrects.
//  * the sentinel value (INT64_MIN) marks an empty slot; rows whose key IS the sentinel go to the extra slot
//    `cap`, whose key word the host initialises to the sentinel, so compaction treats it like any other slot.
//
// The host side (ops.hash_group_ids) compacts the occupied slots, sorts only the distinct keys and maps slot ->
// rank, so the result is exactly torch.unique(sorted=True, return_inverse=True) at O(n) + O(g log g).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace {

constexpr unsigned long long kEmpty = 0x8000000000000000ull;

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

constexpr int kCache = 1024;   // per-workgroup LDS cache of key -> slot (12 KiB)
constexpr int kCacheProbe = 4;

// Global probe: the slot holding k after this call (claimed by this row if it was empty).
__device__ __forceinline__ unsigned long long probe_global(unsigned long long* table, unsigned long long mask,
                                                           unsigned long long k, unsigned long long h,
                                                           bool& claimed) {
  unsigned long long s = h & mask;
  claimed = false;
  // the table has >= 2x the rows' slots, so a probe always meets the key or an empty slot
  for (;;) {
    unsigned long long cur = __hip_atomic_load(table + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == kEmpty) {
      // cur: the slot's value before the exchange (kEmpty when this row claimed it)
      __hip_atomic_compare_exchange_strong(table + s, &cur, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      if (cur == kEmpty) {
        claimed = true;
        return s;
      }
    }
    if (cur == k) return s;
    s = (s + 1) & mask;
  }
}

// Grid-stride over the rows. A workgroup first looks a key up in its LDS cache (a low-cardinality column
// resolves almost every row there, so the hot table slots are not hammered from every CU), and on a miss
// probes the global table and caches the slot. A slot is written to occ by the one row that claimed it.
__global__ __launch_bounds__(256) void hash_group_insert_kernel(const unsigned long long* __restrict__ keys,
                                                                long long n, unsigned long long* table,
                                                                unsigned long long mask, int* __restrict__ slot_of,
                                                                int* __restrict__ occ) {
  __shared__ unsigned long long ckey[kCache];
  __shared__ int cslot[kCache];
  for (int i = threadIdx.x; i < kCache; i += blockDim.x) {
    ckey[i] = kEmpty;
    cslot[i] = -1;
  }
  __syncthreads();
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    const unsigned long long k = keys[i];
    if (k == kEmpty) {                              // the sentinel's own slot
      slot_of[i] = (int)(mask + 1);
      occ[mask + 1] = 1;
      continue;
    }
    const unsigned long long h = mix64(k);
    int s = -1, free_c = -1;
#pragma unroll
    for (int j = 0; j < kCacheProbe; ++j) {
      const int c = (int)((h >> 40) + j) & (kCache - 1);
      const unsigned long long ck = ckey[c];
      if (ck == k) {
        s = cslot[c];                               // -1 while the inserting lane has not written it yet
        break;
      }
      if (ck == kEmpty) {
        free_c = c;
        break;
      }
    }
    if (s < 0) {
      bool claimed;
      s = (int)probe_global(table, mask, k, h, claimed);
      if (claimed) occ[s] = 1;
      if (free_c >= 0) {
        unsigned long long e = kEmpty;
        if (__hip_atomic_compare_exchange_strong(ckey + free_c, &e, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP))
          __hip_atomic_store(cslot + free_c, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    slot_of[i] = s;
  }
}

}  // namespace

extern "C" {

// keys: n int64 on the device; table: cap + 1 words (cap a power of two >= 2n) preset to INT64_MIN;
// occ: cap + 1 ints preset to 0; slot_of: n ints.
int nsdb_hash_group_insert(const void* keys, long long n, void* table, long long cap, int* slot_of, int* occ,
                           hipStream_t st) {
  if (n <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) != 0 || cap < 2 * n) return (int)hipErrorInvalidValue;
  const long long blocks = std::min<long long>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(hash_group_insert_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const unsigned long long*)keys, n, (unsigned long long*)table,
                     (unsigned long long)(cap - 1), slot_of, occ);
  return (int)hipGetLastError();
}

}  // extern "C"
