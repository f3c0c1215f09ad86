// Device hash table for exact group-by on 64-bit keys (execution/kernels.py group_ids). The reference groups
// records through C++ hash maps on the CPU (src/queryExecution aggregation processors, PDBMap inside pages);
// here one launch inserts a whole key column into an open-addressing table in HBM and records each row's slot:
//
//  * nsdb_hash_group_insert — linear probing over a power-of-two table (load factor <= 1/2). A probe first
//    reads the slot with a device-coherent load and only issues the 64-bit compare-and-swap when the slot is
//    empty, so a low-cardinality column (TPC-H flags, dates, nations: millions of rows on a handful of keys)
//    costs one coherent load per row instead of millions of atomics serialised on one address. The slots live
//    in the memory-side coherence domain (agent-scope atomics), which is what makes the table consistent
//    across the 8 XCDs' private L2s.
//  * the sentinel value (INT64_MIN) marks an empty slot; rows whose key IS the sentinel go to the extra slot
//    `cap`, whose key word the host initialises to the sentinel, so compaction treats it like any other slot.
//
// The host side (ops.hash_group_ids) compacts the occupied slots, sorts only the distinct keys and maps slot ->
// rank, so the result is exactly torch.unique(sorted=True, return_inverse=True) at O(n) + O(g log g).
#include <hip/hip_runtime.h>
#include <stdint.h>

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

__global__ __launch_bounds__(256) void hash_group_insert_kernel(const unsigned long long* __restrict__ keys,
                                                                long long n, unsigned long long* table,
                                                                unsigned long long mask, int* __restrict__ slot_of,
                                                                int* __restrict__ occ) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long k = keys[i];
  unsigned long long s;
  if (k == kEmpty) {
    s = mask + 1;                                   // the sentinel's own slot
  } else {
    s = mix64(k) & mask;
    // the table has >= 2x the rows' slots, so a probe always meets the key or an empty slot
    for (;;) {
      unsigned long long cur = __hip_atomic_load(table + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cur == kEmpty) {
        cur = kEmpty;
        __hip_atomic_compare_exchange_strong(table + s, &cur, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        // cur: the slot's value before the exchange (kEmpty when this row claimed it)
        if (cur == kEmpty) cur = k;
      }
      if (cur == k) break;
      s = (s + 1) & mask;
    }
  }
  slot_of[i] = (int)s;
  occ[s] = 1;                                       // same value from every row of the group
}

}  // namespace

extern "C" {

// keys: n int64 on the device; table: cap + 1 words (cap a power of two >= 2n) preset to INT64_MIN;
// occ: cap + 1 ints preset to 0; slot_of: n ints.
int nsdb_hash_group_insert(const void* keys, long long n, void* table, long long cap, int* slot_of, int* occ,
                           hipStream_t st) {
  if (n <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) != 0 || cap < 2 * n) return (int)hipErrorInvalidValue;
  const long long blocks = (n + 255) / 256;
  hipLaunchKernelGGL(hash_group_insert_kernel, dim3((unsigned)blocks), dim3(256), 0, st,
                     (const unsigned long long*)keys, n, (unsigned long long*)table,
                     (unsigned long long)(cap - 1), slot_of, occ);
  return (int)hipGetLastError();
}

}  // extern "C"
