// Device relational operators: hash aggregation, hash join (build / probe / expand) and the partition+pack
// permutation of the shuffle sink. Reference: netsDB aggregates through C++ hash maps per page
// (src/queryExecution/headers/AggregationProcessor.h:16, CombinerProcessor, PartitionedHashSet.h:20), joins
// through JoinMap / PairArray (src/lambdas/headers/JoinTuple.h:434 JoinProbe, :1243 PartitionedJoinSink,
// HashSink.h:14) and partitions with HashPartitionSink. Here each is a few device launches over whole columns.
//
// Hash aggregation of n rows (one int64 key per row; multi-column keys are packed or hashed by the caller,
// execution/kernels.py) with F value columns (8-byte: double or int64; op sum / min / max; a row count always):
//
//  * agg_sample: ONE workgroup hashes 4096 evenly spaced rows into an LDS table with counts and writes the Chao1
//    estimate of the distinct keys into a device word. Every later kernel reads it and returns at once when its
//    path is not the one taken, so the choice costs no host round trip (the only host read of the whole
//    aggregation is the final group count).
//  * LOW path (few groups): agg_low — each workgroup pre-aggregates its rows in an LDS hash table (claim by LDS
//    CAS, f64 / u64 LDS atomics; rows loaded four per thread, the next batch in flight while one is inserted),
//    rows whose key does not fit go straight to a small global table, and at the end each workgroup flushes its
//    LDS entries ONCE into the global table (agent-scope atomics): one global atomic per (workgroup, key), not per
//    row. If the global table overflows (the sample under-estimated the groups) a device flag routes the work to:
//  * PART path (many groups): 256 level-1 buckets by the top hash bits (agg_hist: per-workgroup LDS histograms;
//    scan_rows / scan_tot: block scans; agg_scatter: tile-staged counting sort in LDS, so each bucket's rows leave
//    as one coalesced run per tile), then agg_bucket: workgroup b owns bucket b whole. If its share of the
//    estimate fits the LDS table it aggregates the bucket there and writes the groups straight to the dense
//    output (their keys occur in no other bucket); otherwise it splits the bucket again by the next hash bits
//    (its own histogram + staged scatter into a second buffer) and aggregates four sub-buckets at a time in four
//    quarter tables. Rows whose LDS probe window is full go to a small overflow table (agg_emit copies those).
//    No global atomic per row anywhere: per-row atomics on global memory execute at the memory side.
//  * agg_fix_inv turns per-row global-slot references into dense group ids (only when the caller wants the
//    per-row inverse); want_first = 0 drops the row ids from the partition passes altogether.
// Dense group ids come from one device counter bumped once per emitted run, so there is no compaction pass over
// the tables and no nonzero()/sort.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace nsdb_rel {

typedef unsigned long long u64;
typedef long long i64;
constexpr u64 kEmpty = 0x8000000000000000ull;   // empty-slot marker (rows whose key is this value get a slot of their own)

__device__ __forceinline__ u64 mix64(u64 x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  return x;
}

// ---------------------------------------------------------------- accumulators (8-byte words)
enum AggOp : int { OP_SUM = 0, OP_MIN = 1, OP_MAX = 2 };

// order-preserving u64 image of a double / int64, so min / max are unsigned integer atomics
__device__ __forceinline__ u64 ord_of(double v) {
  const u64 b = __double_as_longlong(v);
  return (b & kEmpty) ? ~b : (b | kEmpty);
}
__device__ __forceinline__ u64 ord_of(i64 v) { return (u64)v ^ kEmpty; }
__device__ __forceinline__ double ord_to_f64(u64 o) {
  return __longlong_as_double((o & kEmpty) ? (i64)(o & ~kEmpty) : (i64)~o);
}
__device__ __forceinline__ i64 ord_to_i64(u64 o) { return (i64)(o ^ kEmpty); }

template <typename VT, int OP>
__host__ __device__ __forceinline__ u64 acc_identity() {
  if constexpr (OP == OP_MIN) return ~0ull;
  else if constexpr (OP == OP_MAX) return 0ull;
  else return 0ull;   // +0.0 and integer 0 are both all-zero bits
}

template <typename VT, int OP, int SCOPE>
__device__ __forceinline__ void acc_add(u64* p, VT v) {
  if constexpr (OP == OP_SUM) {
    if constexpr (sizeof(VT) == 8 && __is_same(VT, double))
      __hip_atomic_fetch_add(reinterpret_cast<double*>(p), v, __ATOMIC_RELAXED, SCOPE);
    else
      __hip_atomic_fetch_add(p, (u64)v, __ATOMIC_RELAXED, SCOPE);
  } else if constexpr (OP == OP_MIN) {
    __hip_atomic_fetch_min(p, ord_of(v), __ATOMIC_RELAXED, SCOPE);
  } else {
    __hip_atomic_fetch_max(p, ord_of(v), __ATOMIC_RELAXED, SCOPE);
  }
}

// merge an already-accumulated word (an LDS partial) into a global accumulator
template <typename VT, int OP>
__device__ __forceinline__ void acc_merge_global(u64* p, u64 w) {
  if constexpr (OP == OP_SUM) {
    if constexpr (__is_same(VT, double))
      __hip_atomic_fetch_add(reinterpret_cast<double*>(p), __longlong_as_double((i64)w), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    else
      __hip_atomic_fetch_add(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (OP == OP_MIN) {
    __hip_atomic_fetch_min(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    __hip_atomic_fetch_max(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// accumulator word -> output value bits
template <typename VT, int OP>
__device__ __forceinline__ u64 acc_out(u64 w) {
  if constexpr (OP == OP_SUM) return w;
  else if constexpr (__is_same(VT, double)) return (u64)__double_as_longlong(ord_to_f64(w));
  else return (u64)ord_to_i64(w);
}

// ---------------------------------------------------------------- shared state of one aggregation
// One int64 word array zeroed by the host per call.
struct AggMeta {
  i64 est;            // distinct keys in the sample
  i64 low;            // 1: the sample says few groups -> LOW path first
  i64 ng_low;         // groups created by the LOW path
  i64 ng_part;        // groups created by the PART path
  i64 fail_low;       // LOW global table overflowed -> PART path runs
  i64 fail_part;      // PART global table overflowed -> the caller falls back
  i64 sentinel_low;   // the kEmpty key's group was created (LOW / PART)
  i64 sentinel_part;
  i64 occ_low;        // slots claimed in the LOW global table (its fill, apart from the group count)
  i64 occ_part;       // slots claimed in the PART overflow table
  i64 lowp;           // key partitions of the MID path (low == 2)
  i64 pad[5];
};

struct GTable {                     // open-addressing global table: cap slots + one slot (cap) for the kEmpty key
  u64* key;                         // [cap + 1], preset kEmpty
  u64* acc;                         // [(cap + 1) * F], preset to the op identity
  u64* cnt;                         // [cap + 1], preset 0
  u64* rmin;                        // [cap + 1], preset ~0: smallest row index of the group
  i64* gid_of_slot;                 // [cap + 1]
  u64 mask;                         // cap - 1
  i64* occ;                         // claimed-slot counter (AggMeta::occ_*)
};

struct AggOut {
  i64* reps;        // [n] dense group keys
  u64* aggs;        // [n * F]
  i64* cnt;         // [n]
  i64* slot_of_gid; // [n] (unused region of the output buffer: kept so the bindings' offsets stay put)
  i64* first;       // [n] smallest row index of each group (its representative row)
  i64* inv;         // [n] or null
};

__device__ __forceinline__ bool take_low(const AggMeta* m) { return m->low != 0; }
__device__ __forceinline__ bool take_part(const AggMeta* m) { return m->low == 0 || m->fail_low != 0; }

constexpr int kLdsProbe = 64;     // LDS probe window: a row whose window is full goes to the global table
constexpr u64 kGlobalProbe = 1024;  // global probe window: beyond it the table counts as full (fail flag)

// Global slot of key k (created on first sight). Returns -1 when the table is full (fail flag set).
__device__ __forceinline__ i64 gtable_slot(GTable t, u64 k, i64* ngroups, i64* sentinel, i64* fail, AggOut o) {
  if (k == kEmpty) {
    const u64 s = t.mask + 1;
    i64 exp0 = 0;
    if (__hip_atomic_compare_exchange_strong(sentinel, &exp0, (i64)1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT)) {
      const i64 gid = __hip_atomic_fetch_add(ngroups, (i64)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t.gid_of_slot[s] = gid;
      o.reps[gid] = (i64)k;
    }
    return (i64)s;
  }
  u64 s = mix64(k) & t.mask;
  const u64 window = t.mask < kGlobalProbe ? t.mask + 1 : kGlobalProbe;
  for (u64 p = 0; p < window; ++p) {
    u64 cur = __hip_atomic_load(t.key + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == kEmpty) {
      if (__hip_atomic_compare_exchange_strong(t.key + s, &cur, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        const i64 gid = __hip_atomic_fetch_add(ngroups, (i64)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the table more than half full: probe windows grow long -> give up on this table
        const i64 used = __hip_atomic_fetch_add(t.occ, (i64)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((u64)used > (t.mask >> 1)) __hip_atomic_store(fail, (i64)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t.gid_of_slot[s] = gid;
        o.reps[gid] = (i64)k;
        return (i64)s;
      }
      // cur now holds the key another row claimed this slot with
    }
    if (cur == k) return (i64)s;
    s = (s + 1) & t.mask;
  }
  __hip_atomic_store(fail, (i64)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return -1;
}

// LDS table of one workgroup: key words, F accumulators, counts, and the global slot / group id each entry
// ends up in. Laid out as [key | acc | cnt | ref] in one dynamic LDS array.
struct LTable {
  u64* key;
  u64* acc;
  unsigned* cnt;
  int* ref;          // dense group id, or -(global slot + 1) (rows < 2^31)
  unsigned* rmin;    // smallest row index of the entry's rows
  int cap;   // power of two
};

// [key | acc | ref | rmin | cnt]: 20 + 8F bytes per entry
__device__ __forceinline__ LTable ltable_at(char* base, int cap, int F) {
  LTable t;
  t.key = reinterpret_cast<u64*>(base);
  t.acc = t.key + cap;
  t.ref = reinterpret_cast<int*>(t.acc + (size_t)cap * F);
  t.rmin = reinterpret_cast<unsigned*>(t.ref + cap);
  t.cnt = t.rmin + cap;
  t.cap = cap;
  return t;
}

template <typename VT, int OP>
__device__ __forceinline__ void ltable_clear(LTable t, int F, int lt = -1, int gs = 0) {
  if (lt < 0) {
    lt = threadIdx.x;
    gs = blockDim.x;
  }
  for (int i = lt; i < t.cap; i += gs) {
    t.key[i] = kEmpty;
    t.cnt[i] = 0;
    t.ref[i] = 0;
    t.rmin[i] = ~0u;
  }
  for (int i = lt; i < t.cap * F; i += gs) t.acc[i] = acc_identity<VT, OP>();
}

// LDS slot of k (inserted if absent), or -1 if its probe window is full.
__device__ __forceinline__ int ltable_slot(LTable t, u64 k, u64 h) {
  const int mask = t.cap - 1;
  int s = (int)(h & (u64)mask);
  const int window = t.cap < kLdsProbe ? t.cap : kLdsProbe;
  for (int p = 0; p < window; ++p) {
    u64 cur = t.key[s];
    if (cur == kEmpty) {
      u64 e = kEmpty;
      __hip_atomic_compare_exchange_strong(t.key + s, &e, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
      cur = e;   // kEmpty if this row claimed the slot, else the key that did
      if (cur == kEmpty) return s;
    }
    if (cur == k) return s;
    s = (s + 1) & mask;
  }
  return -1;
}

// lookup only (the key is known to be present when this is called for a row that hit the LDS table)
__device__ __forceinline__ int ltable_find(LTable t, u64 k, u64 h) {
  const int mask = t.cap - 1;
  int s = (int)(h & (u64)mask);
  const int window = t.cap < kLdsProbe ? t.cap : kLdsProbe;
  for (int p = 0; p < window; ++p) {
    const u64 cur = t.key[s];
    if (cur == k) return s;
    if (cur == kEmpty) return -1;
    s = (s + 1) & mask;
  }
  return -1;
}

template <typename VT, int OP>
__device__ __forceinline__ void row_into_global(GTable g, u64 k, const VT* v, int F, i64 cs, i64* ngroups,
                                                i64* sentinel, i64* fail, AggOut o, i64 row) {
  const i64 s = gtable_slot(g, k, ngroups, sentinel, fail, o);
  if (s < 0) return;
  for (int f = 0; f < F; ++f) acc_add<VT, OP, __HIP_MEMORY_SCOPE_AGENT>(g.acc + s * F + f, v[f * cs]);
  __hip_atomic_fetch_add(g.cnt + s, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_min(g.rmin + s, (u64)row, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (o.inv) o.inv[row] = -(s + 1);
}

// ---------------------------------------------------------------- sample estimate
// One workgroup hashes 4096 evenly spaced rows into an LDS table with per-key counts and writes the Chao1
// estimate of the distinct keys, d + f1^2 / (2 f2) (f1 / f2: keys seen once / twice in the sample; exact d when
// every row was sampled), clamped to [d, n]. The PART path sizes its sub-partitions from it.
constexpr int kSample = 4096;
// MID path: at most this many key partitions. Every workgroup of a row group reads all of its rows' keys through its
// own CU, so the per-CU load stream grows with P: measured (profiles/r5_relops) 16 M rows, 10 k keys at P = 5 took
// 0.65 ms against the PART path's 0.47, so MID stops at P = 3 (~6 k groups).
constexpr int kMidPMax = 3;

// The sampled rows' keys into sbuf[4096]: the random reads spread over 64 workgroups (one CU's outstanding-miss
// budget made a single-workgroup sample latency-bound).
__global__ __launch_bounds__(64) void agg_sample_gather_kernel(const u64* __restrict__ keys, i64 n,
                                                               u64* __restrict__ sbuf) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const int ns = (int)std::min<i64>(kSample, n);
  const i64 r = (n <= kSample) ? i : ((i64)i * n) / kSample;   // n < 2^31: no overflow
  sbuf[i] = i < ns ? keys[r] : kEmpty;
}

__global__ __launch_bounds__(1024) void agg_sample_kernel(const u64* __restrict__ sbuf, i64 n, int low_thr,
                                                          int mid_keys, AggMeta* meta) {
  constexpr int S = kSample, CAP = 8192;
  __shared__ u64 tab[CAP];
  __shared__ unsigned tcnt[CAP];
  __shared__ unsigned fsum[3];
  for (int i = threadIdx.x; i < CAP; i += blockDim.x) {
    tab[i] = kEmpty;
    tcnt[i] = 0;
  }
  if (threadIdx.x < 3) fsum[threadIdx.x] = 0;
  __syncthreads();
  u64 kk[S / 1024];
#pragma unroll
  for (int j = 0; j < S / 1024; ++j) kk[j] = sbuf[threadIdx.x + j * 1024];   // contiguous, gathered before
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < S / 1024; ++j) {
    const u64 k = kk[j];
    const bool active = k != kEmpty;
    int s = -1;
    if (active) {
      s = (int)(mix64(k) & (CAP - 1));
      for (;;) {
        u64 e = tab[s];   // plain read first: a key already present costs no atomic
        if (e == kEmpty)
          __hip_atomic_compare_exchange_strong(tab + s, &e, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
        if (e == kEmpty || e == k) break;
        s = (s + 1) & (CAP - 1);
      }
    }
    // hot keys: one LDS add per distinct slot for up to 4 slots of the wave (a handful of keys would serialise
    // 64 lanes on one word); the remaining lanes (many distinct keys) add one by one
    u64 todo = __ballot(active);
    for (int r = 0; r < 4 && todo; ++r) {
      const int leader = __ffsll((long long)todo) - 1;
      const int ls = __shfl(s, leader, 64);
      const u64 m = __ballot(active && s == ls);
      if (lane == leader) atomicAdd(tcnt + ls, (unsigned)__popcll(m));
      todo &= ~m;
    }
    if ((todo >> lane) & 1ull) atomicAdd(tcnt + s, 1u);
  }
  __syncthreads();
  unsigned d = 0, f1 = 0, f2 = 0;
  for (int i = threadIdx.x; i < CAP; i += blockDim.x) {
    const unsigned c = tcnt[i];
    d += c > 0;
    f1 += c == 1;
    f2 += c == 2;
  }
  for (int o = 32; o > 0; o >>= 1) {
    d += __shfl_down(d, o, 64);
    f1 += __shfl_down(f1, o, 64);
    f2 += __shfl_down(f2, o, 64);
  }
  if (lane == 0) {
    atomicAdd(fsum, d);
    atomicAdd(fsum + 1, f1);
    atomicAdd(fsum + 2, f2);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double dd = fsum[0], g1 = fsum[1], g2 = fsum[2];
    double est = dd;
    if (n > S) est = g2 > 0 ? dd + g1 * g1 / (2.0 * g2) : dd + g1 * (g1 - 1) / 2.0;
    est = std::min(est, (double)n);
    meta->est = (i64)est;
    // LOW: one small LDS table per workgroup; MID: the key space split into lowp hash partitions, each a large LDS
    // table, the partitions of one row range on one XCD (mid_keys: keys one MID table takes, 0 = no MID path)
    const i64 p = mid_keys > 0 ? (i64)((est + mid_keys - 1) / mid_keys) : 0;
    if (est <= (double)low_thr) {
      meta->low = 1;
      meta->lowp = 1;
    } else if (mid_keys > 0 && p <= kMidPMax) {
      meta->low = 2;
      meta->lowp = p < 1 ? 1 : p;
    } else {
      meta->low = 0;
    }
  }
}

// One launch presets both global tables ([key | acc | cnt | gid] words) and zeroes the meta words.
__global__ __launch_bounds__(256) void agg_init_kernel(u64* glow, i64 cap_low, u64* gpart, i64 cap_part, int F,
                                                       u64 ident, AggMeta* meta) {
  const i64 stride = (i64)gridDim.x * blockDim.x;
  const i64 t0 = (i64)blockIdx.x * blockDim.x + threadIdx.x;
  for (int which = 0; which < 2; ++which) {
    u64* base = which ? gpart : glow;
    if (base == nullptr) continue;               // phased launch: the PART table is set up in phase 2
    const i64 c1 = (which ? cap_part : cap_low) + 1;
    for (i64 i = t0; i < c1 * (3 + F); i += stride) {
      // key: kEmpty; acc: the op identity; cnt: 0; rmin: ~0 (the gid region is written on claim)
      base[i] = i < c1 ? kEmpty : (i < c1 * (1 + F) ? ident : (i < c1 * (2 + F) ? 0ull : ~0ull));
    }
  }
  if (meta != nullptr && t0 < (i64)(sizeof(AggMeta) / 8)) reinterpret_cast<i64*>(meta)[t0] = 0;
}

// ---------------------------------------------------------------- LOW path
constexpr int kU = 4;        // rows per thread loaded before any is processed (memory-level parallelism)
constexpr int kPreF = 1;     // value columns loaded with the keys (the rest at use)

// Row (key, values) batch of one thread: kU rows of a 256*kU-row tile, loaded together. Value (i, f) of the input
// is vals[i * rs + f * cs]: row-major [n, F] (rs = F, cs = 1) or column-major (rs = 1, cs = column pitch), so a
// caller's stacked columns are read in place.
template <typename VT, bool PRE = true>
struct RowBatch {
  u64 k[kU];
  VT v[kU][kPreF];
  // PRE = false (MID path): keys only; a row's values are read at use, by the one workgroup whose partition it is in
  __device__ __forceinline__ void load(const u64* __restrict__ keys, const VT* __restrict__ vals, i64 t0, i64 n,
                                       int F, int nthr, i64 rs, i64 cs) {
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const i64 i = t0 + (i64)j * nthr + threadIdx.x;
      k[j] = i < n ? keys[i] : kEmpty;
#pragma unroll
      for (int f = 0; f < kPreF; ++f) v[j][f] = (PRE && i < n && f < F) ? vals[i * rs + f * cs] : VT(0);
    }
  }
};

template <typename VT, int OP>
__device__ __forceinline__ void ltable_add_row(LTable t, int s, VT v0, const VT* __restrict__ vrow, int F, i64 cs,
                                               u64 row) {
  for (int f = 0; f < F; ++f)
    acc_add<VT, OP, __HIP_MEMORY_SCOPE_WORKGROUP>(t.acc + s * F + f, f == 0 ? v0 : vrow[f * cs]);
  __hip_atomic_fetch_add(t.cnt + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  const unsigned r32 = (unsigned)row;
  if (r32 < t.rmin[s]) __hip_atomic_fetch_min(t.rmin + s, r32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// MODE 1 (LOW): every workgroup aggregates its row tiles into one LDS table of lcap slots. MODE 2 (MID, 1024 threads,
// one workgroup per CU, grid = 256): the key space is split into P = meta->lowp hash partitions; the 32 workgroups
// of each XCD form floor(32 / P) row groups of P workgroups, workgroup (group, part) keeps only the keys of its
// partition in its (large) LDS table, and the P workgroups of a row group share their rows through the XCD's L2
// (HBM reads each row once). Many more groups than one LDS table holds are then aggregated in ONE pass over the
// input, without the PART path's partitioned write + read of every row.
__device__ __forceinline__ int mid_part(u64 k, int P) { return (int)((mix64(k) >> 40) % (u64)P); }

template <typename VT, int OP, int NT, int MODE>
__global__ __launch_bounds__(NT) void agg_low_kernel(const u64* __restrict__ keys, const VT* __restrict__ vals, i64 n,
                                                     int F, i64 rs, i64 cs, int lcap, GTable g, AggMeta* meta,
                                                     AggOut o) {
  if (meta->low != MODE) return;
  int P = 1, part = 0;
  i64 gb = blockIdx.x, ngb = gridDim.x;
  if constexpr (MODE == 2) {
    P = (int)meta->lowp;
    const int xcd = blockIdx.x & 7, m = blockIdx.x >> 3, q = (gridDim.x >> 3) / P;
    if (m >= q * P) return;                      // the workgroups left over when P does not divide 32
    part = m % P;
    gb = xcd + 8 * (m / P);
    ngb = 8 * q;
  }
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  LTable t = ltable_at(lds_raw, lcap, F);
  ltable_clear<VT, OP>(t, F);
  __syncthreads();
  constexpr int TILE = NT * kU;
  const i64 tstride = ngb * TILE;
  int it = 0;
  RowBatch<VT, MODE == 1> cur, nxt;
  i64 t0 = gb * TILE;
  if (t0 < n) cur.load(keys, vals, t0, n, F, NT, rs, cs);
  for (; t0 < n; t0 += tstride, ++it) {
    if ((it & 15) == 15 && __hip_atomic_load(&meta->fail_low, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    if (t0 + tstride < n) nxt.load(keys, vals, t0 + tstride, n, F, NT, rs, cs);   // in flight during this tile
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const i64 i = t0 + j * NT + threadIdx.x;
      if (i >= n) break;
      const u64 k = cur.k[j];
      if (MODE == 2 && (k == kEmpty ? part != 0 : mid_part(k, P) != part)) continue;   // another partition's key
      const VT* v = vals + i * rs;
      const int s = k != kEmpty ? ltable_slot(t, k, mix64(k)) : -1;
      if (s >= 0) {
        ltable_add_row<VT, OP>(t, s, MODE == 1 ? cur.v[j][0] : (F > 0 ? v[0] : VT(0)), v, F, cs, (u64)i);
      } else {   // rare: the values are re-read from memory
        row_into_global<VT, OP>(g, k, v, F, cs, &meta->ng_low, &meta->sentinel_low, &meta->fail_low, o, i);
      }
    }
    cur = nxt;
  }
  __syncthreads();
  // one flush per (workgroup, key)
  for (int e = threadIdx.x; e < lcap; e += blockDim.x) {
    const u64 k = t.key[e];
    if (k == kEmpty) continue;
    const i64 s = gtable_slot(g, k, &meta->ng_low, &meta->sentinel_low, &meta->fail_low, o);
    t.ref[e] = (int)-(s + 1);
    if (s < 0) continue;
    for (int f = 0; f < F; ++f) acc_merge_global<VT, OP>(g.acc + s * F + f, t.acc[e * F + f]);
    __hip_atomic_fetch_add(g.cnt + s, (u64)t.cnt[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_min(g.rmin + s, (u64)t.rmin[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (o.inv == nullptr) return;
  __syncthreads();
  for (i64 t0 = gb * TILE; t0 < n; t0 += tstride) {
    u64 k[kU];
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const i64 i = t0 + j * NT + threadIdx.x;
      k[j] = i < n ? keys[i] : kEmpty;
    }
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const i64 i = t0 + j * NT + threadIdx.x;
      if (k[j] == kEmpty || i >= n) continue;
      if (MODE == 2 && mid_part(k[j], P) != part) continue;
      const int s = ltable_find(t, k[j], mix64(k[j]));
      if (s >= 0) o.inv[i] = t.ref[s];
    }
  }
}

// ---------------------------------------------------------------- PART path
// bucket of a key: the top pbits of its hash (the LDS slot uses the low bits)
__device__ __forceinline__ int bucket_of(u64 k, int pbits) {
  return pbits == 0 ? 0 : (int)(mix64(k) >> (64 - pbits));
}

// Exclusive scan over a block (blockDim a multiple of 64, <= 1024; one value per thread); returns the
// thread's prefix, *total (shared) the block sum.
template <typename T>
__device__ __forceinline__ T block_scan_excl_t(T v, T* wsum, T* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  T x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const T y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[wave] = x;
  __syncthreads();
  if (threadIdx.x < 64) {
    T w = threadIdx.x < nw ? wsum[threadIdx.x] : T(0);
    T z = w;
#pragma unroll
    for (int d = 1; d < 16; d <<= 1) {
      const T y = __shfl_up(z, d, 64);
      if (threadIdx.x >= d) z += y;
    }
    if (threadIdx.x < nw) wsum[threadIdx.x] = z - w;
    if (threadIdx.x == nw - 1) *total = z;
  }
  __syncthreads();
  const T r = wsum[wave] + x - v;
  __syncthreads();   // wsum may be reused by the caller's next scan
  return r;
}

// rows [wg * rpw, min(n, (wg + 1) * rpw)) per workgroup; hist is bucket-major [P][G]
__global__ __launch_bounds__(1024) void agg_hist_kernel(const u64* __restrict__ keys, i64 n, i64 rpw, int pbits,
                                                        unsigned* __restrict__ hist, const AggMeta* meta) {
  if (!take_part(meta)) return;
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  unsigned* h = reinterpret_cast<unsigned*>(lds_raw);
  const int P = 1 << pbits;
  for (int i = threadIdx.x; i < P; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const i64 r0 = (i64)blockIdx.x * rpw, r1 = std::min<i64>(n, r0 + rpw);
  // 16-byte loads (two keys per lane), the next batch in flight while this one is counted
  constexpr int U = 4;
  const i64 step = (i64)U * 2 * 1024;
  const i64 e2 = r0 + ((r1 - r0) & ~(i64)1);   // even part: pairs
  u64 k[U][2], nk[U][2];
  auto load = [&](i64 b0, u64 (&kk)[U][2]) {
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 i = b0 + (i64)(j * 1024 + threadIdx.x) * 2;
      if (i < e2) {
        const ulonglong2 v = *reinterpret_cast<const ulonglong2*>(keys + i);
        kk[j][0] = v.x;
        kk[j][1] = v.y;
      }
    }
  };
  const bool aligned = ((reinterpret_cast<uintptr_t>(keys + r0)) & 15) == 0;
  if (aligned) {
    if (r0 < e2) load(r0, k);
    for (i64 b0 = r0; b0 < e2; b0 += step) {
      if (b0 + step < e2) load(b0 + step, nk);
#pragma unroll
      for (int j = 0; j < U; ++j) {
        const i64 i = b0 + (i64)(j * 1024 + threadIdx.x) * 2;
        if (i < e2) {
          atomicAdd(h + bucket_of(k[j][0], pbits), 1u);
          atomicAdd(h + bucket_of(k[j][1], pbits), 1u);
        }
      }
#pragma unroll
      for (int j = 0; j < U; ++j) {
        k[j][0] = nk[j][0];
        k[j][1] = nk[j][1];
      }
    }
    if (threadIdx.x == 0 && e2 < r1) atomicAdd(h + bucket_of(keys[e2], pbits), 1u);   // odd tail row
  } else {
    for (i64 i = r0 + threadIdx.x; i < r1; i += blockDim.x) atomicAdd(h + bucket_of(keys[i], pbits), 1u);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < P; b += blockDim.x) hist[(size_t)b * gridDim.x + blockIdx.x] = h[b];
}

// workgroup b: exclusive scan of hist[b][0..G) in place (G <= 1024, one entry per thread), tot[b] = its sum
__global__ __launch_bounds__(1024) void scan_rows_kernel(unsigned* __restrict__ hist, int G, i64* __restrict__ tot,
                                                         const AggMeta* meta, int guard) {
  if (guard && !take_part(meta)) return;
  __shared__ unsigned wsum[16], total;
  unsigned* row = hist + (size_t)blockIdx.x * G;
  const unsigned v = (int)threadIdx.x < G ? row[threadIdx.x] : 0u;
  const unsigned pre = block_scan_excl_t<unsigned>(v, wsum, &total);
  if ((int)threadIdx.x < G) row[threadIdx.x] = pre;
  if (threadIdx.x == 0) tot[blockIdx.x] = total;
}

// one workgroup: bstart = exclusive scan of tot[P] (P <= 2048), bstart[P] = the total
__global__ __launch_bounds__(1024) void scan_tot_kernel(const i64* __restrict__ tot, int P, i64* __restrict__ bstart,
                                                        AggMeta* meta, int guard) {
  if (guard && !take_part(meta)) return;
  __shared__ i64 wsum[16], total;
  const int c0 = threadIdx.x * 2;
  const i64 a = c0 < P ? tot[c0] : 0, b = c0 + 1 < P ? tot[c0 + 1] : 0;
  const i64 pre = block_scan_excl_t<i64>(a + b, wsum, &total);
  if (c0 < P) bstart[c0] = pre;
  if (c0 + 1 < P) bstart[c0 + 1] = pre + a;
  if (threadIdx.x == 0) bstart[P] = total;
}

// Tile-staged scatter of rows [r0, r1) (read through rows_of, or 0..: plain row ids) into bucket runs: each
// 1024-thread pass stages up to T rows in LDS sorted by bucket (counting sort: LDS histogram, block scan,
// ranks from the histogram atomics), then writes each bucket's run contiguously at run[b], so the global
// stores are long coalesced runs instead of one random 8-byte store per row. run[] (LDS, i64 [P]) is
// advanced by the tile's counts. Row order inside a bucket is not preserved (the aggregates keep min row ids).
template <typename VT, int R>
__device__ __forceinline__ void staged_scatter(const u64* __restrict__ skey, const VT* __restrict__ sval, i64 rs,
                                               i64 cs, const int* __restrict__ srow, i64 r0, i64 r1, int F, int shift,
                                               int P, int T, char* lds, i64* run, unsigned* cnt, unsigned* off,
                                               unsigned* wsum, u64* __restrict__ dkey, VT* __restrict__ dval,
                                               int* __restrict__ drow) {
  // R rows per thread per tile (T <= R * blockDim)
  const int nthr = blockDim.x;
  u64* st_key = reinterpret_cast<u64*>(lds);
  VT* st_val = reinterpret_cast<VT*>(st_key + T);
  int* st_row = reinterpret_cast<int*>(st_val + (size_t)T * F);
  unsigned short* st_b = reinterpret_cast<unsigned short*>(st_row + T);
  __shared__ unsigned tot_sh;
  const unsigned pmask = (unsigned)P - 1;
  const int rowsrc = srow != nullptr;
  const bool rows = drow != nullptr;      // carry row ids (first-row / inverse outputs wanted)
  // the next tile's keys / first value / row ids are loaded while this tile goes through its LDS phases
  u64 k[R], nk[R];
  VT v0[R], nv0[R];
  int rw[R], nrw[R];
  auto load_tile = [&](i64 tb, u64 (&kk)[R], VT (&vv)[R], int (&rr)[R]) {
    const int tnn = (int)std::min<i64>(T, r1 - tb);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int p = threadIdx.x + j * nthr;
      const bool in = p < tnn;
      kk[j] = in ? skey[tb + p] : 0;
      vv[j] = (in && F > 0) ? sval[(tb + p) * rs] : VT(0);
      rr[j] = (in && rows) ? (rowsrc ? srow[tb + p] : (int)(tb + p)) : 0;
    }
  };
  if (r0 < r1) load_tile(r0, k, v0, rw);
  for (i64 t0 = r0; t0 < r1; t0 += T) {
    const int tn = (int)std::min<i64>(T, r1 - t0);
    for (int b = threadIdx.x; b < P; b += blockDim.x) cnt[b] = 0;
    __syncthreads();
    int bk[R];
    unsigned rk[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int p = threadIdx.x + j * nthr;
      if (p < tn) {
        bk[j] = P == 1 ? 0 : (int)((mix64(k[j]) >> shift) & pmask);
        rk[j] = atomicAdd(cnt + bk[j], 1u);
      }
    }
    if (t0 + T < r1) load_tile(t0 + T, nk, nv0, nrw);
    __syncthreads();
    // exclusive scan of cnt[0..P) (P <= 4 * blockDim buckets)
    {
      const int per = (P + nthr - 1) / nthr;
      const int c0 = threadIdx.x * per;
      unsigned sum = 0;
      for (int c = c0; c < c0 + per && c < P; ++c) sum += cnt[c];
      unsigned pre = block_scan_excl_t<unsigned>(sum, wsum, &tot_sh);
      for (int c = c0; c < c0 + per && c < P; ++c) {
        off[c] = pre;
        pre += cnt[c];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int p = threadIdx.x + j * nthr;
      if (p < tn) {
        const unsigned q = off[bk[j]] + rk[j];
        const i64 i = t0 + p;
        st_key[q] = k[j];
        if (rows) st_row[q] = rw[j];
        st_b[q] = (unsigned short)bk[j];
        for (int f = 0; f < F; ++f) st_val[(size_t)q * F + f] = f == 0 ? v0[j] : sval[i * rs + f * cs];
      }
    }
    __syncthreads();
    for (int q = threadIdx.x; q < tn; q += blockDim.x) {
      const int b = st_b[q];
      const i64 dst = run[b] + (q - (int)off[b]);
      dkey[dst] = st_key[q];
      if (rows) drow[dst] = st_row[q];
      for (int f = 0; f < F; ++f) dval[dst * F + f] = st_val[(size_t)q * F + f];
    }
    __syncthreads();
    for (int b = threadIdx.x; b < P; b += blockDim.x) run[b] += cnt[b];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < R; ++j) {
      k[j] = nk[j];
      v0[j] = nv0[j];
      rw[j] = nrw[j];
    }
  }
}

// level-1 scatter: workgroup g packs its rows [g * rpw, ...) into the P1 buckets at bstart[b] + hist[b][g]
template <typename VT>
__global__ __launch_bounds__(1024) void agg_scatter_kernel(const u64* __restrict__ keys, const VT* __restrict__ vals,
                                                           i64 rs, i64 cs, i64 n, int F, i64 rpw, int pbits, int T,
                                                           const unsigned* __restrict__ hist,
                                                           const i64* __restrict__ bstart, u64* __restrict__ pkey,
                                                           VT* __restrict__ pval, int* __restrict__ prow,
                                                           const AggMeta* meta) {
  if (!take_part(meta)) return;
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  __shared__ i64 run[1024];
  __shared__ unsigned cnt[1024], off[1024], wsum[16];
  const int P = 1 << pbits;
  for (int b = threadIdx.x; b < P; b += blockDim.x) run[b] = bstart[b] + hist[(size_t)b * gridDim.x + blockIdx.x];
  __syncthreads();
  const i64 r0 = (i64)blockIdx.x * rpw, r1 = std::min<i64>(n, r0 + rpw);
  staged_scatter<VT, 4>(keys, vals, rs, cs, nullptr, r0, r1, F, 64 - pbits, P, T, lds_raw, run, cnt, off, wsum, pkey, pval,
                        prow);
}

// ngrp thread groups (blockDim / ngrp threads each, ngrp <= 4) each aggregate their rows [a, e) of (key, val,
// row) in their own LDS table t (cleared first), then write the groups straight to the dense output: the caller
// guarantees a range holds every row of its keys. Every thread of the block calls this (block-wide barriers);
// rows whose LDS probe window is full go to the global table (emitted later by agg_emit). One global atomic per
// call reserves the dense ids of all groups of all ranges.
template <typename VT, int OP>
__device__ __forceinline__ void agg_ranges_dense(const u64* __restrict__ pkey, const VT* __restrict__ pval,
                                                 const int* __restrict__ prow, i64 a, i64 e, int F, LTable t,
                                                 int ngrp, GTable g, AggMeta* meta, AggOut o) {
  __shared__ int nocc[4];
  __shared__ i64 base_sh[4];
  const int gs = blockDim.x / ngrp, gi = threadIdx.x / gs, lt = threadIdx.x % gs;
  ltable_clear<VT, OP>(t, F, lt, gs);
  if (threadIdx.x < 4) nocc[threadIdx.x] = 0;
  __syncthreads();
  // double-buffered row batches: batch b+1 is in flight while batch b goes into the LDS table
  const i64 step = (i64)gs * kU;
  u64 k[kU], nk[kU];
  int rw[kU], nrw[kU];
  VT v0[kU], nv0[kU];
  auto load_b = [&](i64 b0, u64 (&kk)[kU], int (&rr)[kU], VT (&vv)[kU]) {
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const i64 r = b0 + (i64)j * gs + lt;
      const bool in = r < e;
      kk[j] = in ? pkey[r] : kEmpty;
      rr[j] = (in && prow) ? prow[r] : 0;
      vv[j] = (in && F > 0) ? pval[r * F] : VT(0);
    }
  };
  if (a < e) load_b(a, k, rw, v0);
  for (i64 b0 = a; b0 < e; b0 += step) {
    if (b0 + step < e) load_b(b0 + step, nk, nrw, nv0);
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      const i64 r = b0 + (i64)j * gs + lt;
      if (r >= e) break;
      const VT* v = pval + r * F;
      const int sl = k[j] != kEmpty ? ltable_slot(t, k[j], mix64(k[j])) : -1;
      if (sl >= 0) {
        ltable_add_row<VT, OP>(t, sl, v0[j], v, F, 1, (u64)rw[j]);
      } else {   // rare (the table's probe window is full): the values are re-read from memory
        row_into_global<VT, OP>(g, k[j], v, F, 1, &meta->ng_part, &meta->sentinel_part, &meta->fail_part, o, rw[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < kU; ++j) {
      k[j] = nk[j];
      rw[j] = nrw[j];
      v0[j] = nv0[j];
    }
  }
  __syncthreads();
  for (int x = lt; x < t.cap; x += gs)
    if (t.key[x] != kEmpty) t.ref[x] = atomicAdd(&nocc[gi], 1);   // local id (any order)
  __syncthreads();
  if (threadIdx.x == 0) {
    i64 tot = 0;
    for (int q = 0; q < ngrp; ++q) tot += nocc[q];
    i64 b = tot ? __hip_atomic_fetch_add(&meta->ng_part, tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    for (int q = 0; q < ngrp; ++q) {
      base_sh[q] = b;
      b += nocc[q];
    }
  }
  __syncthreads();
  const i64 base = base_sh[gi];
  for (int x = lt; x < t.cap; x += gs) {
    const u64 k = t.key[x];
    if (k == kEmpty) continue;
    const i64 gid = base + t.ref[x];
    t.ref[x] = (int)gid;
    o.reps[gid] = (i64)k;
    o.cnt[gid] = (i64)t.cnt[x];
    o.first[gid] = (i64)t.rmin[x];
    for (int f = 0; f < F; ++f) o.aggs[gid * F + f] = acc_out<VT, OP>(t.acc[x * F + f]);
  }
  if (o.inv != nullptr) {
    __syncthreads();
    for (i64 r = a + lt; r < e; r += gs) {
      const u64 k = pkey[r];
      if (k == kEmpty) continue;
      const int sl = ltable_find(t, k, mix64(k));
      if (sl >= 0) o.inv[prow[r]] = t.ref[sl];
    }
  }
  __syncthreads();
}

// Workgroup b owns level-1 bucket b whole (no other workgroup sees its keys). When the estimated distinct keys
// of the bucket fit the LDS table at load <= 1/2 it aggregates the bucket directly; otherwise it first splits the
// bucket into P2 sub-buckets by the next hash bits (its own histogram + staged scatter into the second buffer,
// same positions) and aggregates them four at a time (four thread groups, four LDS tables of a quarter each).
// No global atomics per row: one per group flush and one per round for the dense ids.
template <typename VT, int OP>
__global__ __launch_bounds__(1024) void agg_bucket_kernel(const u64* __restrict__ pkey, const VT* __restrict__ pval,
                                                          const int* __restrict__ prow, int F, int lcap, int p1bits,
                                                          int T, i64 n, const i64* __restrict__ bstart,
                                                          u64* __restrict__ qkey, VT* __restrict__ qval,
                                                          int* __restrict__ qrow, GTable g, AggMeta* meta, AggOut o) {
  if (!take_part(meta)) return;
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  __shared__ i64 run[1024];
  __shared__ unsigned cnt[1024], off[1024], wsum[16], sb[1025];
  const int b = blockIdx.x;
  const i64 r0 = bstart[b], r1 = bstart[b + 1], nb = r1 - r0;
  if (nb == 0) return;
  const int P1 = 1 << p1bits;
  // expected distinct keys of this bucket: the estimate's share with 25 % slack (Chao1 on a 4096-row sample is
  // within a few % on uniform keys), never above its rows; tables are filled to <= 3/4 (a miss-sized bucket
  // only sends its overflow rows to the global table)
  const i64 est = meta->est;
  const i64 db = std::min<i64>(nb, (5 * ((est + P1 - 1) / P1)) / 4 + 16);
  if (4 * db <= 3 * lcap) {
    int cap = 256;   // direct path: LDS is plentiful, keep the load <= 1/4 (short probes; measured faster)
    while (cap < lcap && cap < 4 * db) cap <<= 1;
    agg_ranges_dense<VT, OP>(pkey, pval, prow, r0, r1, F, ltable_at(lds_raw, cap, F), 1, g, meta, o);
    return;
  }
  constexpr int NG = 4;
  const int qcap = lcap / NG;   // each group's table
  int p2bits = 0;
  while (p2bits < 10 && (db >> p2bits) * 4 > 3 * qcap) ++p2bits;
  const int P2 = 1 << p2bits;
  const int shift = 64 - p1bits - p2bits;
  const unsigned pmask = (unsigned)P2 - 1;
  // histogram of the sub-buckets
  for (int c = threadIdx.x; c < P2; c += blockDim.x) cnt[c] = 0;
  __syncthreads();
  for (i64 b0 = r0; b0 < r1; b0 += 8 * 1024) {
    u64 k[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const i64 r = b0 + j * 1024 + threadIdx.x;
      k[j] = r < r1 ? pkey[r] : 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (b0 + j * 1024 + threadIdx.x < r1) atomicAdd(cnt + ((mix64(k[j]) >> shift) & pmask), 1u);
  }
  __syncthreads();
  {
    __shared__ unsigned tot_sh2;
    const unsigned v = threadIdx.x < P2 ? cnt[threadIdx.x] : 0u;
    const unsigned pre = block_scan_excl_t<unsigned>(v, wsum, &tot_sh2);
    if (threadIdx.x < P2) {
      sb[threadIdx.x] = pre;
      run[threadIdx.x] = r0 + pre;
    }
    if (threadIdx.x == 0) sb[P2] = (unsigned)nb;
  }
  __syncthreads();
  staged_scatter<VT, 2>(pkey, pval, F, 1, prow, r0, r1, F, shift, P2, T, lds_raw, run, cnt, off, wsum, qkey, qval, qrow);
  // this workgroup reads back what its own waves stored: drain the stores, then drop this CU's L1 lines
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const i64 dsub = std::min<i64>(nb, (db >> p2bits) + 16);
  int cap = 64;
  while (cap < qcap && 3 * cap < 4 * dsub) cap <<= 1;
  const int gi = threadIdx.x / (blockDim.x / NG);
  const LTable t = ltable_at(lds_raw + (size_t)gi * cap * (20 + 8 * F), cap, F);
  for (int s0 = 0; s0 < P2; s0 += NG) {
    const int s2 = s0 + gi;
    const i64 a = s2 < P2 ? r0 + sb[s2] : 0, e = s2 < P2 ? r0 + sb[s2 + 1] : 0;
    agg_ranges_dense<VT, OP>(qkey, qval, qrow, a, e, F, t, NG, g, meta, o);
  }
}

// global-table groups -> dense output: a sweep over the slots of the taken path's table (at most 2^17 + 1;
// the groups written straight from LDS are not visited at all)
template <typename VT, int OP>
__global__ __launch_bounds__(256) void agg_emit_kernel(GTable glow, GTable gpart, int F, const AggMeta* meta,
                                                       AggOut o) {
  const bool low = !take_part(meta);
  const GTable g = low ? glow : gpart;
  const bool sentinel = (low ? meta->sentinel_low : meta->sentinel_part) != 0;
  const i64 nslots = (i64)g.mask + 2;   // cap slots + the kEmpty key's slot
  for (i64 s = (i64)blockIdx.x * blockDim.x + threadIdx.x; s < nslots; s += (i64)gridDim.x * blockDim.x) {
    const bool used = s == nslots - 1 ? sentinel : g.key[s] != kEmpty;
    if (!used) continue;
    const i64 gid = g.gid_of_slot[s];
    o.cnt[gid] = (i64)g.cnt[s];
    o.first[gid] = (i64)g.rmin[s];
    for (int f = 0; f < F; ++f) o.aggs[gid * F + f] = acc_out<VT, OP>(g.acc[s * F + f]);
  }
}

// per-row global-slot references (-(slot + 1)) -> dense group ids
__global__ __launch_bounds__(256) void agg_fix_inv_kernel(i64* __restrict__ inv, i64 n, const i64* __restrict__ gid_low,
                                                          const i64* __restrict__ gid_part, const AggMeta* meta) {
  const i64* gos = take_part(meta) ? gid_part : gid_low;
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    const i64 v = inv[i];
    if (v < 0) inv[i] = gos[-v - 1];
  }
}

// ---------------------------------------------------------------- hash join
// Tables of more than kJWholeWrap slots probe linearly inside aligned regions of kJRegion slots (a chain wraps at its
// region's end) and are built region by region in LDS (join_region_build_kernel); smaller ones (builds up to ~1 M
// rows, whose table fits the MALL) probe the whole table with plain linear probing and take the global-atomic insert
// (no region can fill: no host check). Every probe (join_probe_kernel here, pipeline_core.h join_find /
// join_find_rows, whose JREGION / JWHOLE must equal kJRegion / kJWholeWrap) walks the same order.
constexpr int kJRegionBits = 12;
constexpr u64 kJRegion = 1ull << kJRegionBits;
constexpr u64 kJWholeWrap = 1ull << 22;   // tables of at most this many slots: chains wrap at the table's end
__device__ __forceinline__ u64 jregion_mask(u64 mask) { return mask < kJWholeWrap ? mask : kJRegion - 1; }
__device__ __forceinline__ u64 jnext(u64 s, u64 mask) {
  const u64 rm = jregion_mask(mask);
  return (s & ~rm) | ((s + 1) & rm);
}

// Table: cap + 1 16-byte slots {key, cnt | pay << 32} (slot cap: the kEmpty key). cnt counts the key's build rows
// beyond the first (the kEmpty slot: all of them); pay = the build row itself when the key has one build row (the
// primary-key case), else the start of its CSR run in perm. A probe row is then ONE 16-byte random read (key, count
// and row together) and, for unique build keys, no second lookup; a build without repeated keys needs no CSR pass.
struct JSlot {
  u64 key;
  unsigned cnt;
  unsigned pay;
};

// The row that claims a slot (CAS) is its key's rank 0 and stores itself as the payload; each further row of
// the key takes the next rank with one atomic add on the slot's count of EXTRA rows (a unique-key build does one
// atomic per row). *ndup counts the rows of rank > 0 (one add per wave): zero means the CSR pass is skipped.
__global__ __launch_bounds__(256) void join_insert_kernel(const u64* __restrict__ keys, i64 n, JSlot* tab, u64 mask,
                                                          int* __restrict__ row_slot, unsigned* __restrict__ row_rank,
                                                          unsigned long long* ndup, unsigned* fail) {
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    const u64 k = keys[i];
    u64 s;
    bool claimed = false;
    if (k == kEmpty) {
      s = mask + 1;   // the kEmpty key's own slot: every row counts as an extra, ranks from 1 (fixed below)
    } else {
      s = mix64(k) & mask;
      // CAS first (no separate load of the slot): a claim is ONE memory-side atomic, and a failed CAS returns the
      // slot's key, which is all a load would have told (the key itself, or another key: next slot)
      bool found = false;
      const u64 rm = jregion_mask(mask);
      for (u64 it = 0; it <= rm; ++it) {   // bounded: a full region (never at the table's load) raises *fail
        u64 cur = kEmpty;
        if (__hip_atomic_compare_exchange_strong(&tab[s].key, &cur, k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)) {
          claimed = true;
          found = true;
          break;
        }
        if (cur == k) {
          found = true;
          break;
        }
        s = jnext(s, mask);
      }
      if (!found) {
        __hip_atomic_store(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        row_slot[i] = (int)(mask + 1);
        row_rank[i] = 0;
        continue;
      }
    }
    row_slot[i] = (int)s;
    unsigned r = 0;
    if (claimed) {
      tab[s].pay = (unsigned)i;
    } else {
      r = __hip_atomic_fetch_add(&tab[s].cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + (k == kEmpty ? 0u : 1u);
      if (r == 0) tab[s].pay = (unsigned)i;   // the kEmpty slot's first row
    }
    row_rank[i] = r;
    const u64 dups = __ballot(r != 0);
    if (dups != 0 && (threadIdx.x & 63) == (unsigned)(__ffsll((long long)__ballot(1)) - 1))
      __hip_atomic_fetch_add(ndup, (unsigned long long)__popcll(dups), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Every slot {kEmpty, 0, 0} in one streaming pass of 16-B stores (two strided torch fills wrote each line twice).
__global__ __launch_bounds__(256) void join_init_kernel(JSlot* tab, i64 nslots) {
  for (i64 s = (i64)blockIdx.x * blockDim.x + threadIdx.x; s < nslots; s += (i64)gridDim.x * blockDim.x)
    tab[s] = JSlot{kEmpty, 0u, 0u};
}

// Runs of the keys with more than one build row, with no host decision: every slot whose key repeated takes a run
// of perm, moves its claiming row (the payload) to the run's first entry and makes the run start its payload. Runs
// come from one bump counter with ONE atomic per 4096-slot tile (thread sums -> block scan; a per-wave atomic on
// one address serialised at the memory side: 6 ms for a 15 M-row build). Both kernels return at once when the
// insert saw no repeated key (*ndup == 0).
constexpr int kRunsPer = 16;   // slots per thread per tile (strided by the block)

__device__ __forceinline__ unsigned join_run_len(const JSlot& e, i64 s, u64 sent) {
  const bool is_sent = (u64)s == sent;
  const unsigned tot = (!is_sent && e.key == kEmpty) ? 0u : e.cnt + (is_sent ? 0u : 1u);
  return tot > 1 ? tot : 0u;
}

__global__ __launch_bounds__(256) void join_runs_kernel(JSlot* tab, u64 mask, const unsigned long long* ndup,
                                                        unsigned long long* bump, i64* __restrict__ perm) {
  if (*ndup == 0) return;
  __shared__ unsigned wsum[4], tsum;
  __shared__ unsigned long long base_sh;
  const u64 sent = mask + 1;
  const i64 nslots = (i64)mask + 2;
  constexpr i64 TILE = 256 * kRunsPer;
  for (i64 t0 = (i64)blockIdx.x * TILE; t0 < nslots; t0 += (i64)gridDim.x * TILE) {
    unsigned mine = 0;
#pragma unroll 4
    for (int q = 0; q < kRunsPer; ++q) {
      const i64 s = t0 + q * 256 + threadIdx.x;
      if (s < nslots) mine += join_run_len(tab[s], s, sent);
    }
    const unsigned pre = block_scan_excl_t<unsigned>(mine, wsum, &tsum);
    if (threadIdx.x == 0)
      base_sh = tsum ? __hip_atomic_fetch_add(bump, (unsigned long long)tsum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : 0ull;
    __syncthreads();
    i64 o = (i64)base_sh + pre;
    if (mine) {
      for (int q = 0; q < kRunsPer; ++q) {
        const i64 s = t0 + q * 256 + threadIdx.x;
        if (s >= nslots) break;
        const JSlot e = tab[s];
        const unsigned len = join_run_len(e, s, sent);
        if (len == 0) continue;
        perm[o] = (i64)e.pay;              // the claiming row is rank 0
        tab[s].pay = (unsigned)o;
        o += len;
      }
    }
    __syncthreads();
  }
}

// rows of rank > 0: perm[run start + rank] = row
__global__ __launch_bounds__(256) void join_perm_kernel(const int* __restrict__ row_slot,
                                                        const unsigned* __restrict__ row_rank, i64 n,
                                                        const unsigned long long* ndup, const JSlot* tab,
                                                        i64* __restrict__ perm) {
  if (*ndup == 0) return;
  for (i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (i64)gridDim.x * blockDim.x) {
    const unsigned r = row_rank[i];
    if (r == 0) continue;
    perm[(i64)tab[row_slot[i]].pay + r] = i;
  }
}

// Probe filter of a large table (a blocked Bloom filter, one 64-bit word per 2^shift consecutive HOME slots, two bits
// per key from the slot hash's high bits). A probe reads its word — the filter is ~2 bytes per build row, L2-resident
// where the table is not — and touches the table only when both bits are set: most probe rows of a selective join
// (TPC-H Q12: 15 M orders against 0.3 M late lineitems) then never leave L2. Built from the finished table, one
// thread per word over its slot range (no atomics for keys at their home word; the few displaced past the range end
// OR into their home word atomically).
__device__ __forceinline__ u64 bloom_bits(u64 f) { return (1ull << ((f >> 40) & 63)) | (1ull << ((f >> 46) & 63)); }

// ---- partitioned build of a table of more than one region (cap > kJRegion): rows are partitioned by home region
// (histogram per workgroup chunk, a bin-major scan, an LDS-ranked scatter of (key, row)), then ONE workgroup per
// region inserts its rows into an LDS image of the region (LDS CAS / add: no memory-side atomics, which bound the
// global insert at ~10 G claims/s once the table outgrows the MALL) and writes the region out in one coalesced
// pass, with its probe-filter words. Bin P holds the rows whose key is kEmpty (the sentinel slot, global atomics).
// Per row (in partition order) the build keeps its slot and rank for the CSR pass of repeated keys.
constexpr int kJPartThreads = 512;

// bin of a key: its home region >> sh (sh > 0: the coarse bins of a two-level partition), P for the kEmpty key
__device__ __forceinline__ unsigned jbin_of(u64 k, u64 mask, unsigned P, int sh) {
  return k == kEmpty ? P : (unsigned)((mix64(k) & mask) >> (kJRegionBits + sh));
}

// hist [G chunks][P + 1 bins] (chunk-major: each workgroup's row of counts is one coalesced store); chunk g = rows
// [g * rpw, min(n, g * rpw + rpw))
__global__ __launch_bounds__(kJPartThreads) void jpart_hist_kernel(const u64* __restrict__ keys, i64 n, i64 rpw,
                                                                   u64 mask, unsigned P, int sh,
                                                                   unsigned* __restrict__ hist,
                                                                   JSlot* tab) {
  extern __shared__ unsigned lh[];
  const unsigned g = blockIdx.x;
  for (unsigned b = threadIdx.x; b <= P; b += blockDim.x) lh[b] = 0;
  if (g == 0 && threadIdx.x == 0) tab[mask + 1] = JSlot{kEmpty, 0u, 0u};   // the sentinel slot (bin P uses it)
  __syncthreads();
  const i64 r0 = (i64)g * rpw, r1 = min(n, r0 + rpw);
  constexpr int U = 8;                                  // 8 key loads in flight per thread
  for (i64 c0 = r0; c0 < r1; c0 += (i64)U * blockDim.x) {
    u64 k[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 i = c0 + (i64)j * blockDim.x + threadIdx.x;
      k[j] = i < r1 ? keys[i] : 0;
    }
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (c0 + (i64)j * blockDim.x + threadIdx.x < r1) atomicAdd(&lh[jbin_of(k[j], mask, P, sh)], 1u);
  }
  __syncthreads();
  for (unsigned b = threadIdx.x; b <= P; b += blockDim.x) hist[(i64)g * (P + 1) + b] = lh[b];
}

// per bin (one thread each): exclusive scan over the G chunks' counts in place, down the column (for each chunk the
// threads of a wave read adjacent bins: coalesced); the bin's total into btot[b]
__global__ __launch_bounds__(256) void jpart_colscan_kernel(unsigned* __restrict__ hist, unsigned G, unsigned nb,
                                                            i64* __restrict__ btot) {
  const unsigned b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  unsigned run = 0;
  constexpr unsigned B = 16;            // 16 chunk counts loaded before any is rewritten: their latencies overlap
  for (unsigned g0 = 0; g0 < G; g0 += B) {
    unsigned v[B];
#pragma unroll
    for (unsigned j = 0; j < B; ++j) v[j] = g0 + j < G ? hist[(i64)(g0 + j) * nb + b] : 0u;
#pragma unroll
    for (unsigned j = 0; j < B; ++j) {
      if (g0 + j < G) hist[(i64)(g0 + j) * nb + b] = run;
      run += v[j];
    }
  }
  btot[b] = run;
}

// one workgroup: bbase[b] = exclusive scan of btot over the P + 1 bins, bbase[P + 1] = n
__global__ __launch_bounds__(1024) void jpart_totscan_kernel(const i64* __restrict__ btot, unsigned nb,
                                                             i64* __restrict__ bbase) {
  __shared__ i64 ws[16], tot;
  const unsigned per = (nb + 1023) / 1024, b0 = threadIdx.x * per;
  i64 mine = 0;
  for (unsigned b = b0; b < min(nb, b0 + per); ++b) mine += btot[b];
  // block exclusive scan of the 1024 thread sums (64-bit)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  i64 x = mine;
  for (int d = 1; d < 64; d <<= 1) {
    const i64 y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) ws[wave] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    i64 acc = 0;
    for (int w = 0; w < 16; ++w) {
      const i64 t = ws[w];
      ws[w] = acc;
      acc += t;
    }
    tot = acc;
  }
  __syncthreads();
  i64 o = ws[wave] + x - mine;
  for (unsigned b = b0; b < min(nb, b0 + per); ++b) {
    bbase[b] = o;
    o += btot[b];
  }
  if (threadIdx.x == 0) bbase[nb] = tot;
}

// scatter: chunk g's rows to bbase[bin] + hist[bin][g] + (LDS rank inside the chunk's share of the bin)
__global__ __launch_bounds__(kJPartThreads) void jpart_scatter_kernel(const u64* __restrict__ keys, i64 n, i64 rpw,
                                                                      u64 mask, unsigned P, int sh,
                                                                      const unsigned* __restrict__ hist,
                                                                      const i64* __restrict__ bbase,
                                                                      u64* __restrict__ ikey, unsigned* __restrict__ irow) {
  extern __shared__ unsigned lo[];     // [P + 1] running offset (relative to bbase) of this chunk in each bin
  const unsigned g = blockIdx.x;
  for (unsigned b = threadIdx.x; b <= P; b += blockDim.x) lo[b] = hist[(i64)g * (P + 1) + b];
  __syncthreads();
  const i64 r0 = (i64)g * rpw, r1 = min(n, r0 + rpw);
  constexpr int U = 8;
  for (i64 c0 = r0; c0 < r1; c0 += (i64)U * blockDim.x) {
    u64 k[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 i = c0 + (i64)j * blockDim.x + threadIdx.x;
      k[j] = i < r1 ? keys[i] : 0;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 i = c0 + (i64)j * blockDim.x + threadIdx.x;
      if (i >= r1) continue;
      const unsigned b = jbin_of(k[j], mask, P, sh);
      const i64 pos = bbase[b] + atomicAdd(&lo[b], 1u);
      ikey[pos] = k[j];
      irow[pos] = (unsigned)i;
    }
  }
}

// The coarse scatter of a two-level partition (<= kJStageBins bins), staged through LDS: each 4096-row tile is
// counting-sorted by bin in LDS, then written out bin run by bin run (consecutive threads, consecutive addresses of
// one run: ~16 rows = 128 B of keys per run at 257 bins) instead of every row to a line of its own.
constexpr int kJStageBins = 1024, kJTileRows = 4096;
__global__ __launch_bounds__(kJPartThreads) void jpart_scatter_staged_kernel(
    const u64* __restrict__ keys, i64 n, i64 rpw, u64 mask, unsigned P, int sh, const unsigned* __restrict__ hist,
    const i64* __restrict__ bbase, u64* __restrict__ ikey, unsigned* __restrict__ irow) {
  __shared__ u64 lk[kJTileRows];
  __shared__ unsigned lr[kJTileRows];
  __shared__ unsigned short lb[kJTileRows];
  __shared__ unsigned tcnt[kJStageBins], tst[kJStageBins], lo[kJStageBins];
  __shared__ unsigned wsum[kJPartThreads / 64], tsum;
  const unsigned g = blockIdx.x, nb = P + 1;
  for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) lo[b] = (unsigned)(bbase[b] + hist[(i64)g * nb + b]);
  const i64 r0 = (i64)g * rpw, r1 = min(n, r0 + rpw);
  constexpr int U = kJTileRows / kJPartThreads;
  const unsigned per = (nb + kJPartThreads - 1) / kJPartThreads;
  for (i64 t0 = r0; t0 < r1; t0 += kJTileRows) {
    u64 k[U];
    unsigned bj[U], rk[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 i = t0 + j * kJPartThreads + threadIdx.x;
      k[j] = i < r1 ? keys[i] : 0;
    }
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) tcnt[b] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 i = t0 + j * kJPartThreads + threadIdx.x;
      bj[j] = jbin_of(k[j], mask, P, sh);
      if (i < r1) rk[j] = atomicAdd(&tcnt[bj[j]], 1u);
    }
    __syncthreads();
    // tile-local bin starts: each thread sums `per` consecutive bins, one block scan
    unsigned mine = 0;
    for (unsigned q = 0; q < per; ++q) {
      const unsigned b = threadIdx.x * per + q;
      if (b < nb) mine += tcnt[b];
    }
    unsigned o = block_scan_excl_t<unsigned>(mine, wsum, &tsum);
    for (unsigned q = 0; q < per; ++q) {
      const unsigned b = threadIdx.x * per + q;
      if (b < nb) {
        tst[b] = o;
        o += tcnt[b];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 i = t0 + j * kJPartThreads + threadIdx.x;
      if (i >= r1) continue;
      const unsigned q = tst[bj[j]] + rk[j];
      lk[q] = k[j];
      lr[q] = (unsigned)i;
      lb[q] = (unsigned short)bj[j];
    }
    __syncthreads();
    const unsigned rows = (unsigned)min((i64)kJTileRows, r1 - t0);
    for (unsigned q = threadIdx.x; q < rows; q += blockDim.x) {
      const unsigned b = lb[q];
      const i64 dst = (i64)lo[b] + (q - tst[b]);
      ikey[dst] = lk[q];
      irow[dst] = lr[q];
    }
    __syncthreads();
    for (unsigned b = threadIdx.x; b < nb; b += blockDim.x) lo[b] += tcnt[b];
    __syncthreads();
  }
}

// Second level of a two-level partition (tables of many regions: one scatter over thousands of bins wrote every
// row to its own cache line): one workgroup per coarse bin c splits its rows over the bin's 2^sh regions (an LDS
// counting pass, then ranked writes to 2^sh growing runs) and publishes the regions' bases; workgroup Pc carries the
// kEmpty rows to bin P.
__global__ __launch_bounds__(1024) void jpart_sub_kernel(const u64* __restrict__ ikey1, const unsigned* __restrict__ irow1,
                                                         const i64* __restrict__ cbase, u64 mask, int sh, unsigned Pc,
                                                         unsigned P, i64* __restrict__ bbase, u64* __restrict__ ikey2,
                                                         unsigned* __restrict__ irow2) {
  __shared__ unsigned sc[1024], so[1024];
  const unsigned c = blockIdx.x;
  const i64 i0 = cbase[c], i1 = cbase[c + 1];
  if (c == Pc) {
    for (i64 p = i0 + threadIdx.x; p < i1; p += blockDim.x) {
      ikey2[p] = ikey1[p];
      irow2[p] = irow1[p];
    }
    if (threadIdx.x == 0) {
      bbase[P] = i0;
      bbase[P + 1] = i1;
    }
    return;
  }
  const unsigned S = 1u << sh, sm = S - 1;
  for (unsigned j = threadIdx.x; j < S; j += blockDim.x) sc[j] = 0;
  __syncthreads();
  constexpr int U = 8;
  for (i64 c0 = i0; c0 < i1; c0 += (i64)U * blockDim.x) {
    u64 k[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 p = c0 + (i64)j * blockDim.x + threadIdx.x;
      k[j] = p < i1 ? ikey1[p] : 0;
    }
#pragma unroll
    for (int j = 0; j < U; ++j)
      if (c0 + (i64)j * blockDim.x + threadIdx.x < i1)
        atomicAdd(&sc[(unsigned)((mix64(k[j]) & mask) >> kJRegionBits) & sm], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned acc = 0;
    for (unsigned j = 0; j < S; ++j) {
      so[j] = acc;
      bbase[((i64)c << sh) + j] = i0 + acc;
      acc += sc[j];
    }
  }
  __syncthreads();
  for (i64 c0 = i0; c0 < i1; c0 += (i64)U * blockDim.x) {
    u64 k[U];
    unsigned r[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const i64 p = c0 + (i64)j * blockDim.x + threadIdx.x;
      k[j] = p < i1 ? ikey1[p] : 0;
      r[j] = p < i1 ? irow1[p] : 0u;
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (c0 + (i64)j * blockDim.x + threadIdx.x >= i1) continue;
      const i64 pos = i0 + atomicAdd(&so[(unsigned)((mix64(k[j]) & mask) >> kJRegionBits) & sm], 1u);
      ikey2[pos] = k[j];
      irow2[pos] = r[j];
    }
  }
}

// one workgroup per region (blockIdx.x < P) builds it in LDS; workgroup P takes the kEmpty rows. islot / irank per
// row in partition order; *fail when a region would be left without an empty slot (its chains could not end).
// bloom: the table's probe filter (nullptr: none), 2^bshift slots per word, bshift <= kJRegionBits.
__global__ __launch_bounds__(kJPartThreads) void join_region_build_kernel(
    const u64* __restrict__ ikey, const unsigned* __restrict__ irow, const i64* __restrict__ bbase, u64 mask,
    unsigned P, JSlot* __restrict__ tab, int* __restrict__ islot, unsigned* __restrict__ irank,
    unsigned long long* ndup, unsigned* fail, unsigned long long* __restrict__ bloom, int bshift) {
  __shared__ u64 lkey[kJRegion];
  __shared__ unsigned lcnt[kJRegion], lpay[kJRegion];
  __shared__ u64 lbl[kJRegion / 4];
  __shared__ unsigned nclaim, ndl;
  const unsigned b = blockIdx.x;
  const i64 p0 = bbase[b], p1 = bbase[b + 1];
  if (b == P) {                                  // rows whose key is the kEmpty marker: the sentinel slot
    const u64 sent = mask + 1;
    unsigned d = 0;
    for (i64 p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
      const unsigned r = __hip_atomic_fetch_add(&tab[sent].cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (r == 0) tab[sent].pay = irow[p];
      islot[p] = (int)sent;
      irank[p] = r;
      d += r != 0;
    }
    if (d) __hip_atomic_fetch_add(ndup, (unsigned long long)d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const u64 rm = kJRegion - 1;
  const int wpr = bloom ? (int)(kJRegion >> bshift) : 0;   // filter words of this region
  // the first IPT items of every thread are loaded before the LDS image is cleared (their latency overlaps it),
  // and each later round's loads are all in flight before its inserts
  constexpr int IPT = 8;
  u64 kk[IPT];
  unsigned rr[IPT];
  auto load = [&](i64 c0) {
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const i64 p = c0 + j * kJPartThreads + threadIdx.x;
      if (p < p1) {
        kk[j] = ikey[p];
        rr[j] = irow[p];
      }
    }
  };
  load(p0);
  for (unsigned s = threadIdx.x; s < kJRegion; s += blockDim.x) {
    lkey[s] = kEmpty;
    lcnt[s] = 0;
  }
  for (int w = threadIdx.x; w < wpr; w += blockDim.x) lbl[w] = 0;
  if (threadIdx.x == 0) {
    nclaim = 0;
    ndl = 0;
  }
  __syncthreads();
  const i64 sbase = (i64)b << kJRegionBits;
  unsigned d = 0, cl = 0;
  bool bad = false;
  for (i64 c0 = p0; c0 < p1; c0 += (i64)IPT * kJPartThreads) {
#pragma unroll
    for (int j = 0; j < IPT; ++j) {
      const i64 p = c0 + j * kJPartThreads + threadIdx.x;
      if (p >= p1) continue;
      const u64 k = kk[j];
      u64 s = mix64(k) & rm;
      unsigned r = 0;
      bool done = false;
      for (u64 it = 0; it < kJRegion; ++it) {
        const u64 prev = atomicCAS(&lkey[s], kEmpty, k);
        if (prev == kEmpty) {
          lpay[s] = rr[j];
          ++cl;
          done = true;
          break;
        }
        if (prev == k) {
          r = atomicAdd(&lcnt[s], 1u) + 1u;
          done = true;
          break;
        }
        s = (s + 1) & rm;
      }
      bad |= !done;
      islot[p] = (int)(sbase + (i64)s);
      irank[p] = r;
      d += r != 0;
    }
    if (c0 + (i64)IPT * kJPartThreads < p1) load(c0 + (i64)IPT * kJPartThreads);
  }
  if (cl) atomicAdd(&nclaim, cl);
  if (d) atomicAdd(&ndl, d);
  if (bad) atomicOr(&ndl, 0x80000000u);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (nclaim >= kJRegion || (ndl & 0x80000000u))
      __hip_atomic_store(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned dd = ndl & 0x7fffffffu;
    if (dd) __hip_atomic_fetch_add(ndup, (unsigned long long)dd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // the region out (16-B slot stores, coalesced), and its filter words from the LDS image
  for (unsigned s = threadIdx.x; s < kJRegion; s += blockDim.x) {
    const u64 k = lkey[s];
    tab[sbase + s] = JSlot{k, lcnt[s], lpay[s]};
    if (wpr && k != kEmpty) {
      const u64 f = mix64(k);
      atomicOr(&lbl[(f & rm) >> bshift], bloom_bits(f));
    }
  }
  if (wpr) {
    __syncthreads();
    for (int w = threadIdx.x; w < wpr; w += blockDim.x) bloom[(i64)b * wpr + w] = lbl[w];
  }
}

// rows of rank > 0 of a partitioned build: perm[run start + rank] = row (the rows in partition order)
__global__ __launch_bounds__(256) void join_perm_items_kernel(const int* __restrict__ islot,
                                                              const unsigned* __restrict__ irank,
                                                              const unsigned* __restrict__ irow, i64 n,
                                                              const unsigned long long* ndup, const JSlot* tab,
                                                              i64* __restrict__ perm) {
  if (*ndup == 0) return;
  for (i64 p = (i64)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (i64)gridDim.x * blockDim.x) {
    const unsigned r = irank[p];
    if (r == 0) continue;
    perm[(i64)tab[islot[p]].pay + r] = (i64)irow[p];
  }
}

__global__ __launch_bounds__(256) void join_bloom_kernel(const JSlot* __restrict__ tab, u64 mask, int shift, i64 W,
                                                         unsigned long long* __restrict__ bloom) {
  const i64 w = (i64)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= W) return;
  u64 bits = 0;
  const i64 s0 = w << shift, s1 = (w + 1) << shift;
  for (i64 s = s0; s < s1; ++s) {
    const u64 k = tab[s].key;
    if (k == kEmpty) continue;
    const u64 f = mix64(k);
    const i64 hw = (i64)((f & mask) >> shift);
    if (hw == w) bits |= bloom_bits(f);
    else __hip_atomic_fetch_or(bloom + hw, bloom_bits(f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (bits) __hip_atomic_fetch_or(bloom + w, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int kJTile = 4096;   // probe rows per workgroup tile (256 threads x 16)


// probe: matches (cnt) and payload per probe row, and the match total of each 4096-row tile. The first-slot
// reads of all 16 rows of a thread are issued together (16 independent 16-byte loads in flight); only rows
// whose first slot holds another key walk the probe chain.
__global__ __launch_bounds__(256) void join_probe_kernel(const u64* __restrict__ keys, i64 m,
                                                         const JSlot* __restrict__ tab, u64 mask,
                                                         unsigned* __restrict__ cnt, unsigned* __restrict__ pay,
                                                         i64* __restrict__ tile_sum,
                                                         const unsigned long long* __restrict__ bloom, int bshift) {
  __shared__ u64 ws[4];   // match totals in 64 bits: a skewed many-to-many tile can exceed 2^32 pairs
  constexpr int J = kJTile / 256;
  const i64 t0 = (i64)blockIdx.x * kJTile;
  u64 local = 0;
  u64 k[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const i64 i = t0 + j * 256 + threadIdx.x;
    k[j] = i < m ? keys[i] : 0;
  }
  u64 sl[J];
  JSlot e[J];
  bool may[J];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const u64 f = mix64(k[j]);
    sl[j] = k[j] == kEmpty ? mask + 1 : (f & mask);
    may[j] = true;
    if (bloom && k[j] != kEmpty) {
      const u64 b = bloom_bits(f);
      may[j] = (bloom[sl[j] >> bshift] & b) == b;
    }
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (may[j]) e[j] = tab[sl[j]];
    else e[j] = JSlot{kEmpty, 0u, 0u};              // filtered out: reads as an empty first slot (no match)
  }
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const i64 i = t0 + j * 256 + threadIdx.x;
    if (i >= m) continue;
    unsigned c = 0, p = 0;
    if (e[j].key == k[j]) {   // total rows: the extras + the claiming row (the kEmpty slot counts all of its rows)
      c = e[j].cnt + (k[j] != kEmpty ? 1u : 0u);
      p = e[j].pay;
    } else if (e[j].key != kEmpty && k[j] != kEmpty) {
      u64 s = jnext(sl[j], mask);
      for (u64 it = 0; it <= jregion_mask(mask); ++it) {   // a region always keeps an empty slot (the build checks it)
        const JSlot x = tab[s];
        if (x.key == k[j]) {
          c = x.cnt + 1u;
          p = x.pay;
          break;
        }
        if (x.key == kEmpty) break;
        s = jnext(s, mask);
      }
    }
    cnt[i] = c;
    pay[i] = p;
    local += c;
  }
  // workgroup sum
  for (int d = 32; d > 0; d >>= 1) local += __shfl_down(local, d, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = local;
  __syncthreads();
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = (i64)(ws[0] + ws[1] + ws[2] + ws[3]);
}

// expand: tile bases = exclusive scan of tile_sum; inside a tile, a block scan per 256-row slab gives each probe
// row its output offset, so pairs come out probe-major with no full-length scan pass
__global__ __launch_bounds__(256) void join_expand_kernel(const unsigned* __restrict__ cnt,
                                                          const unsigned* __restrict__ pay, i64 m,
                                                          const i64* __restrict__ tile_base,
                                                          const i64* __restrict__ perm, i64* __restrict__ bidx,
                                                          i64* __restrict__ pidx) {
  __shared__ u64 wsum[4];           // 64-bit prefixes (see join_probe_kernel)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const i64 t0 = (i64)blockIdx.x * kJTile;
  i64 base = tile_base[blockIdx.x];
  for (int j = 0; j < kJTile / 256; ++j) {
    const i64 i = t0 + j * 256 + threadIdx.x;
    const u64 c = i < m ? (u64)cnt[i] : 0ull;
    u64 x = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const u64 y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    u64 before = 0, slab = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const u64 t = wsum[w];
      before += w < wave ? t : 0u;
      slab += t;
    }
    const i64 o = base + (i64)(before + x - c);
    if (c == 1) {
      const unsigned p = pay[i];
      bidx[o] = (i64)p;
      pidx[o] = i;
    } else if (c > 1) {
      const i64 b0 = (i64)pay[i];
      for (u64 q = 0; q < c; ++q) {
        bidx[o + q] = perm[b0 + q];
        pidx[o + q] = i;
      }
    }
    base += (i64)slab;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- partition + pack (shuffle sink)
// dest[i] in [0, P): per-workgroup histograms (bucket-major), then a stable-within-chunk scatter of row ids
__global__ __launch_bounds__(1024) void part_hist_kernel(const i64* __restrict__ dest, i64 n, i64 rpw, int P,
                                                         unsigned* __restrict__ hist) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  unsigned* h = reinterpret_cast<unsigned*>(lds_raw);
  for (int i = threadIdx.x; i < P; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const i64 r0 = (i64)blockIdx.x * rpw, r1 = std::min<i64>(n, r0 + rpw);
  for (i64 i = r0 + threadIdx.x; i < r1; i += blockDim.x) atomicAdd(h + dest[i], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < P; b += blockDim.x) hist[(size_t)b * gridDim.x + blockIdx.x] = h[b];
}

// Rows are placed in input order within each destination: the chunk is walked in 1024-row tiles; inside a tile
// each wave ranks its lanes per destination with ballots (lanes of one destination, in lane order), the waves'
// counts are prefix-summed in LDS, and a running per-destination base carries over to the next tile.
__global__ __launch_bounds__(1024) void part_scatter_kernel(const i64* __restrict__ dest, i64 n, i64 rpw, int P,
                                                            const unsigned* __restrict__ hist,
                                                            const i64* __restrict__ bstart, i64* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  unsigned* base = reinterpret_cast<unsigned*>(lds_raw);   // [P] running base within this chunk
  unsigned* wc = base + P;                                  // [16][P] per-wave counts of the current tile
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int b = threadIdx.x; b < P; b += blockDim.x) base[b] = 0;
  const i64 r0 = (i64)blockIdx.x * rpw, r1 = std::min<i64>(n, r0 + rpw);
  for (i64 t0 = r0; t0 < r1; t0 += 1024) {
    for (int j = threadIdx.x; j < 16 * P; j += blockDim.x) wc[j] = 0;
    __syncthreads();
    const i64 i = t0 + threadIdx.x;
    const bool valid = i < r1;
    const int d = valid ? (int)dest[i] : -1;
    // rank among this wave's lanes of the same destination
    u64 todo = __ballot(valid);
    int rank = 0;
    while (todo) {
      const int leader = __ffsll((long long)todo) - 1;
      const int dl = __shfl(d, leader, 64);
      const u64 m = __ballot(valid && d == dl);
      if (d == dl && valid) rank = __popcll(m & ((1ull << lane) - 1));
      if (lane == leader) wc[wave * P + dl] = __popcll(m);
      todo &= ~m;
    }
    __syncthreads();
    if (valid) {
      unsigned before = 0;
      for (int w = 0; w < wave; ++w) before += wc[w * P + d];
      perm[bstart[d] + hist[(size_t)d * gridDim.x + blockIdx.x] + base[d] + before + rank] = i;
    }
    __syncthreads();
    for (int b = threadIdx.x; b < P; b += blockDim.x) {
      unsigned s = 0;
      for (int w = 0; w < 16; ++w) s += wc[w * P + b];
      base[b] += s;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- key hashing
// out = mix64((x ^ y) + GOLD) over int64 columns (y optional): the engine's join / partition key hash
// (execution/kernels.py mix64 / column_to_int64, = netsdb_amd._native.hash64) as ONE streaming pass, where the torch
// expression is eleven elementwise kernels over the column. 2 rows per thread (16-B loads / stores).
__global__ __launch_bounds__(256) void mix64_kernel(const u64* __restrict__ x, const u64* __restrict__ y, u64* out, i64 n) {
  const i64 stride = (i64)gridDim.x * blockDim.x * 2;
  for (i64 i = ((i64)blockIdx.x * blockDim.x + threadIdx.x) * 2; i < n; i += stride) {
    if (i + 1 < n) {
      ulonglong2 a = *reinterpret_cast<const ulonglong2*>(x + i);
      if (y) {
        const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(y + i);
        a.x ^= b.x;
        a.y ^= b.y;
      }
      *reinterpret_cast<ulonglong2*>(out + i) = make_ulonglong2(mix64(a.x + 0x9E3779B97F4A7C15ull),
                                                                mix64(a.y + 0x9E3779B97F4A7C15ull));
    } else {
      const u64 a = x[i] ^ (y ? y[i] : 0ull);
      out[i] = mix64(a + 0x9E3779B97F4A7C15ull);
    }
  }
}

// ---------------------------------------------------------------- stable stream compaction (mask -> row ids)
// The row ids of the nonzero bytes of a 0/1 byte mask, in row order (a filter's selection): per-tile counts, one
// scan, then every tile writes its ids at its offset, each wave a contiguous run per 64 rows (ballot + popcount).
constexpr int CT_ROWS = 8192;   // rows per tile (one 256-thread workgroup)

__global__ __launch_bounds__(256) void compact_count_kernel(const unsigned char* __restrict__ mask, i64 n,
                                                            unsigned* __restrict__ cnt) {
  const i64 t0 = (i64)blockIdx.x * CT_ROWS;
  unsigned c = 0;
  for (int r = threadIdx.x * 16; r < CT_ROWS; r += 256 * 16) {
    const i64 i = t0 + r;
    if (i + 16 <= n) {
      const uint4 w = *reinterpret_cast<const uint4*>(mask + i);      // 16 bytes of 0 / 1
      const u64 a = ((u64)w.y << 32) | w.x, b = ((u64)w.w << 32) | w.z;
      // every nonzero byte -> 1, then the 16 bytes summed by one multiply
      const u64 lo7 = 0x7F7F7F7F7F7F7F7Full, hi = 0x8080808080808080ull;
      const u64 na = ((((a & lo7) + lo7) | a) & hi) >> 7, nb = ((((b & lo7) + lo7) | b) & hi) >> 7;
      c += (unsigned)(((na + nb) * 0x0101010101010101ull) >> 56);
    } else {
      for (i64 k = i; k < n && k < i + 16; ++k) c += mask[k] != 0;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  __shared__ unsigned ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// exclusive scan of T tile counts (one workgroup): off[t], off[T] = total
__global__ __launch_bounds__(1024) void compact_scan_kernel(const unsigned* __restrict__ cnt, int T, i64* __restrict__ off) {
  __shared__ i64 part[1024];
  const int per = (T + 1023) / 1024;
  const int b = threadIdx.x * per;
  i64 s = 0;
  for (int k = b; k < b + per && k < T; ++k) s += cnt[k];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const i64 v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  i64 run = part[threadIdx.x] - s;
  for (int k = b; k < b + per && k < T; ++k) {
    off[k] = run;
    run += cnt[k];
  }
  if (threadIdx.x == 1023) off[T] = part[1023];
}

__global__ __launch_bounds__(256) void compact_write_kernel(const unsigned char* __restrict__ mask, i64 n,
                                                            const i64* __restrict__ off, i64* __restrict__ out) {
  __shared__ unsigned wc[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const i64 t0 = (i64)blockIdx.x * CT_ROWS;
  i64 base = off[blockIdx.x];
  const u64 lt = (1ull << lane) - 1;
  for (int r = 0; r < CT_ROWS; r += 256) {
    const i64 i = t0 + r + threadIdx.x;
    const bool on = i < n && mask[i] != 0;
    const u64 bal = __builtin_amdgcn_ballot_w64(on);
    if (lane == 0) wc[wave] = (unsigned)__builtin_popcountll(bal);
    __syncthreads();
    unsigned before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      before += w < wave ? wc[w] : 0u;
      tot += wc[w];
    }
    if (on) out[base + before + __builtin_popcountll(bal & lt)] = i;
    base += tot;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- clustered-key aggregation (runs of equal keys)
// A group-by whose key column arrives ordered (TPC-H lineitem is stored by l_orderkey, so the late lineitems' order
// keys of Q04 and the (orderkey, date, priority) keys of Q03's probe come out of a scan in runs) needs no hash table:
// every run of equal consecutive keys is one group. Three passes, no atomics on data: run heads counted per tile
// (with a flag for any descending step: unordered keys go to the hash path), the heads' row ids written in order
// (the compaction's tile scan), and one thread per group reduces its run. A descending step anywhere means equal keys
// may not be adjacent, so the caller falls back to hash aggregation; a non-descending column has each key in one run.
__device__ __forceinline__ bool run_head(const u64* __restrict__ k, i64 i) { return i == 0 || k[i] != k[i - 1]; }

__global__ __launch_bounds__(256) void run_count_kernel(const u64* __restrict__ k, i64 n, unsigned* __restrict__ cnt,
                                                        unsigned long long* __restrict__ desc) {
  const i64 t0 = (i64)blockIdx.x * CT_ROWS;
  unsigned c = 0;
  bool down = false;
  for (int r = threadIdx.x; r < CT_ROWS; r += 256) {
    const i64 i = t0 + r;
    if (i >= n) break;
    const u64 x = k[i];
    const u64 p = i > 0 ? k[i - 1] : x;
    c += (i == 0 || x != p) ? 1u : 0u;
    down |= (long long)x < (long long)p;              // int64 order (a key column may hold negative values)
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  __shared__ unsigned ws[4];
  __shared__ int sdown;
  if (threadIdx.x == 0) sdown = 0;
  __syncthreads();
  if (down) sdown = 1;
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    cnt[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
    if (sdown) atomicOr(desc, 1ull);
  }
}

__global__ __launch_bounds__(256) void run_write_kernel(const u64* __restrict__ k, i64 n, const i64* __restrict__ off,
                                                        const unsigned long long* __restrict__ desc,
                                                        i64* __restrict__ heads) {
  if (*desc) return;                                   // unordered: the caller takes the hash path
  __shared__ unsigned wc[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const i64 t0 = (i64)blockIdx.x * CT_ROWS;
  i64 base = off[blockIdx.x];
  const u64 lt = (1ull << lane) - 1;
  for (int r = 0; r < CT_ROWS; r += 256) {
    const i64 i = t0 + r + threadIdx.x;
    const bool on = i < n && run_head(k, i);
    const u64 bal = __builtin_amdgcn_ballot_w64(on);
    if (lane == 0) wc[wave] = (unsigned)__builtin_popcountll(bal);
    __syncthreads();
    unsigned before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      before += w < wave ? wc[w] : 0u;
      tot += wc[w];
    }
    if (on) heads[base + before + __builtin_popcountll(bal & lt)] = i;
    base += tot;
    __syncthreads();
  }
}

// group g = rows [heads[g], heads[g + 1]) (the last ends at n): its key, row count and F reduced values (vals read in
// place: element (row, f) at vals[row * rs + f * cs]); op 0 sum, 1 min, 2 max — in row order, as a sequential fold
template <typename VT>
__global__ __launch_bounds__(256) void run_reduce_kernel(const u64* __restrict__ k, const VT* __restrict__ vals,
                                                         i64 rs, i64 cs, int F, int op, i64 n,
                                                         const i64* __restrict__ heads, const i64* __restrict__ ng,
                                                         const unsigned long long* __restrict__ desc,
                                                         i64* __restrict__ okey, VT* __restrict__ oagg,
                                                         i64* __restrict__ ocnt) {
  if (*desc) return;
  const i64 G = *ng;
  for (i64 g = (i64)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (i64)gridDim.x * blockDim.x) {
    const i64 lo = heads[g], hi = g + 1 < G ? heads[g + 1] : n;
    okey[g] = (i64)k[lo];
    ocnt[g] = hi - lo;
    for (int f = 0; f < F; ++f) {
      const VT* p = vals + f * cs;
      VT acc = p[lo * rs];
      for (i64 r = lo + 1; r < hi; ++r) {
        const VT x = p[r * rs];
        acc = op == 0 ? acc + x : (op == 1 ? (x < acc ? x : acc) : (x > acc ? x : acc));
      }
      oagg[g * F + f] = acc;
    }
  }
}

// ---------------------------------------------------------------- host launchers
// rows staged per scatter pass: a multiple of 1024, <= 4096, staging <= budget bytes
inline int stage_rows(int F, int budget = 48 * 1024, int nthr = 512) {
  const int t = (int)(budget / (14 + 8 * F)) / 256 * 256;   // wide rows (F up to 16): tiles below one row per thread
  return std::max(256, std::min(4 * nthr, t));
}

// level-1 histogram / scatter workgroups (one per CU), >= 16 Ki rows each
inline int agg_groups(long long n) { return (int)std::min<long long>(256, std::max<long long>(1, (n + 16383) / 16384)); }

// phase 0: every kernel (the device decides LOW / PART); phased launches let the host size the PART scratch only when
// the PART path runs: 1 = init + sample + LOW, 2 = PART (its table initialised first), 3 = emit + inverse fix-up.
// out: [reps ocap | aggs ocap*F | cnt ocap | slot_of_gid ocap | first ocap] (ocap: the groups the run may create);
// inv_v: [n] per-row group ids (want_inv), shared by every phase.
template <typename VT, int OP>
int agg_launch_t(const void* keys, const void* vals, i64 n, int F, int want_inv, int want_first, void* meta_v, void* glow_v,
                 i64 gcap_low, void* gpart_v, i64 gcap_part, void* out_v, void* inv_v, i64 ocap, int phase, void* work_v,
                 int pbits, int lcap_low, int lcap_part, int low_thr, int lcap_mid, i64 rs, i64 cs, hipStream_t st) {
  AggMeta* meta = reinterpret_cast<AggMeta*>(meta_v);
  // glow / gpart: [key (cap+1) | acc (cap+1)*F | cnt (cap+1) | gid (cap+1)] u64 words, preset by the caller
  auto mk = [&](void* base, i64 cap) {
    GTable t;
    u64* p = reinterpret_cast<u64*>(base);
    t.key = p;
    t.acc = p + (cap + 1);
    t.cnt = t.acc + (cap + 1) * F;
    t.rmin = t.cnt + (cap + 1);
    t.gid_of_slot = reinterpret_cast<i64*>(t.rmin + (cap + 1));
    t.mask = (u64)(cap - 1);
    return t;
  };
  GTable glow = mk(glow_v, gcap_low), gpart = mk(gpart_v, gcap_part);
  glow.occ = &meta->occ_low;
  gpart.occ = &meta->occ_part;
  i64* ob = reinterpret_cast<i64*>(out_v);   // [reps ocap | aggs ocap*F | cnt ocap | slot_of_gid ocap | first ocap]
  AggOut o;
  o.reps = ob;
  o.aggs = reinterpret_cast<u64*>(ob + ocap);
  o.cnt = ob + ocap + ocap * F;
  o.slot_of_gid = o.cnt + ocap;
  o.first = o.slot_of_gid + ocap;
  o.inv = want_inv ? reinterpret_cast<i64*>(inv_v) : nullptr;
  const u64* k = reinterpret_cast<const u64*>(keys);
  const VT* v = reinterpret_cast<const VT*>(vals);
  const size_t lbytes_low = (size_t)lcap_low * (20 + 8 * F);
  const size_t lbytes_part = (size_t)lcap_part * (20 + 8 * F);

  if (phase == 0 || phase == 1) {
    hipLaunchKernelGGL(agg_init_kernel, dim3(512), dim3(256), 0, st, reinterpret_cast<u64*>(glow_v), gcap_low,
                       phase == 0 ? reinterpret_cast<u64*>(gpart_v) : nullptr, gcap_part, F, acc_identity<VT, OP>(), meta);
    u64* sbuf = reinterpret_cast<u64*>(meta) + sizeof(AggMeta) / 8;   // [4096] after the meta words
    hipLaunchKernelGGL(agg_sample_gather_kernel, dim3(kSample / 64), dim3(64), 0, st, k, n, sbuf);
    hipLaunchKernelGGL(agg_sample_kernel, dim3(1), dim3(1024), 0, st, sbuf, n, low_thr, lcap_mid / 2, meta);
    const int gl = (int)std::min<i64>(1024, std::max<i64>(1, (n + 2047) / 2048));
    hipLaunchKernelGGL((agg_low_kernel<VT, OP, 256, 1>), dim3(gl), dim3(256), lbytes_low, st, k, v, n, F, rs, cs, lcap_low,
                       glow, meta, o);
    if (lcap_mid > 0)   // returns at once unless the sample chose the MID path
      hipLaunchKernelGGL((agg_low_kernel<VT, OP, 1024, 2>), dim3(256), dim3(1024), (size_t)lcap_mid * (20 + 8 * F), st, k,
                         v, n, F, rs, cs, lcap_mid, glow, meta, o);
  }
  if (phase == 2)
    hipLaunchKernelGGL(agg_init_kernel, dim3(512), dim3(256), 0, st, (u64*)nullptr, gcap_low,
                       reinterpret_cast<u64*>(gpart_v), gcap_part, F, acc_identity<VT, OP>(), (AggMeta*)nullptr);
  // PART: work buffers [hist P*G u32 | tot P | bstart P+1 | pkey n | pval n*F | prow n (i32) | qkey | qval | qrow]
  const int P = 1 << pbits;
  const int G = agg_groups(n);
  const i64 rpw = (((n + G - 1) / G) + 1) & ~(i64)1;   // even: every workgroup's range starts 16-byte aligned
  char* w = reinterpret_cast<char*>(work_v);
  unsigned* hist = reinterpret_cast<unsigned*>(w);
  i64* tot = reinterpret_cast<i64*>(w + (((size_t)P * G * 4 + 15) & ~(size_t)15));
  i64* bstart = tot + P;
  u64* pkey = reinterpret_cast<u64*>(bstart + P + 2);
  VT* pval = reinterpret_cast<VT*>(pkey + n);
  int* prow = reinterpret_cast<int*>(pval + n * F);
  u64* qkey = reinterpret_cast<u64*>(prow + ((n + 1) & ~(i64)1));
  VT* qval = reinterpret_cast<VT*>(qkey + n);
  int* qrow = reinterpret_cast<int*>(qval + n * F);
  if (!want_inv && !want_first) prow = qrow = nullptr;   // no row ids through the partitions
  const int T = stage_rows(F, 96 * 1024, 1024);   // level-1 scatter: one 1024-thread workgroup per CU
  const size_t stage_bytes = (size_t)T * (14 + 8 * F);
  const int T2 = std::min(2048, stage_rows(F, 96 * 1024, 1024));   // bucket kernel's sub-partition tiles (2 rows / thread)
  const size_t lds_bucket = std::max((size_t)T2 * (14 + 8 * F), lbytes_part);
  if (phase == 0 || phase == 2) {
    hipLaunchKernelGGL(agg_hist_kernel, dim3(G), dim3(1024), (size_t)P * 4, st, k, n, rpw, pbits, hist, meta);
    hipLaunchKernelGGL(scan_rows_kernel, dim3(P), dim3(1024), 0, st, hist, G, tot, meta, 1);
    hipLaunchKernelGGL(scan_tot_kernel, dim3(1), dim3(1024), 0, st, tot, P, bstart, meta, 1);
    hipLaunchKernelGGL((agg_scatter_kernel<VT>), dim3(G), dim3(1024), stage_bytes, st, k, v, rs, cs, n, F, rpw, pbits, T,
                       hist, bstart, pkey, pval, prow, meta);
    hipLaunchKernelGGL((agg_bucket_kernel<VT, OP>), dim3(P), dim3(1024), lds_bucket, st, pkey, pval, prow, F, lcap_part,
                       pbits, T2, n, bstart, qkey, qval, qrow, gpart, meta, o);
  }
  if (phase == 0 || phase == 2 || phase == 3) {
    // a phase-3 (LOW) emit never reads the PART table: take_part() is false there
    hipLaunchKernelGGL((agg_emit_kernel<VT, OP>),
                       dim3((unsigned)(((phase == 3 ? gcap_low : std::max(gcap_low, gcap_part)) + 2 + 255) / 256)),
                       dim3(256), 0, st, glow, gpart, F, meta, o);
    if (want_inv)
      hipLaunchKernelGGL(agg_fix_inv_kernel, dim3((unsigned)std::min<i64>(2048, (n + 255) / 256)), dim3(256), 0, st,
                         o.inv, n, glow.gid_of_slot, gpart.gid_of_slot, meta);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- multi-column gather
// dst_c[i] = src_c[idx[i]] for up to kTakeCols columns of one row selection in ONE launch (a join output's columns
// read together: Q02's lazily gathered columns were ~170 index_select launches per query, each ~6 us of host time).
// Row width per column 1, 2, 4, 8 or 16 bytes (a column of wider rows is split by the host into 16-B words, a
// multiple of them per row). blockIdx.y = column: the width switch is uniform per workgroup. Out-of-range ids write
// zeros and raise *bad (the host checks it with the batch's other reads, never a fault).
constexpr int kTakeCols = 48;
struct TakeCol {
  const char* src;
  char* dst;
  long long nsrc;    // rows of the source
  int w;             // bytes per element: 1, 2, 4, 8, 16
  int per;           // elements per row (row = per * w bytes)
};
struct TakeArgs {
  TakeCol c[kTakeCols];
};

template <typename T>
__device__ __forceinline__ void take_rows(const TakeCol& c, const i64* __restrict__ idx, i64 n, int* bad) {
  const T* __restrict__ src = reinterpret_cast<const T*>(c.src);
  T* __restrict__ dst = reinterpret_cast<T*>(c.dst);
  const i64 tot = n * c.per;
  for (i64 e = (i64)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (i64)gridDim.x * blockDim.x) {
    const i64 i = c.per == 1 ? e : e / c.per;
    const int q = c.per == 1 ? 0 : (int)(e - i * c.per);
    const i64 r = idx[i];
    if (r >= 0 && r < c.nsrc) {
      dst[e] = src[r * c.per + q];
    } else {
      dst[e] = T{};
      *bad = 1;
    }
  }
}

__global__ __launch_bounds__(256) void take_many_kernel(TakeArgs a, const i64* __restrict__ idx, i64 n, int* bad) {
  const TakeCol& c = a.c[blockIdx.y];
  switch (c.w) {
    case 1: take_rows<unsigned char>(c, idx, n, bad); break;
    case 2: take_rows<unsigned short>(c, idx, n, bad); break;
    case 4: take_rows<unsigned>(c, idx, n, bad); break;
    case 8: take_rows<u64>(c, idx, n, bad); break;
    default: take_rows<uint4>(c, idx, n, bad); break;
  }
}

}  // namespace nsdb_rel

using namespace nsdb_rel;

extern "C" {

// Byte size of the PART work buffer for (n, F, pbits).
long long nsdb_agg_work_bytes(long long n, int F, int pbits, int want_inv) {
  const long long P = 1LL << pbits;
  const long long G = agg_groups(n);
  (void)want_inv;
  return ((P * G * 4 + 15) & ~15LL) + 8 * (2 * P + 2) + 2 * (8 * n + 8 * n * F + 4 * (n + 1)) + 64;
}

// vt: 0 double, 1 int64; op: 0 sum, 1 min, 2 max. Value (i, f) is vals[i * vrs + f * vcs] (vrs = vcs = 0: row-major
// [n, F]).
int nsdb_hash_aggregate(const void* keys, const void* vals, long long n, int F, int vt, int op, int want_inv,
                        int want_first, void* meta, void* glow, long long gcap_low, void* gpart, long long gcap_part,
                        void* out, void* inv, long long ocap, int phase, void* work, int pbits, int lcap_low,
                        int lcap_part, int low_thr, int lcap_mid, long long vrs, long long vcs, hipStream_t st) {
  if (n <= 0) return 0;
  if (lcap_mid < 0 || (lcap_mid > 0 && ((lcap_mid & (lcap_mid - 1)) || (size_t)lcap_mid * (20 + 8 * F) > 160 * 1024 ||
                                        gcap_low < 2LL * kMidPMax * (lcap_mid / 2))))
    return (int)hipErrorInvalidValue;   // the MID table fits one CU's LDS; the global table holds every MID group
  if (phase < 0 || phase > 3 || ocap <= 0 || (want_inv && inv == nullptr)) return (int)hipErrorInvalidValue;
  if ((phase == 0 || phase == 2) && (ocap < n || work == nullptr || gpart == nullptr)) return (int)hipErrorInvalidValue;
  if (ocap < gcap_low + 1 && ocap < n) return (int)hipErrorInvalidValue;   // every LOW group needs an output row
  if (n >= (1LL << 31)) return (int)hipErrorInvalidValue;
  if (F < 0 || F > 16 || pbits < 0 || pbits > 10) return (int)hipErrorInvalidValue;
  auto pow2 = [](long long x) { return x > 0 && (x & (x - 1)) == 0; };
  if (!pow2(gcap_low) || !pow2(gcap_part) || !pow2(lcap_low) || !pow2(lcap_part)) return (int)hipErrorInvalidValue;
  if ((size_t)lcap_low * (20 + 8 * F) > 65536 || (size_t)lcap_part * (20 + 8 * F) > 131072) return (int)hipErrorInvalidValue;
  if ((size_t)stage_rows(F, 96 * 1024, 1024) * (14 + 8 * F) > 131072) return (int)hipErrorInvalidValue;
  if (F > 0 && (vrs < 0 || vcs < 0)) return (int)hipErrorInvalidValue;
  if (vrs == 0 && vcs == 0) {   // default: row-major [n, F]
    vrs = F;
    vcs = 1;
  }
#define NSDB_AGG(VT, OP) agg_launch_t<VT, OP>(keys, vals, n, F, want_inv, want_first, meta, glow, gcap_low, gpart, gcap_part, out, inv, ocap, phase, work, pbits, lcap_low, lcap_part, low_thr, lcap_mid, vrs, vcs, st)
  if (vt == 0) {
    if (op == 0) return NSDB_AGG(double, OP_SUM);
    if (op == 1) return NSDB_AGG(double, OP_MIN);
    if (op == 2) return NSDB_AGG(double, OP_MAX);
  } else if (vt == 1) {
    if (op == 0) return NSDB_AGG(i64, OP_SUM);
    if (op == 1) return NSDB_AGG(i64, OP_MIN);
    if (op == 2) return NSDB_AGG(i64, OP_MAX);
  }
#undef NSDB_AGG
  return (int)hipErrorInvalidValue;
}

int nsdb_take_many(const void* const* src, void* const* dst, const long long* nsrc, const int* w, const int* per,
                   int ncols, const long long* idx, long long n, int* bad, hipStream_t st) {
  if (ncols <= 0 || n <= 0) return 0;
  if (ncols > kTakeCols) return (int)hipErrorInvalidValue;
  TakeArgs a{};
  long long maxe = 0;
  for (int c = 0; c < ncols; ++c) {
    if (!(w[c] == 1 || w[c] == 2 || w[c] == 4 || w[c] == 8 || w[c] == 16) || per[c] < 1) return (int)hipErrorInvalidValue;
    a.c[c] = TakeCol{(const char*)src[c], (char*)dst[c], nsrc[c], w[c], per[c]};
    maxe = std::max(maxe, n * (long long)per[c]);
  }
  const unsigned gx = (unsigned)std::max<long long>(1, std::min<long long>(2048, (maxe + 255) / 256));
  hipLaunchKernelGGL(take_many_kernel, dim3(gx, (unsigned)ncols), dim3(256), 0, st, a, (const i64*)idx, (i64)n, bad);
  return (int)hipGetLastError();
}

// Partitioned build (tables of 2..kJPartMaxRegions regions): bytes of its workspace. Up to kJPartOneLevel regions
// the rows are partitioned straight into regions; beyond, into kJPartCoarse coarse bins first (sh = log2 of the
// regions per coarse bin), then split per coarse bin (jpart_sub_kernel).
constexpr long long kJPartMaxRegions = 8192;
constexpr unsigned kJPartOneLevel = 2048, kJPartCoarse = 256;
static void jpart_geometry(long long n, long long cap, unsigned& P, unsigned& G, long long& rpw, int& sh) {
  P = (unsigned)(cap >> kJRegionBits);
  G = (unsigned)std::max<long long>(1, std::min<long long>(1024, (n + 16383) / 16384));
  rpw = (n + G - 1) / G;
  sh = 0;
  if (P > kJPartOneLevel)
    while ((P >> sh) > kJPartCoarse) ++sh;
}
long long nsdb_jpart_work_bytes(long long n, long long cap) {
  unsigned P, G;
  long long rpw;
  int sh;
  jpart_geometry(n, cap, P, G, rpw, sh);
  const unsigned Pc = P >> sh;
  const long long hist = (((long long)(Pc + 1) * G * 4) + 15) & ~15LL;
  return hist + (long long)(Pc + 1) * 8 + (long long)(Pc + 2) * 8 + (long long)(P + 2) * 8 +
         n * (8 + 4 + 4 + 4) + (sh ? n * 12 : 0) + 64;
}

// tab: cap + 1 slots (any content: every region and the sentinel slot are written); ctr: 3 zeroed u64 {rows of rank
// > 0, run bump, fail}; bloom: W = cap >> bshift zeroed-or-not words (every word is written), or nullptr.
int nsdb_join_build_part(const void* keys, long long n, void* tab, long long cap, void* work,
                         unsigned long long* ctr, unsigned long long* bloom, int bshift, long long* perm, hipStream_t st) {
  if (n <= 0 || cap <= (long long)kJWholeWrap || (cap & (cap - 1)) != 0 || cap < 2 * n || cap >= (1LL << 31))
    return (int)hipErrorInvalidValue;
  unsigned P, G;
  long long rpw;
  int sh;
  jpart_geometry(n, cap, P, G, rpw, sh);
  if (P > kJPartMaxRegions || (bloom && (bshift < 2 || bshift > kJRegionBits))) return (int)hipErrorInvalidValue;
  const unsigned Pc = P >> sh;
  char* w = (char*)work;
  unsigned* hist = (unsigned*)w;
  w += (((long long)(Pc + 1) * G * 4) + 15) & ~15LL;
  i64* btot = (i64*)w;
  w += (long long)(Pc + 1) * 8;
  i64* cbase = (i64*)w;
  w += (long long)(Pc + 2) * 8;
  i64* bbase = (i64*)w;
  w += (long long)(P + 2) * 8;
  u64* ikey = (u64*)w;
  w += n * 8;
  int* islot = (int*)w;
  w += n * 4;
  unsigned* irank = (unsigned*)w;
  w += n * 4;
  unsigned* irow = (unsigned*)w;
  w += n * 4;
  u64* ikey1 = sh ? (u64*)w : ikey;
  unsigned* irow1 = sh ? (unsigned*)(w + n * 8) : irow;
  const u64 mask = (u64)(cap - 1);
  const size_t lds = (size_t)(Pc + 1) * 4;
  hipLaunchKernelGGL(jpart_hist_kernel, dim3(G), dim3(kJPartThreads), lds, st, (const u64*)keys, (i64)n, (i64)rpw, mask,
                     Pc, sh, hist, (JSlot*)tab);
  hipLaunchKernelGGL(jpart_colscan_kernel, dim3((Pc + 1 + 255) / 256), dim3(256), 0, st, hist, G, Pc + 1, btot);
  hipLaunchKernelGGL(jpart_totscan_kernel, dim3(1), dim3(1024), 0, st, (const i64*)btot, Pc + 1, sh ? cbase : bbase);
  if (sh && Pc + 1 <= (unsigned)kJStageBins)
    hipLaunchKernelGGL(jpart_scatter_staged_kernel, dim3(G), dim3(kJPartThreads), 0, st, (const u64*)keys, (i64)n,
                       (i64)rpw, mask, Pc, sh, (const unsigned*)hist, (const i64*)cbase, ikey1, irow1);
  else
    hipLaunchKernelGGL(jpart_scatter_kernel, dim3(G), dim3(kJPartThreads), lds, st, (const u64*)keys, (i64)n, (i64)rpw,
                       mask, Pc, sh, (const unsigned*)hist, (const i64*)(sh ? cbase : bbase), ikey1, irow1);
  if (sh)
    hipLaunchKernelGGL(jpart_sub_kernel, dim3(Pc + 1), dim3(1024), 0, st, (const u64*)ikey1, (const unsigned*)irow1,
                       (const i64*)cbase, mask, sh, Pc, P, bbase, ikey, irow);
  hipLaunchKernelGGL(join_region_build_kernel, dim3(P + 1), dim3(kJPartThreads), 0, st, (const u64*)ikey,
                     (const unsigned*)irow, (const i64*)bbase, mask, P, (JSlot*)tab, islot, irank, ctr,
                     (unsigned*)(ctr + 2), bloom, bshift);
  const unsigned gs = (unsigned)std::min<long long>(4096, (cap + 1 + 255) / 256);
  hipLaunchKernelGGL(join_runs_kernel, dim3(gs), dim3(256), 0, st, (JSlot*)tab, mask, (const unsigned long long*)ctr,
                     ctr + 1, (i64*)perm);
  const unsigned g = (unsigned)std::min<long long>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(join_perm_items_kernel, dim3(g), dim3(256), 0, st, (const int*)islot, (const unsigned*)irank,
                     (const unsigned*)irow, (i64)n, (const unsigned long long*)ctr, (const JSlot*)tab, (i64*)perm);
  return (int)hipGetLastError();
}

// Preset a join table's cap + 1 slots to {kEmpty, 0, 0}.
int nsdb_join_init(void* tab, long long cap, hipStream_t st) {
  if (cap <= 0) return (int)hipErrorInvalidValue;
  const long long nslots = cap + 1;
  const unsigned g = (unsigned)std::min<long long>(8192, (nslots + 255) / 256);
  hipLaunchKernelGGL(join_init_kernel, dim3(g), dim3(256), 0, st, (JSlot*)tab, (i64)nslots);
  return (int)hipGetLastError();
}

// Join build over n int64 keys: tab [cap + 1] 16-byte slots preset {kEmpty, 0, 0} (cap a power of two >= 2n).
int nsdb_join_insert(const void* keys, long long n, void* tab, long long cap, int* row_slot, unsigned* row_rank,
                     unsigned long long* ndup, unsigned* fail, hipStream_t st) {
  if (n <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) != 0 || cap < 2 * n || cap >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const unsigned g = (unsigned)std::min<long long>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(join_insert_kernel, dim3(g), dim3(256), 0, st, (const u64*)keys, n, (JSlot*)tab, (u64)(cap - 1),
                     row_slot, row_rank, ndup, fail);
  return (int)hipGetLastError();
}

// CSR runs of the repeated keys (device-guarded by *ndup; bump: one zeroed u64).
int nsdb_join_perm(const int* row_slot, const unsigned* row_rank, long long n, const unsigned long long* ndup,
                   unsigned long long* bump, void* tab, long long cap, long long* perm, hipStream_t st) {
  if (n <= 0) return 0;
  const unsigned gs = (unsigned)std::min<long long>(4096, (cap + 1 + 255) / 256);
  hipLaunchKernelGGL(join_runs_kernel, dim3(gs), dim3(256), 0, st, (JSlot*)tab, (u64)(cap - 1), ndup, bump, perm);
  const unsigned g = (unsigned)std::min<long long>(4096, (n + 255) / 256);
  hipLaunchKernelGGL(join_perm_kernel, dim3(g), dim3(256), 0, st, row_slot, row_rank, n, ndup, (const JSlot*)tab,
                     perm);
  return (int)hipGetLastError();
}

long long nsdb_join_tiles(long long m) { return (m + kJTile - 1) / kJTile; }

// cnt / pay [m] u32, tile_sum [nsdb_join_tiles(m)] i64
int nsdb_join_probe(const void* keys, long long m, const void* tab, long long cap, unsigned* cnt, unsigned* pay,
                    long long* tile_sum, const unsigned long long* bloom, int bshift, hipStream_t st) {
  if (m <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) != 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(join_probe_kernel, dim3((unsigned)nsdb_join_tiles(m)), dim3(256), 0, st, (const u64*)keys, m,
                     (const JSlot*)tab, (u64)(cap - 1), cnt, pay, tile_sum, bloom, bshift);
  return (int)hipGetLastError();
}

// the table's probe filter: W words (a power of two <= cap), bloom zeroed by the caller
int nsdb_join_bloom(const void* tab, long long cap, long long W, unsigned long long* bloom, hipStream_t st) {
  if (W <= 0 || (W & (W - 1)) != 0 || W > cap || (cap & (cap - 1)) != 0) return (int)hipErrorInvalidValue;
  int shift = 0;
  while ((W << shift) < cap) ++shift;
  hipLaunchKernelGGL(join_bloom_kernel, dim3((unsigned)((W + 255) / 256)), dim3(256), 0, st, (const JSlot*)tab,
                     (u64)(cap - 1), shift, (i64)W, bloom);
  return (int)hipGetLastError();
}

// tile_base: exclusive scan of tile_sum
int nsdb_join_expand(const unsigned* cnt, const unsigned* pay, long long m, const long long* tile_base,
                     const long long* perm, long long* bidx, long long* pidx, hipStream_t st) {
  if (m <= 0) return 0;
  hipLaunchKernelGGL(join_expand_kernel, dim3((unsigned)nsdb_join_tiles(m)), dim3(256), 0, st, cnt, pay, m, tile_base,
                     perm, bidx, pidx);
  return (int)hipGetLastError();
}

// Stable partition permutation: dest [n] in [0, P), P <= 2048. work: hist P*G u32 + tot P i64 + bstart P+1 i64.
long long nsdb_part_work_bytes(long long n, int P) {
  const long long G = std::min<long long>(256, std::max<long long>(1, (n + 16383) / 16384));
  return ((P * G * 4 + 15) & ~15LL) + 8 * (2 * P + 1) + 64;
}

int nsdb_partition_perm(const long long* dest, long long n, int P, void* work, long long* perm, long long* counts,
                        hipStream_t st) {
  if (n <= 0) return 0;
  if (P <= 0 || P > 2048 || n >= (1LL << 31)) return (int)hipErrorInvalidValue;
  const int G = (int)std::min<long long>(256, std::max<long long>(1, (n + 16383) / 16384));
  const long long rpw = (n + G - 1) / G;
  const size_t lds = (size_t)P * 4 * 17;
  if (lds > 163840) return (int)hipErrorInvalidValue;
  char* w = reinterpret_cast<char*>(work);
  unsigned* hist = reinterpret_cast<unsigned*>(w);
  long long* tot = reinterpret_cast<long long*>(w + (((size_t)P * G * 4 + 15) & ~(size_t)15));
  long long* bstart = tot + P;
  hipLaunchKernelGGL(part_hist_kernel, dim3(G), dim3(1024), (size_t)P * 4, st, dest, n, rpw, P, hist);
  hipLaunchKernelGGL(scan_rows_kernel, dim3(P), dim3(1024), 0, st, hist, G, tot, (const AggMeta*)nullptr, 0);
  hipLaunchKernelGGL(scan_tot_kernel, dim3(1), dim3(1024), 0, st, tot, P, bstart, (AggMeta*)nullptr, 0);
  hipLaunchKernelGGL(part_scatter_kernel, dim3(G), dim3(1024), lds, st, dest, n, rpw, P, hist, bstart, perm);
  if (counts) (void)hipMemcpyAsync(counts, tot, sizeof(long long) * P, hipMemcpyDeviceToDevice, st);
  return (int)hipGetLastError();
}

// Tiles of a compaction and its scratch (tile counts u32 + offsets i64 [T + 1]).
long long nsdb_compact_tiles(long long n) { return (n + nsdb_rel::CT_ROWS - 1) / nsdb_rel::CT_ROWS; }

// Phase 1: tile counts + offsets (off[T] = the number of set rows, which the caller reads to size the output).
int nsdb_compact_count(const unsigned char* mask, long long n, unsigned* cnt, long long* off, hipStream_t st) {
  const long long T = nsdb_compact_tiles(n);
  if (T <= 0 || T > (1LL << 30) || (reinterpret_cast<uintptr_t>(mask) & 15)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(compact_count_kernel, dim3((unsigned)T), dim3(256), 0, st, mask, n, cnt);
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, (int)T, off);
  return (int)hipGetLastError();
}

// Phase 2: the row ids, in order, at out[0 .. off[T]).
int nsdb_compact_write(const unsigned char* mask, long long n, const long long* off, long long* out, hipStream_t st) {
  const long long T = nsdb_compact_tiles(n);
  if (T <= 0) return 0;
  hipLaunchKernelGGL(compact_write_kernel, dim3((unsigned)T), dim3(256), 0, st, mask, n, off, out);
  return (int)hipGetLastError();
}

// Clustered-key aggregation, phase 1: run heads per tile and the descending-step flag. off has T + 2 words:
// off[T] = the number of runs (groups), off[T + 1] = nonzero when the keys are not ordered (the caller reads both).
int nsdb_run_count(const void* keys, long long n, unsigned* cnt, long long* off, hipStream_t st) {
  const long long T = nsdb_compact_tiles(n);
  if (T <= 0 || T > (1LL << 30)) return (int)hipErrorInvalidValue;
  hipMemsetAsync(off + T + 1, 0, sizeof(long long), st);
  hipLaunchKernelGGL(run_count_kernel, dim3((unsigned)T), dim3(256), 0, st, reinterpret_cast<const u64*>(keys), n, cnt,
                     reinterpret_cast<unsigned long long*>(off + T + 1));
  hipLaunchKernelGGL(compact_scan_kernel, dim3(1), dim3(1024), 0, st, cnt, (int)T, off);
  return (int)hipGetLastError();
}

// phase 2: heads[G] and the groups (keys, counts, F values reduced with op 0 sum / 1 min / 2 max); vt 0 f64, 1 i64
int nsdb_run_reduce(const void* keys, const void* vals, long long rs, long long cs, int F, int vt, int op, long long n,
                    const long long* off, long long G, long long* heads, long long* okey, void* oagg, long long* ocnt,
                    hipStream_t st) {
  const long long T = nsdb_compact_tiles(n);
  if (T <= 0) return 0;
  const u64* k = reinterpret_cast<const u64*>(keys);
  const unsigned long long* desc = reinterpret_cast<const unsigned long long*>(off + T + 1);
  hipLaunchKernelGGL(run_write_kernel, dim3((unsigned)T), dim3(256), 0, st, k, n, off, desc, heads);
  const unsigned blocks = (unsigned)std::max<long long>(1, std::min<long long>(16384, (G + 255) / 256));
  if (vt == 1)
    hipLaunchKernelGGL(run_reduce_kernel<long long>, dim3(blocks), dim3(256), 0, st, k,
                       reinterpret_cast<const long long*>(vals), rs, cs, F, op, n, heads, off + T, desc, okey,
                       reinterpret_cast<long long*>(oagg), ocnt);
  else
    hipLaunchKernelGGL(run_reduce_kernel<double>, dim3(blocks), dim3(256), 0, st, k,
                       reinterpret_cast<const double*>(vals), rs, cs, F, op, n, heads, off + T, desc, okey,
                       reinterpret_cast<double*>(oagg), ocnt);
  return (int)hipGetLastError();
}

int nsdb_mix64(const void* x, const void* y, void* out, long long n, hipStream_t st) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(out)) & 15)
    return (int)hipErrorInvalidValue;                  // 16-B row pairs
  const long long blocks = std::min<long long>(8192, (n + 511) / 512);
  hipLaunchKernelGGL(mix64_kernel, dim3((unsigned)blocks), dim3(256), 0, st, reinterpret_cast<const u64*>(x),
                     reinterpret_cast<const u64*>(y), reinterpret_cast<u64*>(out), n);
  return (int)hipGetLastError();
}

}  // extern "C"
