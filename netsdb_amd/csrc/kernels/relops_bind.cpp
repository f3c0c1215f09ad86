// PyTorch bindings of the device relational operators (relops.hip): hash aggregation, hash join build /
// probe, and the stable partition permutation of the shuffle sink. Every entry checks device / dtype / shape
// on the host before anything is launched, and launches on the current HIP stream.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <limits>
#include <string>
#include <tuple>
#include <vector>

typedef long long ll;
template <typename T> ll* LL(T* p) { return reinterpret_cast<ll*>(p); }

extern "C" {
long long nsdb_agg_work_bytes(long long n, int F, int pbits, int want_inv);
int nsdb_hash_aggregate(const void* keys, const void* vals, long long n, int F, int vt, int op, int want_inv,
                        int want_first, void* meta, void* glow, long long gcap_low, void* gpart, long long gcap_part,
                        void* out, void* inv, long long ocap, int phase, void* work, int pbits, int lcap_low,
                        int lcap_part, int low_thr, int lcap_mid, long long vrs, long long vcs, hipStream_t st);
int nsdb_join_insert(const void* keys, long long n, void* tab, long long cap, int* row_slot, unsigned* row_rank,
                     unsigned long long* ndup, unsigned* fail, hipStream_t st);
long long nsdb_jpart_work_bytes(long long n, long long cap);
int nsdb_join_build_part(const void* keys, long long n, void* tab, long long cap, void* work,
                         unsigned long long* ctr, unsigned long long* bloom, int bshift, long long* perm, hipStream_t st);
int nsdb_join_perm(const int* row_slot, const unsigned* row_rank, long long n, const unsigned long long* ndup,
                   unsigned long long* bump, void* tab, long long cap, long long* perm, hipStream_t st);
long long nsdb_join_tiles(long long m);
int nsdb_join_probe(const void* keys, long long m, const void* tab, long long cap, unsigned* cnt, unsigned* pay,
                    long long* tile_sum, const unsigned long long* bloom, int bshift, hipStream_t st);
int nsdb_join_bloom(const void* tab, long long cap, long long W, unsigned long long* bloom, hipStream_t st);
int nsdb_join_init(void* tab, long long cap, hipStream_t st);
int nsdb_take_many(const void* const* src, void* const* dst, const long long* nsrc, const int* w, const int* per,
                   int ncols, const long long* idx, long long n, int* bad, hipStream_t st);
int nsdb_join_expand(const unsigned* cnt, const unsigned* pay, long long m, const long long* tile_base,
                     const long long* perm, long long* bidx, long long* pidx, hipStream_t st);
long long nsdb_part_work_bytes(long long n, int P);
int nsdb_mix64(const void* x, const void* y, void* out, long long n, hipStream_t st);
long long nsdb_compact_tiles(long long n);
int nsdb_compact_count(const unsigned char* mask, long long n, unsigned* cnt, long long* off, hipStream_t st);
int nsdb_compact_write(const unsigned char* mask, long long n, const long long* off, long long* out, hipStream_t st);
int nsdb_partition_perm(const long long* dest, long long n, int P, void* work, long long* perm, long long* counts,
                        hipStream_t st);
int nsdb_run_count(const void* keys, long long n, unsigned* cnt, long long* off, hipStream_t st);
int nsdb_run_reduce(const void* keys, const void* vals, long long rs, long long cs, int F, int vt, int op, long long n,
                    const long long* off, long long G, long long* heads, long long* okey, void* oagg, long long* ocnt,
                    hipStream_t st);
}

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

bool g_agg_mid = true;   // the MID group-by path (agg_set_mid: A/B and tests)
bool g_join_bloom = true; // probe filters of large join tables (join_set_bloom: A/B and tests)
bool g_join_part = true;  // partitioned (LDS region) build of multi-region join tables (join_set_part: A/B and tests)
int64_t g_join_bloom_min_bytes = int64_t(4) << 20;   // ... of tables with more slot bytes than this (past the L2)
int64_t g_join_bloom_max_bytes = int64_t(4) << 20;   // ... whose filter has at most this many bytes

void rc_ok(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed with code ", rc, " (", hipGetErrorString((hipError_t)(rc > 0 ? rc : 0)), ")");
}

int64_t pow2_at_least(int64_t x) {
  int64_t c = 1;
  while (c < x) c <<= 1;
  return c;
}
int64_t pow2_at_most(int64_t x) {
  int64_t c = 1;
  while (c * 2 <= x) c <<= 1;
  return c;
}

// Word offsets of the AggMeta fields (relops.hip): est, low, ng_low, ng_part, fail_low, fail_part, ...
constexpr int kMetaWords = 16 + 4096;   // AggMeta + the sampled keys (relops.hip agg_sample_*)

// Group n int64 keys and reduce F value columns per group on the device.
//   vals: [n, F] float64 or int64 (or None / F == 0: counts only); op: "sum" | "min" | "max".
// Returns (reps [g] i64, aggs [g, F] (vals dtype), counts [g] i64, first [g] i64 (smallest row of each group; only
// meaningful with want_first, which otherwise lets the partition passes skip row ids),
// inv [n] i64 (or empty), status): status = [g, path (0 LOW, 1 PART), ok (0: the PART table overflowed; outputs
// invalid, fall back), distinct keys in the 4096-row sample, scratch bytes used]. low_threshold: largest estimated
// group count for the LOW path (0: automatic).
//
// Scratch is sized for the path that runs. Phase 1 (sample + LOW) needs O(groups) words: the LOW global table and an
// output of gcap_low + 1 groups. Only when the device reports that the LOW path did not take the rows (one host read,
// which the LOW path needs anyway for its group count) are the PART buffers allocated — about 2 (12 + 8 F) n bytes of
// partitioned rows plus an n-group output — and `scratch(+bytes)` / `scratch(-bytes)` (a Python callable, e.g. the
// storage manager's device-budget accounting) is told before they are allocated and after they are released.
std::vector<torch::Tensor> hash_aggregate(torch::Tensor keys, c10::optional<torch::Tensor> vals, const std::string& op,
                                          bool want_inv, int64_t low_threshold, bool want_first,
                                          pybind11::object scratch) {
  TORCH_CHECK(keys.is_cuda(), "keys must be a GPU tensor");
  TORCH_CHECK(keys.scalar_type() == torch::kInt64 && keys.dim() == 1, "keys must be 1-D int64");
  keys = keys.contiguous();
  const int64_t n = keys.numel();
  TORCH_CHECK(n < (int64_t(1) << 31), "hash_aggregate: at most 2^31 - 1 rows per call (the caller chunks)");
  int opc = op == "sum" ? 0 : op == "min" ? 1 : op == "max" ? 2 : -1;
  TORCH_CHECK(opc >= 0, "op must be sum, min or max");
  int F = 0, vt = 0;
  int64_t vrs = 0, vcs = 0;
  torch::Tensor v;
  auto vdtype = torch::kFloat64;
  if (vals.has_value() && vals->defined() && vals->numel() > 0) {
    v = *vals;
    TORCH_CHECK(v.is_cuda() && v.device() == keys.device(), "vals must be on the keys' device");
    TORCH_CHECK(v.scalar_type() == torch::kFloat64 || v.scalar_type() == torch::kInt64, "vals must be float64 or int64");
    if (v.dim() == 1) v = v.unsqueeze(1);
    TORCH_CHECK(v.dim() == 2 && v.size(0) == n, "vals must be [n] or [n, F]");
    // row-major [n, F] or column-major (the transpose of a contiguous [F, n] stack) are read in place
    const bool colmajor = v.size(1) > 1 && v.stride(0) == 1 && v.stride(1) >= n;
    if (!colmajor) v = v.contiguous();
    vrs = v.size(1) > 1 ? v.stride(0) : 1;
    vcs = v.size(1) > 1 ? v.stride(1) : 1;
    F = (int)v.size(1);
    TORCH_CHECK(F <= 16, "at most 16 value columns");
    vt = v.scalar_type() == torch::kInt64 ? 1 : 0;
    vdtype = v.scalar_type();
  }
  auto i64 = keys.options().dtype(torch::kInt64);
  if (n == 0) {
    return {torch::empty({0}, i64), torch::empty({0, F}, keys.options().dtype(vdtype)), torch::empty({0}, i64),
            torch::empty({0}, i64), torch::empty({0}, i64), torch::tensor({0, 0, 1, 0, 0}, torch::kInt64)};
  }
  // LDS tables: LOW <= 64 KiB (two workgroups per CU), PART <= 128 KiB. PART: level-1 buckets = one per CU
  // (256) once there are >= 2048 rows per bucket; each bucket workgroup splits its bucket further on the device
  // from the sampled distinct-key estimate (relops.hip agg_bucket_kernel), so no host decision needs the data.
  const int64_t entry = 20 + 8 * F;
  const int64_t lcap_low = std::min<int64_t>(1024, pow2_at_most(65536 / entry));   // <= 36 KB: 4+ LOW workgroups per CU
  const int64_t lcap_part = std::min<int64_t>(4096, pow2_at_most(131072 / entry));
  int pbits = 0;
  while (pbits < 8 && (n >> (pbits + 1)) >= 2048) ++pbits;
  // MID path (relops.hip agg_low_kernel MODE 2): up to 8 hash partitions of the key space, each one CU-sized LDS
  // table of lcap_mid slots (half full at most); 0 disables it. The LOW global table then holds every MID group.
  // (an explicit low_threshold pins the LOW / PART boundary: no MID path then)
  const int64_t lcap_mid =
      g_agg_mid && low_threshold <= 0 ? std::min<int64_t>(4096, pow2_at_most(160 * 1024 / entry)) : 0;
  const int64_t gcap_low = std::max<int64_t>(4 * lcap_low, lcap_mid > 0 ? 2 * 8 * (lcap_mid / 2) : 0);
  // overflow table of the PART path (keys whose LDS probe window filled): a miss-sized estimate only
  const int64_t gcap_part = std::max<int64_t>(4096, std::min<int64_t>(pow2_at_least(2 * n), int64_t(1) << 17));
  const int64_t thr = low_threshold > 0 ? low_threshold : lcap_low / 4;

  auto meta = torch::empty({kMetaWords}, i64);
  auto glow = torch::empty({(gcap_low + 1) * (4 + F)}, i64);
  auto inv = want_inv ? torch::empty({n}, i64) : torch::empty({0}, i64);
  const int64_t ocap_low = std::min<int64_t>(n, gcap_low + 1);
  auto out = torch::empty({ocap_low * (4 + F)}, i64);
  int64_t ocap = ocap_low;
  auto launch = [&](int phase, void* gpart, void* work) {
    rc_ok(nsdb_hash_aggregate(keys.data_ptr(), F ? v.data_ptr() : nullptr, n, F, vt, opc, want_inv ? 1 : 0,
                              want_first ? 1 : 0, meta.data_ptr(), glow.data_ptr(), gcap_low, gpart, gcap_part,
                              out.data_ptr(), want_inv ? inv.data_ptr() : nullptr, ocap, phase, work, pbits,
                              (int)lcap_low, (int)lcap_part, (int)thr, (int)lcap_mid, (long long)vrs, (long long)vcs,
                              stream()),
          "hash_aggregate");
  };
  launch(1, nullptr, nullptr);
  auto m = meta.narrow(0, 0, 16).cpu();   // the host read: group count and path flags
  const ll* mp = LL(m.data_ptr<int64_t>());
  // AggMeta words: 0 est, 1 low, 2 ng_low, 3 ng_part, 4 fail_low, 5 fail_part
  const bool low_ok = mp[1] != 0 && mp[4] == 0;
  int64_t scratch_bytes = (int64_t)(meta.numel() + glow.numel() + inv.numel() + out.numel()) * 8;
  bool ok = true;
  int64_t g = 0;
  if (low_ok) {
    launch(3, nullptr, nullptr);
    g = (int64_t)mp[2];
  } else {
    const int64_t wbytes = nsdb_agg_work_bytes(n, F, pbits, want_inv ? 1 : 0);
    const int64_t part_bytes = ((gcap_part + 1) * (4 + F) + n * (4 + F)) * 8 + wbytes;
    if (!scratch.is_none()) scratch(part_bytes);
    try {
      auto gpart = torch::empty({(gcap_part + 1) * (4 + F)}, i64);
      auto work = torch::empty({(wbytes + 7) / 8}, i64);
      ocap = n;
      out = torch::empty({n * (4 + F)}, i64);
      launch(2, gpart.data_ptr(), work.data_ptr());
      auto m2 = meta.narrow(0, 0, 16).cpu();
      const ll* mp2 = LL(m2.data_ptr<int64_t>());
      g = (int64_t)mp2[3];
      ok = mp2[5] == 0;
      scratch_bytes += part_bytes - (int64_t)ocap_low * (4 + F) * 8;
    } catch (...) {
      if (!scratch.is_none()) scratch(-part_bytes);
      throw;
    }
    if (!scratch.is_none()) scratch(-part_bytes);
  }
  auto status = torch::tensor({(int64_t)g, (int64_t)(low_ok ? 0 : 1), (int64_t)(ok ? 1 : 0), (int64_t)mp[0],
                               scratch_bytes}, torch::kInt64);
  if (!ok) return {torch::Tensor(), torch::Tensor(), torch::Tensor(), torch::Tensor(), torch::Tensor(), status};
  auto reps = out.narrow(0, 0, g);
  auto aggs = out.narrow(0, ocap, g * F).view({g, F});
  if (vt == 0) aggs = aggs.view(torch::kFloat64);
  auto cnt = out.narrow(0, ocap + ocap * F, g);
  auto first = out.narrow(0, ocap * (3 + F), g);
  // the views keep the whole ocap-row buffer alive: copy small results out of a large one
  if (ocap > ocap_low && g * 4 < ocap) {
    reps = reps.clone();
    aggs = aggs.clone();
    cnt = cnt.clone();
    first = first.clone();
  }
  return {reps, aggs, cnt, first, inv, status};
}

// Join build: returns (table [cap+1, 2] i64 of 16-byte slots {key, cnt | pay << 32}, perm [n] i64: the CSR runs of
// repeated keys; untouched when no key repeats, every payload being the build row itself). No host read.
std::vector<torch::Tensor> join_build(torch::Tensor keys) {
  TORCH_CHECK(keys.is_cuda() && keys.scalar_type() == torch::kInt64 && keys.dim() == 1, "keys: 1-D int64 GPU tensor");
  keys = keys.contiguous();
  const int64_t n = keys.numel();
  TORCH_CHECK(n < (int64_t(1) << 29), "join_build: at most 2^29 build rows per table");
  // load factor: <= 1/8 for builds up to 256 k rows (a <= 64 MiB table: a probe of an ABSENT key — most probe rows of
  // a selective join, TPC-H Q17's 60 M lineitems against ~2 k parts — expects ~1.1 slot reads instead of ~2.5 at 1/2),
  // <= 1/4 up to 4 M rows, <= 1/2 beyond
  const int64_t f = n <= (int64_t(1) << 18) ? 8 : (n <= (int64_t(1) << 22) ? 4 : 2);
  int64_t cap = pow2_at_least(std::max<int64_t>(1024, f * n));
  auto i64 = keys.options().dtype(torch::kInt64);
  // Tables of more than 2^22 slots: chains wrap inside regions of kJRegion = 4096 slots (relops.hip), the table is
  // built region by region in LDS (join_build_part) and checked once on the host for a region left without an empty
  // slot (a hash pile-up far outside the load's statistics), in which case it doubles and is rebuilt. Smaller ones:
  // the global insert, whole-table linear probing.
  constexpr int64_t R = 4096, kMaxRegions = 8192, kWhole = int64_t(1) << 22;   // relops.hip kJRegion, kJWholeWrap
  for (int attempt = 0;; ++attempt) {
    auto tab = torch::empty({cap + 1, 2}, i64);
    auto ctr = torch::zeros({3}, i64);   // [repeated-key rows, run bump counter, fail]
    auto* c = reinterpret_cast<unsigned long long*>(ctr.data_ptr<int64_t>());
    auto perm = torch::empty({n}, i64);
    // probe filter for tables past the L2 (> 4 MiB of slots): ~16 filter bits per build row, one word per 2^shift slots
    torch::Tensor bloom = torch::empty({0}, i64);
    int bshift = -1;
    // ... while the filter itself stays L2-sized (<= 4 MiB: builds up to ~2 M rows). A larger one sits in the MALL
    // next to the table, and its word is a second dependent far read for every probe that matches (16 M-row build,
    // 90 % matching probes: 0.89 ms with the filter, 0.70 without, profiles/r6_join)
    if (g_join_bloom && cap * 16 > g_join_bloom_min_bytes &&
        std::min<int64_t>(cap, pow2_at_least(std::max<int64_t>(64, (16 * n + 63) / 64))) * 8 <= g_join_bloom_max_bytes) {
      const int64_t W = std::min<int64_t>(cap, pow2_at_least(std::max<int64_t>(64, (16 * n + 63) / 64)));
      bshift = 0;
      while ((W << bshift) < cap) ++bshift;
      bloom = torch::empty({W}, i64);
    }
    const bool regions = cap > kWhole;                        // chains wrap inside 4096-slot regions
    const bool part = regions && (cap / R) <= kMaxRegions && g_join_part;
    bool bloom_done = false;
    if (part) {
      const bool fold = bshift >= 2 && bshift <= 12;          // filter words written with their region
      auto work = torch::empty({(nsdb_jpart_work_bytes(n, cap) + 7) / 8}, i64);
      rc_ok(nsdb_join_build_part(keys.data_ptr(), n, tab.data_ptr(), cap, work.data_ptr(), c,
                                 fold ? reinterpret_cast<unsigned long long*>(bloom.data_ptr<int64_t>()) : nullptr,
                                 bshift, LL(perm.data_ptr<int64_t>()), stream()),
            "join_build_part");
      bloom_done = fold;
    } else {
      rc_ok(nsdb_join_init(tab.data_ptr(), cap, stream()), "join_init");
      auto row_slot = torch::empty({n}, keys.options().dtype(torch::kInt32));
      auto row_rank = torch::empty({n}, keys.options().dtype(torch::kInt32));
      rc_ok(nsdb_join_insert(keys.data_ptr(), n, tab.data_ptr(), cap, row_slot.data_ptr<int>(),
                             reinterpret_cast<unsigned*>(row_rank.data_ptr<int>()), c,
                             reinterpret_cast<unsigned*>(c + 2), stream()),
            "join_insert");
      // the table keeps each key's EXTRA-row count (join_probe adds the claiming row)
      rc_ok(nsdb_join_perm(row_slot.data_ptr<int>(), reinterpret_cast<const unsigned*>(row_rank.data_ptr<int>()), n, c,
                           c + 1, tab.data_ptr(), cap, LL(perm.data_ptr<int64_t>()), stream()),
            "join_perm");
    }
    if (bshift >= 0 && !bloom_done) {
      bloom.zero_();
      rc_ok(nsdb_join_bloom(tab.data_ptr(), cap, bloom.numel(),
                            reinterpret_cast<unsigned long long*>(bloom.data_ptr<int64_t>()), stream()),
            "join_bloom");
    }
    // Region tables (builds past ~1 M rows) read {fail, largest extra-row count} in one transfer: a region left
    // without an empty slot is rebuilt larger; the count is the table's max multiplicity - 1 (JoinTable
    // .max_multiplicity, which sizes the fused probes' output regions, needs no read of its own). Whole-table tables
    // cannot fill (load <= 1/2): no host read.
    torch::Tensor stat = torch::empty({0}, i64);
    if (regions) {
      stat = torch::stack({ctr[2], tab.select(1, 1).bitwise_and(0xFFFFFFFFLL).max()}).cpu();
      if (stat[0].item<int64_t>() != 0) {                    // a region without an empty slot: rebuild larger
        TORCH_CHECK(attempt < 2 && cap * 2 < (int64_t(1) << 31),
                    "join_build: hash regions overflow even at ", cap, " slots for ", n, " rows");
        cap *= 2;
        continue;
      }
    }
    return {tab, perm, bloom, stat};
  }
}

// bloom: the table's probe filter from join_build (empty: none); shift = log2(slots per filter word)
int bloom_shift(const torch::Tensor& tab, const c10::optional<torch::Tensor>& bloom) {
  if (!bloom.has_value() || !bloom->defined() || bloom->numel() == 0) return -1;
  const int64_t cap = tab.size(0) - 1, W = bloom->numel();
  TORCH_CHECK(W <= cap && (W & (W - 1)) == 0 && bloom->is_contiguous() && bloom->scalar_type() == torch::kInt64 &&
                  bloom->device() == tab.device(), "malformed join probe filter");
  int sh = 0;
  while ((W << sh) < cap) ++sh;
  return sh;
}

// Probe a built table with m int64 keys: all (build row, probe row) pairs with equal keys, probe-major.
std::vector<torch::Tensor> join_probe(torch::Tensor tab, torch::Tensor perm, torch::Tensor keys,
                                      c10::optional<torch::Tensor> bloom) {
  TORCH_CHECK(keys.is_cuda() && keys.scalar_type() == torch::kInt64 && keys.dim() == 1, "keys: 1-D int64 GPU tensor");
  TORCH_CHECK(tab.is_cuda() && tab.scalar_type() == torch::kInt64 && tab.dim() == 2 && tab.size(1) == 2 &&
                  tab.is_contiguous() && perm.scalar_type() == torch::kInt64,
              "join table tensors (from join_build) expected");
  const int64_t cap = tab.size(0) - 1;
  TORCH_CHECK(cap >= 1024 && (cap & (cap - 1)) == 0, "malformed join table");
  TORCH_CHECK(keys.device() == tab.device(), "probe keys must be on the table's device");
  keys = keys.contiguous();
  const int64_t m = keys.numel();
  auto i64 = keys.options().dtype(torch::kInt64);
  if (m == 0) return {torch::empty({0}, i64), torch::empty({0}, i64)};   // (an empty perm: unique build keys)
  auto i32 = keys.options().dtype(torch::kInt32);
  auto cnt = torch::empty({m}, i32);
  auto pay = torch::empty({m}, i32);
  const int64_t tiles = nsdb_join_tiles(m);
  auto tsum = torch::empty({tiles + 1}, i64);
  const int bsh = bloom_shift(tab, bloom);
  rc_ok(nsdb_join_probe(keys.data_ptr(), m, tab.data_ptr(), cap, reinterpret_cast<unsigned*>(cnt.data_ptr<int>()),
                        reinterpret_cast<unsigned*>(pay.data_ptr<int>()), LL(tsum.data_ptr<int64_t>()),
                        bsh >= 0 ? reinterpret_cast<const unsigned long long*>(bloom->data_ptr<int64_t>()) : nullptr,
                        bsh, stream()),
        "join_probe");
  auto incl = torch::cumsum(tsum.narrow(0, 0, tiles), 0);
  const int64_t total = incl[tiles - 1].item<int64_t>();   // sizes the output (one host read)
  auto base = incl.sub_(tsum.narrow(0, 0, tiles));
  auto bidx = torch::empty({total}, i64);
  auto pidx = torch::empty({total}, i64);
  if (total > 0)
    rc_ok(nsdb_join_expand(reinterpret_cast<const unsigned*>(cnt.data_ptr<int>()),
                           reinterpret_cast<const unsigned*>(pay.data_ptr<int>()), m, LL(base.data_ptr<int64_t>()),
                           LL(perm.data_ptr<int64_t>()), LL(bidx.data_ptr<int64_t>()), LL(pidx.data_ptr<int64_t>()),
                           stream()),
          "join_expand");
  return {bidx, pidx};
}

// Stable partition permutation of dest (values in [0, P)): rows of partition 0 first (input order), then 1, ...
std::vector<torch::Tensor> partition_perm(torch::Tensor dest, int64_t P) {
  TORCH_CHECK(dest.is_cuda() && dest.scalar_type() == torch::kInt64 && dest.dim() == 1, "dest: 1-D int64 GPU tensor");
  TORCH_CHECK(P >= 1 && P <= 2048, "partition_perm: 1 <= P <= 2048");
  dest = dest.contiguous();
  const int64_t n = dest.numel();
  TORCH_CHECK(n < (int64_t(1) << 31), "partition_perm: at most 2^31 - 1 rows");
  auto i64 = dest.options().dtype(torch::kInt64);
  auto counts = torch::zeros({P}, i64);
  auto perm = torch::empty({n}, i64);
  if (n == 0) return {perm, counts};
  auto work = torch::empty({(nsdb_part_work_bytes(n, (int)P) + 7) / 8}, i64);
  rc_ok(nsdb_partition_perm(LL(dest.data_ptr<int64_t>()), n, (int)P, work.data_ptr(), LL(perm.data_ptr<int64_t>()),
                            LL(counts.data_ptr<int64_t>()), stream()),
        "partition_perm");
  return {perm, counts};
}

// Row ids of the set rows of a 0/1 byte mask (bool or uint8), in order: torch.nonzero(mask).flatten() as three
// streaming launches + one read of the total (the output size).
torch::Tensor compact(torch::Tensor mask) {
  TORCH_CHECK(mask.is_cuda() && mask.dim() == 1 && (mask.scalar_type() == torch::kBool ||
                                                     mask.scalar_type() == torch::kUInt8),
              "compact: 1-D bool / uint8 GPU mask");
  mask = mask.contiguous();
  const int64_t n = mask.numel();
  auto i64 = mask.options().dtype(torch::kInt64);
  if (n == 0) return torch::empty({0}, i64);
  const unsigned char* mp = reinterpret_cast<const unsigned char*>(mask.data_ptr());
  if (reinterpret_cast<uintptr_t>(mp) & 15) {
    mask = mask.clone();
    mp = reinterpret_cast<const unsigned char*>(mask.data_ptr());
  }
  const int64_t T = nsdb_compact_tiles(n);
  auto cnt = torch::empty({T}, mask.options().dtype(torch::kInt32));
  auto off = torch::empty({T + 1}, i64);
  rc_ok(nsdb_compact_count(mp, n, reinterpret_cast<unsigned*>(cnt.data_ptr<int32_t>()), LL(off.data_ptr<int64_t>()),
                           stream()),
        "compact_count");
  const int64_t total = off[T].item<int64_t>();
  auto out = torch::empty({total}, i64);
  if (total > 0)
    rc_ok(nsdb_compact_write(mp, n, LL(off.data_ptr<int64_t>()), LL(out.data_ptr<int64_t>()), stream()),
          "compact_write");
  return out;
}

// mix64((x ^ y) + GOLD) per row (y optional), int64 in / out: the engine's key hash in one pass.
torch::Tensor mix64(torch::Tensor x, c10::optional<torch::Tensor> y) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == torch::kInt64 && x.dim() == 1, "mix64: x must be a 1-D int64 GPU tensor");
  x = x.contiguous();
  const void* yp = nullptr;
  torch::Tensor yc;
  if (y.has_value() && y->defined()) {
    TORCH_CHECK(y->is_cuda() && y->scalar_type() == torch::kInt64 && y->numel() == x.numel() && y->device() == x.device(),
                "mix64: y must be an int64 GPU tensor like x");
    yc = y->contiguous();
    yp = yc.data_ptr();
  }
  auto out = torch::empty_like(x);
  const bool aligned = ((reinterpret_cast<uintptr_t>(x.data_ptr()) | reinterpret_cast<uintptr_t>(yp) |
                         reinterpret_cast<uintptr_t>(out.data_ptr())) & 15) == 0;
  if (!aligned) {                                   // a view at an odd offset: realign first
    x = x.clone();
    if (yp) {
      yc = yc.clone();
      yp = yc.data_ptr();
    }
  }
  rc_ok(nsdb_mix64(x.data_ptr(), yp, out.data_ptr(), x.numel(), stream()), "mix64");
  return out;
}

// Group-by of keys that arrive in runs (relops.hip run_*_kernel): (reps [g], aggs [g, F], counts [g], first [g]) with
// the groups in row order, or an empty list when the keys are not ordered (some key below its predecessor: equal
// keys may then be apart) and the caller must take hash_aggregate. vals as in hash_aggregate; one host read (the
// group count and the order flag together).
std::vector<torch::Tensor> run_aggregate(torch::Tensor keys, c10::optional<torch::Tensor> vals, const std::string& op) {
  TORCH_CHECK(keys.is_cuda() && keys.scalar_type() == torch::kInt64 && keys.dim() == 1, "keys must be 1-D int64 GPU");
  keys = keys.contiguous();
  const int64_t n = keys.numel();
  const int opc = op == "sum" ? 0 : op == "min" ? 1 : op == "max" ? 2 : -1;
  TORCH_CHECK(opc >= 0, "op must be sum, min or max");
  int F = 0, vt = 0;
  int64_t vrs = 0, vcs = 0;
  torch::Tensor v;
  auto vdtype = torch::kFloat64;
  if (vals.has_value() && vals->defined() && vals->numel() > 0) {
    v = *vals;
    TORCH_CHECK(v.is_cuda() && v.device() == keys.device(), "vals must be on the keys' device");
    TORCH_CHECK(v.scalar_type() == torch::kFloat64 || v.scalar_type() == torch::kInt64, "vals must be float64 or int64");
    if (v.dim() == 1) v = v.unsqueeze(1);
    TORCH_CHECK(v.dim() == 2 && v.size(0) == n, "vals must be [n] or [n, F]");
    vrs = v.stride(0);
    vcs = v.stride(1);
    F = (int)v.size(1);
    vt = v.scalar_type() == torch::kInt64 ? 1 : 0;
    vdtype = v.scalar_type();
  }
  auto i64 = keys.options().dtype(torch::kInt64);
  if (n == 0) return {};
  const int64_t T = nsdb_compact_tiles(n);
  auto cnt = torch::empty({T}, keys.options().dtype(torch::kInt32));
  auto off = torch::empty({T + 2}, i64);
  rc_ok(nsdb_run_count(keys.data_ptr(), n, reinterpret_cast<unsigned*>(cnt.data_ptr<int32_t>()),
                       LL(off.data_ptr<int64_t>()), stream()), "run_count");
  const auto st = off.slice(0, T, T + 2).cpu();          // [groups, descending step seen]
  const int64_t G = st[0].item<int64_t>();
  if (st[1].item<int64_t>() != 0) return {};
  auto heads = torch::empty({G}, i64), okey = torch::empty({G}, i64), ocnt = torch::empty({G}, i64);
  auto oagg = torch::empty({G, F}, keys.options().dtype(vdtype));
  rc_ok(nsdb_run_reduce(keys.data_ptr(), F ? v.data_ptr() : nullptr, vrs, vcs, F, vt, opc, n, LL(off.data_ptr<int64_t>()),
                        G, LL(heads.data_ptr<int64_t>()), LL(okey.data_ptr<int64_t>()), F ? oagg.data_ptr() : nullptr,
                        LL(ocnt.data_ptr<int64_t>()), stream()), "run_reduce");
  return {okey, oagg, ocnt, heads};
}


// Rows idx of several device columns in one launch (relops.hip take_many_kernel). Every column: a contiguous tensor
// on idx's device whose rows (dim 0) are 1, 2, 4, 8 or a multiple of 16 bytes wide (narrower multi-byte rows are
// copied element by element). Returns the gathered columns and a device flag word (1: an id was out of range).
// bad: an int32 device word the kernel sets on an out-of-range id (kept by the caller across calls and checked with
// its other reads: no per-call fill launch)
std::vector<torch::Tensor> take_many(std::vector<torch::Tensor> cols, torch::Tensor idx, torch::Tensor bad) {
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == torch::kInt64 && idx.dim() == 1, "take_many: idx 1-D int64 GPU");
  TORCH_CHECK(bad.is_cuda() && bad.device() == idx.device() && bad.scalar_type() == torch::kInt32 && bad.numel() >= 1,
              "take_many: bad must be an int32 word on idx's device");
  idx = idx.contiguous();
  const int64_t n = idx.numel();
  std::vector<torch::Tensor> out;
  out.reserve(cols.size());
  std::vector<const void*> src;
  std::vector<void*> dst;
  std::vector<long long> nsrc;
  std::vector<int> w, per;
  auto flush = [&]() {
    if (!src.empty())
      rc_ok(nsdb_take_many(src.data(), dst.data(), nsrc.data(), w.data(), per.data(), (int)src.size(),
                           LL(idx.data_ptr<int64_t>()), n, bad.data_ptr<int>(), stream()), "take_many");
    src.clear(); dst.clear(); nsrc.clear(); w.clear(); per.clear();
  };
  for (auto& c : cols) {
    TORCH_CHECK(c.is_cuda() && c.device() == idx.device() && c.dim() >= 1 && c.is_contiguous(),
                "take_many: contiguous columns on idx's device expected");
    auto sizes = c.sizes().vec();
    sizes[0] = n;
    auto o = torch::empty(sizes, c.options());
    out.push_back(o);
    TORCH_CHECK(n == 0 || c.size(0) > 0, "take_many: row ids into an empty column");
    const int64_t rowb = c.numel() == 0 ? 0 : (int64_t)c.nbytes() / c.size(0);
    if (n == 0 || rowb == 0) continue;
    int ww, pp;
    if (rowb == 1 || rowb == 2 || rowb == 4 || rowb == 8) { ww = (int)rowb; pp = 1; }
    else if (rowb % 16 == 0) { ww = 16; pp = (int)(rowb / 16); }
    else { ww = (int)c.element_size(); pp = (int)(rowb / ww); }
    if (reinterpret_cast<uintptr_t>(c.data_ptr()) % ww != 0) {   // a view at an offset: element-wide copies
      ww = (int)c.element_size();
      pp = (int)(rowb / ww);
    }
    src.push_back(c.data_ptr()); dst.push_back(o.data_ptr()); nsrc.push_back(c.size(0)); w.push_back(ww); per.push_back(pp);
    if ((int)src.size() == 48) flush();
  }
  flush();
  return out;
}
}  // namespace

std::vector<torch::Tensor> hash_aggregate_impl(torch::Tensor keys, c10::optional<torch::Tensor> vals,
                                               const std::string& op, bool want_inv, int64_t low_threshold) {
  return hash_aggregate(keys, vals, op, want_inv, low_threshold, true, pybind11::none());
}

void register_relops(pybind11::module& m) {
  m.def("hash_aggregate", &hash_aggregate,
        "device hash group-by + aggregate: (reps, aggs, counts, first, inv, status[g, path, ok, sample_distinct, scratch_bytes])",
        pybind11::arg("keys"), pybind11::arg("vals") = pybind11::none(), pybind11::arg("op") = "sum",
        pybind11::arg("want_inv") = false, pybind11::arg("low_threshold") = 0, pybind11::arg("want_first") = true,
        pybind11::arg("scratch") = pybind11::none());
  m.def("take_many", &take_many, "rows idx of several device columns in one launch (bad: int32 device word set on "
        "an out-of-range id)", pybind11::arg("cols"), pybind11::arg("idx"), pybind11::arg("bad"));
  m.def("join_build", &join_build, "device hash-join build: (table, perm, probe filter (empty: none), host [fail, "
        "largest extra-row count] (empty: not read))");
  m.def("join_probe", &join_probe, "device hash-join probe: (build_idx, probe_idx)", pybind11::arg("tab"),
        pybind11::arg("perm"), pybind11::arg("keys"), pybind11::arg("bloom") = pybind11::none());
  m.def("join_set_bloom", [](bool on, int64_t min_table_bytes, int64_t max_filter_bytes) {
          g_join_bloom = on;
          g_join_bloom_min_bytes = min_table_bytes;
          g_join_bloom_max_bytes = max_filter_bytes;
        }, "build probe filters for join tables of more than min_table_bytes of slots whose filter has at most "
        "max_filter_bytes (default on, 4 MiB, 4 MiB)",
        pybind11::arg("on"), pybind11::arg("min_table_bytes") = int64_t(4) << 20,
        pybind11::arg("max_filter_bytes") = int64_t(4) << 20);
  m.def("join_set_part", [](bool on) { g_join_part = on; }, "partitioned LDS-region build of join tables of more than "
        "one 4096-slot region (default on; off: the global-atomic insert)", pybind11::arg("on"));
  m.def("partition_perm", &partition_perm, "stable device partition permutation: (perm, counts)");
  m.def("agg_set_mid", [](bool on) { g_agg_mid = on; }, "enable / disable the MID group-by path (hash-partitioned LDS "
        "tables sharing their rows through L2); returns nothing", pybind11::arg("on"));
  m.def("compact", &compact, "row ids of the set rows of a 0/1 byte mask, in order (stable stream compaction)",
        pybind11::arg("mask"));
  m.def("run_aggregate", &run_aggregate, "group-by of keys arriving in runs: (reps, aggs, counts, first) or [] when "
        "the keys are not ordered", pybind11::arg("keys"), pybind11::arg("vals") = pybind11::none(),
        pybind11::arg("op") = "sum");
  m.def("mix64", &mix64, "key hash mix64((x ^ y) + GOLD) per row, one pass", pybind11::arg("x"),
        pybind11::arg("y") = pybind11::none());
}
