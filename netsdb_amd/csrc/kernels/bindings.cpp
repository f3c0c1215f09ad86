// PyTorch bindings for the netsdb_amd CDNA4 kernels (module netsdb_amd._hip_kernels).
// Every op checks device/dtype/shape on the host BEFORE launching (a bad shape must never reach
// the GPU) and launches on the current HIP stream so ops compose with hipGraph capture.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <limits>
#include <map>
#include <vector>
#include <mutex>
#include <utility>

extern "C" {
int nsdb_gemm_splits(int M, int N, int K, int batch, int cfg);
int nsdb_gemm_prefetch_eligible(int M, int N, int K, int batch, int splits, int cfg);
int nsdb_gemm_launch_wgs(int M, int N, int K, int batch, int splits, int cfg);
int nsdb_gemm_nt_bf16(const void* A, const void* B, void* C, float* ws, const float* bias, int M, int N, int K,
                      long long lda, long long ldb, long long ldc, long long sA, long long sB, long long sC,
                      long long sBias, int batch, int splits, int act, int bias_mode, int out_f32, float alpha,
                      float dropout, unsigned long long seed, int accumulate, long long seg_k, long long seg_stride_b,
                      const void* opts, hipStream_t stream);
int nsdb_gemm_nt_softmax(const void* A, const void* B, float* C, const float* bias, int M, int N, int K, long long lda,
                         long long ldb, long long ldc, int bias_mode, float alpha, int axis, void* part, int* cnt,
                         int* flag, int* dep, int force_fallback, int epi, unsigned long long* stamps,
                         hipStream_t stream);
int nsdb_gemm_nt_f32(const float* A, const float* B, float* C, int M, int N, int K, long long lda, long long ldb,
                     long long ldc, float alpha, int accumulate, hipStream_t stream);
struct ConvOpts {
  int force_generic, variant, max_blocks, kernel, contig;
};
int nsdb_conv2d_igemm(const void* X, const void* Wt, const float* bias, void* out, int N, int C, int H, int W,
                      int OC, int KH, int KW, int stride, int pad, int dil, int ldw, int act, int nchw_out,
                      int out_f32, const void* wfrag, const struct ConvOpts* opts, hipStream_t stream);
int nsdb_prefetch(const void* ptr, long long bytes, unsigned* sink, int blocks, hipStream_t stream);
int nsdb_im2col(const void* X, void* out, int N, int C, int H, int W, int KH, int KW, int stride, int pad, int dil,
                int ldk, hipStream_t stream);
int nsdb_softmax_rows(const void* X, int x_f32, const float* bias, void* Y, int y_f32, int R, int N,
                      long long ldx, long long ldy, int log_out, int plain_loads, hipStream_t st);
int nsdb_bias_act(const void* X, int x_f32, const float* bias, void* Y, int y_f32, int R, int N, int bias_mode,
                  int act, float dropout, unsigned long long seed, hipStream_t st);
int nsdb_lstm_ew(int mode, const float* a, const float* b, const float* c, const float* d, float* out, long long n,
                 hipStream_t st);
int nsdb_lstm_cell(const void* gates, int g_f32, const float* c_prev, void* h_out, int h_f32, float* c_out, int B,
                   int H, hipStream_t st);
int nsdb_embedding_bag(const void* table, int t_f32, const long long* idx, const long long* offsets,
                       const float* weights, float* out, int Bn, int D, int mode, hipStream_t st);
int nsdb_dedup_splits(long long nblocks, long long bytes_per_block);
int nsdb_block_hash(const void* data, long long nblocks, long long words, int S, unsigned long long* partial,
                    hipStream_t st);
int nsdb_block_simcount(const void* pool, const long long* cand, const void* query, long long nblocks, long long elems,
                        int bc, int h, int w, float fp, int is_f32, int S, unsigned* partial, hipStream_t st);
int nsdb_block_maxdiff(const void* pool, const long long* cand, const void* blks, long long nblocks, long long elems,
                       int is_f32, int S, float* partial, hipStream_t st);
int nsdb_str_pack(const void* bytes, const int64_t* starts, const int64_t* ends, int64_t n, int L, int64_t* out,
                  hipStream_t st);
int nsdb_str_hash(const void* bytes, const int64_t* starts, const int64_t* ends, int64_t n, uint64_t* out,
                  hipStream_t st);
int nsdb_str_like(const void* bytes, const int64_t* starts, const int64_t* ends, int64_t n, const uint8_t* pat,
                  int pat_len, const int* seg_start, const int* seg_len, int nseg, int anchor_start, int anchor_end,
                  int negate, uint8_t* out, hipStream_t st);
int nsdb_str_slice(const void* src, const int64_t* starts, int64_t start, const int64_t* out_off, int64_t n,
                   void* dst, hipStream_t st);
int nsdb_str_like_occ(const void* bytes, int64_t nbytes, int64_t payload_end, const int64_t* starts, const int64_t* ends,
                      int64_t n, const uint8_t* pat, int pat_len, const int* seg_start, const int* seg_len, int nseg,
                      int negate, uint64_t* occ, uint8_t* out, hipStream_t st);
int nsdb_str_eq_pairs(const void* a, const int64_t* sta, const int64_t* ena, const int64_t* ia, const void* b,
                      const int64_t* stb, const int64_t* enb, const int64_t* ib, int64_t m, uint8_t* out,
                      hipStream_t st);
int nsdb_str_gather(const void* src, const int64_t* starts, const int64_t* ends, const int64_t* idx,
                    const int64_t* out_off, int64_t m, void* dst, hipStream_t st);
}

void register_relops(pybind11::module& m);
void register_pipeline(pybind11::module& m);
std::vector<torch::Tensor> hash_aggregate_impl(torch::Tensor keys, c10::optional<torch::Tensor> vals,
                                               const std::string& op, bool want_inv, int64_t low_threshold);

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

int64_t g_like_occ_min_rows = 1 << 16;   // str_like: rows from which the occurrence-bitmap form is used (0: off)

// Per-call launch options of the block GEMM (gemm.hip GemmOpts): a forced config or an operand prefetch belongs
// to the one call that passes it.
struct GemmOpts {
  int cfg;
  int epi;
  const void* pf_ptr;
  long long pf_bytes;
  int kinter;
  int mfma;
  int fixup;
  int* fx_state;
};

torch::Tensor softmax_state(const torch::Tensor& like, int64_t need, hipStream_t st);

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed with code ", rc, " (", hipGetErrorString((hipError_t)(rc > 0 ? rc : 0)), ")");
}

void check_cuda(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}

bool is_f32(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == torch::kFloat32 || t.scalar_type() == torch::kBFloat16, name,
              " must be float32 or bfloat16");
  return t.scalar_type() == torch::kFloat32;
}

// C = epi(alpha * A @ B^T); A [b?,M,K] bf16, B [b?,N,K] bf16 (row stride may exceed K), bias f32.
// cfg: -1 auto, 0 (128x128 tile kernel), 2 (256x256 8-phase), 3 / 4 (256x128 / 128x256 skinny stream). prefetch: a later kernel's operand that this
// launch's workgroups read into the Infinity Cache as they finish (the caller checked gemm_prefetch_eligible).
torch::Tensor gemm_nt(torch::Tensor A, torch::Tensor B, c10::optional<torch::Tensor> bias, int64_t bias_mode,
                      int64_t act, bool out_f32, double alpha, double dropout, int64_t seed, int64_t splits,
                      c10::optional<torch::Tensor> out, bool accumulate, int64_t cfg, int64_t epi,
                      c10::optional<torch::Tensor> prefetch, int64_t mfma, int64_t fixup) {
  check_cuda(A, "A");
  check_cuda(B, "B");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && B.scalar_type() == torch::kBFloat16, "A,B must be bf16");
  TORCH_CHECK(A.dim() == B.dim() && (A.dim() == 2 || A.dim() == 3), "A,B must both be 2-D or 3-D");
  TORCH_CHECK(A.stride(-1) == 1 && B.stride(-1) == 1, "A,B must be K-contiguous");
  const bool batched = A.dim() == 3;
  const int64_t batch = batched ? A.size(0) : 1;
  TORCH_CHECK(!batched || B.size(0) == batch, "batch mismatch");
  const int64_t M = A.size(-2), K = A.size(-1), N = B.size(-2);
  TORCH_CHECK(B.size(-1) == K, "K mismatch: A[...,", K, "] vs B[...,", B.size(-1), "]");
  TORCH_CHECK(K % 8 == 0, "K must be a multiple of 8 (pad the block storage)");
  TORCH_CHECK(A.stride(-2) % 8 == 0 && B.stride(-2) % 8 == 0, "row strides must be multiples of 8");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "dims too large");
  const float* bptr = nullptr;
  int64_t sBias = 0;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->is_contiguous(), "bias must be contiguous f32");
    TORCH_CHECK(bias_mode >= 1 && bias_mode <= 3, "bias_mode must be 1 (per row), 2 (per col) or 3 (matrix)");
    if (bias_mode == 3) {   // full [.., M, N] f32 matrix added in the epilogue (LSTM gate biases)
      TORCH_CHECK(bias->size(-1) == N && bias->size(-2) == M, "bias matrix must be [M, N]");
      TORCH_CHECK(bias->dim() == 2 || bias->size(0) == batch, "bias batch mismatch");
      sBias = (bias->dim() == 3) ? M * N : 0;
    } else {
      const int64_t blen = bias->size(-1);
      TORCH_CHECK(blen == (bias_mode == 1 ? M : N), "bias length mismatch");
      sBias = (bias->dim() == 2) ? blen : 0;
      TORCH_CHECK(bias->dim() == 1 || bias->size(0) == batch, "bias batch mismatch");
    }
    bptr = bias->data_ptr<float>();
  }
  auto opts = A.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16);
  torch::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.scalar_type() == opts.dtype(), "out dtype mismatch");
    TORCH_CHECK(C.size(-2) == M && C.size(-1) == N && C.stride(-1) == 1, "out shape mismatch");
  } else {
    TORCH_CHECK(!accumulate, "accumulate=True needs an existing f32 out tensor");
    C = batched ? torch::empty({batch, M, N}, opts) : torch::empty({M, N}, opts);
  }
  TORCH_CHECK(!accumulate || out_f32, "accumulate=True needs out_f32");
  TORCH_CHECK(cfg == -1 || cfg == 0 || (cfg >= 2 && cfg <= 6),
              "gemm_nt: cfg must be -1 (auto), 0, 2, 3, 4, 5 or 6 (study configs: _hip_study)");
  // 5 / 6: the stream tiles 3 / 4 with k-interleaved splits (split s takes k-tiles s, s + S, ...; an A/B arm)
  const int kinter = cfg >= 5 ? 1 : 0;
  if (cfg >= 5) cfg -= 2;
  int s = splits > 0 ? (int)splits : nsdb_gemm_splits((int)M, (int)N, (int)K, (int)batch, (int)cfg);
  torch::Tensor ws;
  float* wsp = nullptr;
  if (s > 1) {
    ws = torch::empty({batch * s * M * N}, A.options().dtype(torch::kFloat32));
    wsp = ws.data_ptr<float>();
  }
  TORCH_CHECK(epi >= -1 && epi <= 1, "gemm_nt: epi must be -1 (auto), 0 (LDS-staged) or 1 (direct)");
  TORCH_CHECK(mfma == 0 || mfma == 16 || mfma == 32, "gemm_nt: mfma must be 0 (auto), 16 or 32");
  GemmOpts o{(int)cfg, (int)epi, nullptr, 0, kinter, (int)mfma, 0, nullptr};
  if (fixup && s > 1) {
    // the in-launch split-K reduction's arrival / departure words: zero between launches on this stream (shared
    // with the fused softmax's, which also leaves them zero)
    const int64_t tiles = ((M + 255) / 256) * ((N + 255) / 256);
    o.fixup = 1;
    o.fx_state = softmax_state(A, 2 * tiles, cur_stream()).data_ptr<int>();
  }
  if (prefetch.has_value() && prefetch->defined() && prefetch->numel() > 0) {
    // the byte span of the tensor's elements (a strided view reads its whole span)
    check_cuda(*prefetch, "prefetch");
    int64_t last = 0;
    for (int64_t d = 0; d < prefetch->dim(); ++d) last += (prefetch->size(d) - 1) * prefetch->stride(d);
    o.pf_ptr = prefetch->data_ptr();
    o.pf_bytes = (last + 1) * (long long)prefetch->element_size();
  }
  const int rc = nsdb_gemm_nt_bf16(
      A.data_ptr(), B.data_ptr(), C.data_ptr(), wsp, bptr, (int)M, (int)N, (int)K, A.stride(-2), B.stride(-2),
      C.stride(-2), batched ? A.stride(0) : 0, batched ? B.stride(0) : 0, batched ? C.stride(0) : 0, sBias,
      (int)batch, s, (int)act, (int)bias_mode, out_f32 ? 1 : 0, (float)alpha, (float)dropout,
      (unsigned long long)seed, accumulate ? 1 : 0, 0, 0, &o, cur_stream());
  check_rc(rc, "gemm_nt");
  return C;
}

// Arrival counters + fallback flags of the fused softmax: zero between launches (the fix-up kernel re-zeroes
// what a launch used), so one persistent buffer per (device, stream) — launches on one stream are ordered.
std::mutex g_sm_mu;
std::map<std::pair<int, hipStream_t>, torch::Tensor> g_sm_state;

torch::Tensor softmax_state(const torch::Tensor& like, int64_t need, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_sm_mu);
  auto key = std::make_pair((int)like.get_device(), st);
  auto it = g_sm_state.find(key);
  if (it == g_sm_state.end() || it->second.numel() < need) {
    auto t = torch::zeros({std::max<int64_t>(need, 4096)}, like.options().dtype(torch::kInt32));
    g_sm_state[key] = t;
    return t;
  }
  return it->second;
}

// C (f32 [M, N]) = softmax(alpha * A . B^T + bias) along axis 1 (every row of C) or 2 (every column), fused
// into the GEMM epilogue (max-subtracted; cross-workgroup partials, see gemm.hip softmax_epilogue_8ph).
torch::Tensor gemm_nt_softmax(torch::Tensor A, torch::Tensor B, c10::optional<torch::Tensor> bias, int64_t bias_mode,
                              int64_t axis, c10::optional<torch::Tensor> out, double alpha, bool force_fallback,
                              int64_t epi, c10::optional<torch::Tensor> stamps) {
  check_cuda(A, "A");
  check_cuda(B, "B");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && B.scalar_type() == torch::kBFloat16, "A,B must be bf16");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2, "A,B must be 2-D");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1, "A,B must be K-contiguous");
  TORCH_CHECK(axis == 1 || axis == 2, "axis must be 1 (rows) or 2 (columns)");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && K % 8 == 0, "K mismatch or K % 8 != 0");
  TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0, "row strides must be multiples of 8");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31), "dims too large");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->is_contiguous() && bias->dim() == 1, "bias f32 1-D");
    TORCH_CHECK(bias_mode == 1 || bias_mode == 2, "fused softmax takes a per-row (1) or per-column (2) bias");
    TORCH_CHECK(bias->numel() == (bias_mode == 1 ? M : N), "bias length mismatch");
    bptr = bias->data_ptr<float>();
  }
  torch::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.scalar_type() == torch::kFloat32 && C.dim() == 2 && C.size(0) == M && C.size(1) == N &&
                C.stride(1) == 1, "out must be f32 [M, N] with unit column stride");
  } else {
    C = torch::empty({M, N}, A.options().dtype(torch::kFloat32));
  }
  const int64_t tm = (M + 255) / 256, tn = (N + 255) / 256;
  // per-group partials [group][256 lines][need rounded up to even] float2 (gemm.hip sm_need_pad)
  const int64_t groups = axis == 1 ? tm : tn, need = axis == 1 ? tn : tm;
  auto part = torch::empty({groups * 256 * ((need + 1) & ~1LL) * 2}, A.options().dtype(torch::kFloat32));
  const hipStream_t st = cur_stream();
  // arrival [max(tm, tn)] | departure [max(tm, tn)] | timed-out flags [tm * tn]: zero on entry, zero on exit
  const int64_t maxg = std::max(tm, tn);
  auto state = softmax_state(A, 2 * maxg + tm * tn, st);
  int* cnt = state.data_ptr<int>();
  unsigned long long* sp = nullptr;
  if (stamps.has_value() && stamps->defined()) {     // diagnostic phase stamps: int64 [tiles * 8]
    check_cuda(*stamps, "stamps");
    TORCH_CHECK(stamps->scalar_type() == torch::kInt64 && stamps->is_contiguous() && stamps->numel() >= tm * tn * 8,
                "stamps must be int64 with >= tiles * 8 entries");
    sp = reinterpret_cast<unsigned long long*>(stamps->data_ptr<int64_t>());
  }
  const int rc = nsdb_gemm_nt_softmax(A.data_ptr(), B.data_ptr(), C.data_ptr<float>(), bptr, (int)M, (int)N, (int)K,
                                      A.stride(0), B.stride(0), C.stride(0), (int)bias_mode, (float)alpha, (int)axis,
                                      part.data_ptr(), cnt, cnt + 2 * maxg, cnt + maxg, force_fallback ? 1 : 0, (int)epi, sp, st);
  check_rc(rc, "gemm_nt_softmax");
  return C;
}

// C = epilogue(A . Bcat^T) where Bcat [N, S*seg_k] is an all-gathered chunk held as [S][N][seg_k] (rank s's
// K slab of every row): the kernel reads each K segment in place (split-K, one or more splits per
// segment), so the gathered buffer needs no permute/reshape copy into a K-contiguous panel.
torch::Tensor gemm_nt_bseg(torch::Tensor A, torch::Tensor Bg, c10::optional<torch::Tensor> bias, int64_t bias_mode,
                           int64_t act, bool out_f32, double alpha, double dropout, int64_t seed,
                           c10::optional<torch::Tensor> out) {
  check_cuda(A, "A");
  check_cuda(Bg, "B");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && Bg.scalar_type() == torch::kBFloat16, "A,B must be bf16");
  TORCH_CHECK(A.dim() == 2 && A.stride(1) == 1 && A.stride(0) % 8 == 0, "A [M, K] K-contiguous");
  TORCH_CHECK(Bg.dim() == 3 && Bg.is_contiguous(), "B must be a contiguous [S, N, seg_k] gathered chunk");
  const int64_t S = Bg.size(0), N = Bg.size(1), segk = Bg.size(2), M = A.size(0), K = S * segk;
  TORCH_CHECK(segk % 64 == 0, "seg_k must be a multiple of 64");
  TORCH_CHECK(A.size(1) == K, "A K must equal S*seg_k");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->is_contiguous() && bias->dim() == 1, "bias f32 1-D");
    TORCH_CHECK(bias->numel() == (bias_mode == 1 ? M : N), "bias length mismatch");
    bptr = bias->data_ptr<float>();
  }
  auto opts = A.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16);
  torch::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.scalar_type() == opts.dtype() && C.size(0) == M && C.size(1) == N && C.stride(1) == 1, "out");
  } else {
    C = torch::empty({M, N}, opts);
  }
  // splits: S segments x d splits per segment (d | seg_k/64), close to the launcher's own choice
  const int auto_s = std::max<int>(1, nsdb_gemm_splits((int)M, (int)N, (int)K, 1, -1));
  const int steps = (int)(segk / 64);
  int d = 1;
  for (int c = 1; c <= steps; ++c)
    if (steps % c == 0 && S * c <= std::max<int64_t>(auto_s, S)) d = c;
  const int s = (int)(S * d);
  torch::Tensor ws;
  float* wsp = nullptr;
  if (s > 1) {
    ws = torch::empty({(int64_t)s * M * N}, A.options().dtype(torch::kFloat32));
    wsp = ws.data_ptr<float>();
  }
  const int rc = nsdb_gemm_nt_bf16(A.data_ptr(), Bg.data_ptr(), C.data_ptr(), wsp, bptr, (int)M, (int)N, (int)K,
                                   A.stride(0), segk, C.stride(0), 0, 0, 0, 0, 1, s, (int)act,
                                   bptr ? (int)bias_mode : 0, out_f32 ? 1 : 0, (float)alpha, (float)dropout,
                                   (unsigned long long)seed, 0, segk, N * segk, nullptr, cur_stream());
  check_rc(rc, "gemm_nt_bseg");
  return C;
}

// C (f32 [M, N]) = alpha * A . B^T (+ C): exact-f32 MFMA (v_mfma_f32_16x16x4_f32) for the analytics libraries.
torch::Tensor gemm_nt_f32(torch::Tensor A, torch::Tensor B, double alpha, c10::optional<torch::Tensor> out,
                          bool accumulate) {
  check_cuda(A, "A");
  check_cuda(B, "B");
  TORCH_CHECK(A.scalar_type() == torch::kFloat32 && B.scalar_type() == torch::kFloat32, "A,B must be f32");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1, "A,B [rows, K] K-contiguous");
  const int64_t M = A.size(0), K = A.size(1), N = B.size(0);
  TORCH_CHECK(B.size(1) == K && K % 4 == 0, "K mismatch or K % 4 != 0");
  TORCH_CHECK(A.stride(0) % 4 == 0 && B.stride(0) % 4 == 0, "row strides must be multiples of 4");
  TORCH_CHECK(M < (1LL << 31) && N < (1LL << 31) && K < (1LL << 31), "dims too large");
  torch::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    TORCH_CHECK(C.scalar_type() == torch::kFloat32 && C.dim() == 2 && C.size(0) == M && C.size(1) == N &&
                C.stride(1) == 1, "out must be f32 [M, N] with unit column stride");
  } else {
    TORCH_CHECK(!accumulate, "accumulate=True needs an existing out tensor");
    C = torch::empty({M, N}, A.options());
  }
  check_rc(nsdb_gemm_nt_f32(A.data_ptr<float>(), B.data_ptr<float>(), C.data_ptr<float>(), (int)M, (int)N, (int)K,
                            A.stride(0), B.stride(0), C.stride(0), (float)alpha, accumulate ? 1 : 0, cur_stream()),
           "gemm_nt_f32");
  return C;
}

int64_t gemm_splits(int64_t M, int64_t N, int64_t K, int64_t batch, int64_t cfg) {
  return nsdb_gemm_splits((int)M, (int)N, (int)K, (int)batch, (int)cfg);
}

torch::Tensor conv2d(torch::Tensor X, torch::Tensor Wt, c10::optional<torch::Tensor> bias, int64_t KH, int64_t KW,
                     int64_t stride, int64_t pad, int64_t dil, int64_t act, bool nchw_out, bool out_f32,
                     c10::optional<torch::Tensor> wfrag, int64_t kernel, int64_t max_blocks, bool force_generic,
                     int64_t variant, int64_t contig) {
  check_cuda(X, "X");
  check_cuda(Wt, "W");
  TORCH_CHECK(X.scalar_type() == torch::kBFloat16 && Wt.scalar_type() == torch::kBFloat16, "X,W must be bf16");
  TORCH_CHECK(X.dim() == 4 && X.is_contiguous(), "X must be contiguous NCHW");
  TORCH_CHECK(Wt.dim() == 2 && Wt.is_contiguous(), "W must be [OC, ldw] contiguous (im2col column order)");
  const int64_t N = X.size(0), C = X.size(1), H = X.size(2), W = X.size(3), OC = Wt.size(0), ldw = Wt.size(1);
  TORCH_CHECK(ldw >= C * KH * KW && ldw % 8 == 0, "W row length must be >= C*KH*KW and a multiple of 8");
  TORCH_CHECK(stride >= 1 && dil >= 1 && pad >= 0, "bad conv geometry");
  const int64_t OH = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  const int64_t OW = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  TORCH_CHECK(OH > 0 && OW > 0, "empty output");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == OC && bias->is_contiguous(), "bias f32[OC]");
    check_cuda(*bias, "bias");
    bptr = bias->data_ptr<float>();
  }
  const void* fptr = nullptr;      // MFMA B-fragment packed filter (ops.conv_filter_fragments): [ceil(OC/64)][4][6][64][8]
  if (wfrag.has_value() && wfrag->defined()) {
    check_cuda(*wfrag, "wfrag");
    TORCH_CHECK(wfrag->scalar_type() == torch::kBFloat16 && wfrag->is_contiguous() &&
                    wfrag->numel() == ((OC + 63) / 64) * 4 * 6 * 64 * 8, "wfrag must be the packed [OC/64][4][6][64][8] filter");
    fptr = wfrag->data_ptr();
  }
  // per-call kernel options (-1: the library default)
  const ConvOpts o{force_generic ? 1 : 0, (int)variant, max_blocks < 0 ? 512 : (int)max_blocks, kernel < 0 ? 5 : (int)kernel,
                   (int)contig};
  auto opts = X.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16);
  torch::Tensor out = nchw_out ? torch::empty({N, OC, OH, OW}, opts) : torch::empty({N * OH * OW, OC}, opts);
  check_rc(nsdb_conv2d_igemm(X.data_ptr(), Wt.data_ptr(), bptr, out.data_ptr(), (int)N, (int)C, (int)H, (int)W,
                             (int)OC, (int)KH, (int)KW, (int)stride, (int)pad, (int)dil, (int)ldw, (int)act,
                             nchw_out ? 1 : 0, out_f32 ? 1 : 0, fptr, &o, cur_stream()),
           "conv2d");
  return out;
}

torch::Tensor im2col(torch::Tensor X, int64_t KH, int64_t KW, int64_t stride, int64_t pad, int64_t dil, int64_t ldk) {
  check_cuda(X, "X");
  TORCH_CHECK(X.scalar_type() == torch::kBFloat16 && X.dim() == 4 && X.is_contiguous(), "X bf16 NCHW contiguous");
  const int64_t N = X.size(0), C = X.size(1), H = X.size(2), W = X.size(3);
  TORCH_CHECK(ldk >= C * KH * KW, "ldk too small");
  const int64_t OH = (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1;
  const int64_t OW = (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1;
  torch::Tensor out = torch::empty({N * OH * OW, ldk}, X.options());
  check_rc(nsdb_im2col(X.data_ptr(), out.data_ptr(), (int)N, (int)C, (int)H, (int)W, (int)KH, (int)KW, (int)stride,
                       (int)pad, (int)dil, (int)ldk, cur_stream()),
           "im2col");
  return out;
}

// Cache warm-up read of each tensor's storage bytes on the current stream (ops.prefetch).
void prefetch(std::vector<torch::Tensor> ts, torch::Tensor sink, int64_t blocks) {
  check_cuda(sink, "sink");
  TORCH_CHECK(sink.scalar_type() == torch::kInt32 && sink.numel() >= 1, "sink must be an int32 scratch word");
  for (auto& t : ts) {
    if (!t.defined() || t.numel() == 0) continue;
    check_cuda(t, "prefetch tensor");
    long long span = 1;                  // elements from the first to the last one the view addresses
    for (int64_t d = 0; d < t.dim(); ++d) span += (t.size(d) - 1) * std::abs(t.stride(d));
    check_rc(nsdb_prefetch(t.data_ptr(), span * (long long)t.element_size(),
                           reinterpret_cast<unsigned*>(sink.data_ptr()), (int)blocks, cur_stream()), "prefetch");
  }
}

torch::Tensor softmax_rows(torch::Tensor X, c10::optional<torch::Tensor> bias, bool out_f32, int64_t mode,
                           bool plain_loads) {
  check_cuda(X, "X");
  TORCH_CHECK(X.dim() == 2 && X.stride(-1) == 1, "X must be 2-D row-contiguous");
  const bool xf = is_f32(X, "X");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == X.size(1), "bias f32[N]");
    bptr = bias->data_ptr<float>();
  }
  auto Y = torch::empty({X.size(0), X.size(1)}, X.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16));
  check_rc(nsdb_softmax_rows(X.data_ptr(), xf, bptr, Y.data_ptr(), out_f32, (int)X.size(0), (int)X.size(1),
                             X.stride(0), Y.stride(0), (int)mode, plain_loads ? 1 : 0, cur_stream()),
           "softmax_rows");
  return Y;
}

torch::Tensor bias_act(torch::Tensor X, c10::optional<torch::Tensor> bias, int64_t bias_mode, int64_t act,
                       double dropout, int64_t seed, bool out_f32) {
  check_cuda(X, "X");
  TORCH_CHECK(X.dim() == 2 && X.is_contiguous(), "X must be contiguous 2-D");
  const bool xf = is_f32(X, "X");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32, "bias f32");
    TORCH_CHECK(bias->numel() == (bias_mode == 1 ? X.size(0) : X.size(1)), "bias length mismatch");
    bptr = bias->data_ptr<float>();
  }
  auto Y = torch::empty_like(X, X.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16));
  check_rc(nsdb_bias_act(X.data_ptr(), xf, bptr, Y.data_ptr(), out_f32, (int)X.size(0), (int)X.size(1),
                         (int)bias_mode, (int)act, (float)dropout, (unsigned long long)seed, cur_stream()),
           "bias_act");
  return Y;
}

std::vector<torch::Tensor> lstm_cell(torch::Tensor gates, c10::optional<torch::Tensor> c_prev, bool h_f32) {
  check_cuda(gates, "gates");
  TORCH_CHECK(gates.dim() == 2 && gates.is_contiguous() && gates.size(1) % 4 == 0, "gates [B,4H] contiguous");
  const bool gf = is_f32(gates, "gates");
  const int64_t B = gates.size(0), H = gates.size(1) / 4;
  const float* cp = nullptr;
  if (c_prev.has_value() && c_prev->defined()) {
    TORCH_CHECK(c_prev->scalar_type() == torch::kFloat32 && c_prev->numel() == B * H && c_prev->is_contiguous(),
                "c_prev f32 [B,H]");
    cp = c_prev->data_ptr<float>();
  }
  auto h = torch::empty({B, H}, gates.options().dtype(h_f32 ? torch::kFloat32 : torch::kBFloat16));
  auto c = torch::empty({B, H}, gates.options().dtype(torch::kFloat32));
  check_rc(nsdb_lstm_cell(gates.data_ptr(), gf, cp, h.data_ptr(), h_f32, c.data_ptr<float>(), (int)B, (int)H,
                          cur_stream()),
           "lstm_cell");
  return {h, c};
}

torch::Tensor lstm_ew(int64_t mode, torch::Tensor a, torch::Tensor b, c10::optional<torch::Tensor> c,
                      c10::optional<torch::Tensor> d) {
  auto chk = [&](const torch::Tensor& t, const char* n) {
    check_cuda(t, n);
    TORCH_CHECK(t.scalar_type() == torch::kFloat32 && t.is_contiguous() && t.numel() == a.numel(),
                n, " must be contiguous f32 of the same size");
  };
  chk(a, "a");
  chk(b, "b");
  const float* cp = nullptr;
  const float* dp = nullptr;
  if (mode == 0) {
    TORCH_CHECK(c.has_value() && d.has_value(), "mode 0 needs 4 inputs");
    chk(*c, "c");
    chk(*d, "d");
    cp = c->data_ptr<float>();
    dp = d->data_ptr<float>();
  }
  auto out = torch::empty_like(a);
  check_rc(nsdb_lstm_ew((int)mode, a.data_ptr<float>(), b.data_ptr<float>(), cp, dp, out.data_ptr<float>(),
                        (long long)a.numel(), cur_stream()),
           "lstm_ew");
  return out;
}

torch::Tensor embedding_bag(torch::Tensor table, torch::Tensor idx, torch::Tensor offsets,
                            c10::optional<torch::Tensor> weights, int64_t mode) {
  check_cuda(table, "table");
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous(), "table [V,D] contiguous");
  const bool tf = is_f32(table, "table");
  TORCH_CHECK(idx.scalar_type() == torch::kInt64 && offsets.scalar_type() == torch::kInt64, "int64 idx/offsets");
  TORCH_CHECK(idx.is_contiguous() && offsets.is_contiguous() && offsets.dim() == 1 && offsets.numel() >= 1,
              "idx/offsets contiguous");
  const float* wp = nullptr;
  if (weights.has_value() && weights->defined()) {
    TORCH_CHECK(weights->scalar_type() == torch::kFloat32 && weights->numel() == idx.numel(), "weights f32[nnz]");
    wp = weights->data_ptr<float>();
  }
  const int64_t Bn = offsets.numel() - 1, D = table.size(1);
  auto out = torch::empty({Bn, D}, table.options().dtype(torch::kFloat32));
  check_rc(nsdb_embedding_bag(table.data_ptr(), tf, (const long long*)idx.data_ptr<int64_t>(), (const long long*)offsets.data_ptr<int64_t>(), wp,
                              out.data_ptr<float>(), (int)Bn, (int)D, (int)mode, cur_stream()),
           "embedding_bag");
  return out;
}

// String columns: bytes u8 [>= payload + 16] (padding read by the dword loads), row bounds as starts / ends i64 [n]
// (a packed column passes offsets[:-1] / offsets[1:]; a gathered view its own arrays).
void check_strings(const torch::Tensor& bytes, const torch::Tensor& st, const torch::Tensor& en) {
  check_cuda(bytes, "bytes");
  check_cuda(st, "starts");
  check_cuda(en, "ends");
  TORCH_CHECK(bytes.scalar_type() == torch::kUInt8 && bytes.dim() == 1 && bytes.is_contiguous(), "bytes u8 1-D");
  for (const torch::Tensor* t : {&st, &en})
    TORCH_CHECK(t->scalar_type() == torch::kInt64 && t->dim() == 1 && (t->numel() <= 1 || t->stride(0) == 1),
                "starts / ends: unit-stride i64");
  TORCH_CHECK(st.numel() == en.numel(), "starts / ends length mismatch");
  TORCH_CHECK(bytes.numel() % 4 == 0 && bytes.numel() >= 16, "bytes must be padded to a multiple of 4, >= 16");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(bytes.data_ptr()) % 4 == 0, "bytes must be 4-byte aligned");
}

torch::Tensor str_hash(torch::Tensor bytes, torch::Tensor st, torch::Tensor en, int64_t payload_end) {
  check_strings(bytes, st, en);
  TORCH_CHECK(payload_end + 16 <= bytes.numel(), "string payload must be followed by >= 16 pad bytes");
  const int64_t n = st.numel();
  auto out = torch::empty({n}, st.options());
  check_rc(nsdb_str_hash(bytes.data_ptr(), st.data_ptr<int64_t>(), en.data_ptr<int64_t>(), n,
                         (uint64_t*)out.data_ptr<int64_t>(), cur_stream()),
           "str_hash");
  return out;
}

// Exact short-string codes (strings.hip str_pack_kernel); the caller guarantees every row is <= L <= 7 bytes.
torch::Tensor str_pack(torch::Tensor bytes, torch::Tensor st, torch::Tensor en, int64_t L) {
  check_strings(bytes, st, en);
  TORCH_CHECK(L >= 0 && L <= 7, "str_pack: L must be in [0, 7]");
  const int64_t n = st.numel();
  auto out = torch::empty({n}, st.options());
  check_rc(nsdb_str_pack(bytes.data_ptr(), st.data_ptr<int64_t>(), en.data_ptr<int64_t>(), n, (int)L,
                         out.data_ptr<int64_t>(), cur_stream()),
           "str_pack");
  return out;
}

torch::Tensor str_like(torch::Tensor bytes, torch::Tensor st, torch::Tensor en, int64_t payload_end,
                       const std::string& pat, std::vector<int64_t> seg_start, std::vector<int64_t> seg_len,
                       bool anchor_start, bool anchor_end, bool negate) {
  check_strings(bytes, st, en);
  TORCH_CHECK(payload_end + 16 <= bytes.numel(), "string payload must be followed by >= 16 pad bytes");
  TORCH_CHECK(seg_start.size() == seg_len.size(), "segment lists differ in length");
  TORCH_CHECK(pat.size() <= 224 && seg_start.size() <= 16, "pattern too long for the kernarg pattern (224 B, 16 segs)");
  std::vector<int> ss(seg_start.begin(), seg_start.end()), sl(seg_len.begin(), seg_len.end());
  const int64_t n = st.numel();
  auto out = torch::empty({n}, bytes.options());
  // floating segments over many rows: the buffer-parallel occurrence-bitmap form (strings.hip like_occ_kernel) when
  // the rows cover the buffer densely (a few rows viewing a large buffer keep the row search: the bitmaps cost the
  // whole buffer)
  const int64_t nseg = (int64_t)ss.size(), nwords = (payload_end + 63) / 64;
  if (!anchor_start && !anchor_end && nseg >= 1 && nseg <= 4 && n >= g_like_occ_min_rows && payload_end <= 256 * n &&
      (reinterpret_cast<uintptr_t>(bytes.data_ptr()) & 15) == 0) {
    auto occ = torch::empty({nseg * nwords}, bytes.options().dtype(torch::kInt64));
    const int rc = nsdb_str_like_occ(bytes.data_ptr(), bytes.numel(), payload_end, st.data_ptr<int64_t>(),
                                     en.data_ptr<int64_t>(), n, (const uint8_t*)pat.data(), (int)pat.size(), ss.data(),
                                     sl.data(), (int)nseg, negate, reinterpret_cast<uint64_t*>(occ.data_ptr<int64_t>()),
                                     out.data_ptr<uint8_t>(), cur_stream());
    if (rc == 0) return out.view(torch::kBool);
    TORCH_CHECK(rc == -4, "str_like_occ failed with code ", rc);      // -4: pattern shape not eligible
  }
  check_rc(nsdb_str_like(bytes.data_ptr(), st.data_ptr<int64_t>(), en.data_ptr<int64_t>(), n, (const uint8_t*)pat.data(),
                         (int)pat.size(), ss.data(), sl.data(), (int)ss.size(), anchor_start, anchor_end, negate,
                         out.data_ptr<uint8_t>(), cur_stream()),
           "str_like");
  return out.view(torch::kBool);
}

// Pack rows idx (or every row when idx is None) of a column into a new padded buffer at out_off. Indices come
// from the column's own row space (the callers derive them on the device).
torch::Tensor str_gather(torch::Tensor bytes, torch::Tensor st, torch::Tensor en, c10::optional<torch::Tensor> idx,
                         torch::Tensor out_off, int64_t out_bytes) {
  check_strings(bytes, st, en);
  check_cuda(out_off, "out_off");
  const int64_t* ip = nullptr;
  int64_t m = st.numel();
  if (idx.has_value() && idx->defined()) {
    check_cuda(*idx, "idx");
    TORCH_CHECK(idx->scalar_type() == torch::kInt64 && idx->is_contiguous() && idx->dim() == 1, "idx i64 1-D");
    ip = idx->data_ptr<int64_t>();
    m = idx->numel();
  }
  TORCH_CHECK(out_off.scalar_type() == torch::kInt64 && out_off.numel() == m + 1, "out_off [m+1]");
  const int64_t padded = ((out_bytes + 16 + 3) / 4) * 4;
  auto dst = torch::zeros({padded}, bytes.options());
  check_rc(nsdb_str_gather(bytes.data_ptr(), st.data_ptr<int64_t>(), en.data_ptr<int64_t>(), ip,
                           out_off.data_ptr<int64_t>(), m, dst.data_ptr(), cur_stream()),
           "str_gather");
  return dst;
}

// out[i] = (a[ia[i]] == b[ib[i]]) byte-exact; ia / ib may be None (identity).
torch::Tensor str_eq_pairs(torch::Tensor a, torch::Tensor sta, torch::Tensor ena, c10::optional<torch::Tensor> ia,
                           torch::Tensor b, torch::Tensor stb, torch::Tensor enb, c10::optional<torch::Tensor> ib,
                           int64_t m) {
  check_strings(a, sta, ena);
  check_strings(b, stb, enb);
  const int64_t* pa = nullptr;
  const int64_t* pb = nullptr;
  if (ia.has_value() && ia->defined()) {
    check_cuda(*ia, "ia");
    TORCH_CHECK(ia->scalar_type() == torch::kInt64 && ia->is_contiguous() && ia->numel() == m, "ia i64 [m]");
    pa = ia->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(sta.numel() >= m, "a has fewer than m rows");
  }
  if (ib.has_value() && ib->defined()) {
    check_cuda(*ib, "ib");
    TORCH_CHECK(ib->scalar_type() == torch::kInt64 && ib->is_contiguous() && ib->numel() == m, "ib i64 [m]");
    pb = ib->data_ptr<int64_t>();
  } else {
    TORCH_CHECK(stb.numel() >= m, "b has fewer than m rows");
  }
  auto out = torch::empty({m}, a.options());
  check_rc(nsdb_str_eq_pairs(a.data_ptr(), sta.data_ptr<int64_t>(), ena.data_ptr<int64_t>(), pa, b.data_ptr(),
                             stb.data_ptr<int64_t>(), enb.data_ptr<int64_t>(), pb, m, out.data_ptr<uint8_t>(),
                             cur_stream()),
           "str_eq_pairs");
  return out.view(torch::kBool);
}

// SUBSTRING of every row: out_off [n+1] (device prefix sums of the clamped lengths), cap = an upper bound of the
// output bytes known on the host (n * length): no device read to size the buffer.
torch::Tensor str_slice(torch::Tensor bytes, torch::Tensor st, torch::Tensor en, int64_t start, torch::Tensor out_off,
                        int64_t cap) {
  check_strings(bytes, st, en);
  check_cuda(out_off, "out_off");
  TORCH_CHECK(start >= 0, "start must be >= 0");
  TORCH_CHECK(out_off.scalar_type() == torch::kInt64 && out_off.numel() == st.numel() + 1, "out_off [n+1]");
  const int64_t padded = ((cap + 16 + 3) / 4) * 4;
  auto dst = torch::zeros({padded}, bytes.options());
  check_rc(nsdb_str_slice(bytes.data_ptr(), st.data_ptr<int64_t>(), start, out_off.data_ptr<int64_t>(), st.numel(),
                          dst.data_ptr(), cur_stream()),
           "str_slice");
  return dst;
}

// Exact group-by of a device int64 key column on the device hash aggregation (relops.hip), returned as
// torch.unique(keys, sorted=True, return_inverse=True) would: (inverse [n] i64, sorted distinct keys [g] i64).
// Only the g distinct keys are sorted.
std::vector<torch::Tensor> hash_group_ids(torch::Tensor keys) {
  check_cuda(keys, "keys");
  TORCH_CHECK(keys.scalar_type() == torch::kInt64 && keys.dim() == 1, "keys must be a 1-D int64 tensor");
  const int64_t n = keys.numel();
  if (n == 0) return {torch::empty({0}, keys.options()), torch::empty({0}, keys.options())};
  auto r = hash_aggregate_impl(keys, c10::nullopt, "sum", true, 0);
  TORCH_CHECK(r[5][2].item<int64_t>() == 1, "hash_group_ids: device table overflow");
  auto sorted = r[0].sort();
  auto rank = torch::empty_like(r[0]);
  rank.index_put_({std::get<1>(sorted)}, torch::arange(r[0].numel(), keys.options()));
  return {rank.index_select(0, r[4]), std::get<0>(sorted)};
}

// Dedup: blocks [n, ...] contiguous (any dtype; bytes per block % 16 == 0) -> [n, S] i64 partial sums.
torch::Tensor block_hash_partial(torch::Tensor blocks) {
  check_cuda(blocks, "blocks");
  TORCH_CHECK(blocks.is_contiguous() && blocks.dim() >= 1, "blocks must be contiguous [n, ...]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(blocks.data_ptr()) % 16 == 0, "blocks must be 16-B aligned");
  const int64_t n = blocks.size(0);
  const int64_t bytes = n ? blocks.numel() / n * blocks.element_size() : 0;
  TORCH_CHECK(bytes % 16 == 0, "bytes per block must be a multiple of 16");
  const int S = nsdb_dedup_splits(n, bytes);
  auto out = torch::empty({n, S}, blocks.options().dtype(torch::kInt64));
  const char* base = (const char*)blocks.data_ptr();
  for (int64_t b0 = 0; b0 < n; b0 += 65535) {           // grid.y limit
    const int64_t nb = std::min<int64_t>(65535, n - b0);
    check_rc(nsdb_block_hash(base + b0 * bytes, nb, bytes / 4, S,
                             (unsigned long long*)out.data_ptr<int64_t>() + b0 * S, cur_stream()),
             "block_hash");
  }
  return out;
}

// max |pool[cand[b]] - blks[b]| per block, [n, S] f32 partials. cand must index rows of pool (the
// caller derives it from a searchsorted over the pool's own keys, so 0 <= cand < pool.size(0)).
torch::Tensor block_maxdiff_partial(torch::Tensor pool, torch::Tensor cand, torch::Tensor blks) {
  check_cuda(pool, "pool");
  check_cuda(cand, "cand");
  check_cuda(blks, "blks");
  TORCH_CHECK(pool.scalar_type() == blks.scalar_type(), "pool/blks dtype mismatch");
  const bool f32 = is_f32(pool, "pool");
  TORCH_CHECK(pool.is_contiguous() && blks.is_contiguous() && cand.is_contiguous(), "contiguous inputs");
  TORCH_CHECK(cand.scalar_type() == torch::kInt64 && cand.dim() == 1 && cand.numel() == blks.size(0), "cand i64 [n]");
  const int64_t n = blks.size(0);
  TORCH_CHECK(pool.size(0) > 0 || n == 0, "empty pool");
  const int64_t elems = n ? blks.numel() / n : 0;
  TORCH_CHECK(pool.numel() == pool.size(0) * elems, "pool/blks block size mismatch");
  const int S = nsdb_dedup_splits(n, elems * blks.element_size());
  auto out = torch::empty({n, S}, blks.options().dtype(torch::kFloat32));
  for (int64_t b0 = 0; b0 < n; b0 += 65535) {
    const int64_t nb = std::min<int64_t>(65535, n - b0);
    check_rc(nsdb_block_maxdiff(pool.data_ptr(), (const long long*)cand.data_ptr<int64_t>() + b0,
                                (const char*)blks.data_ptr() + b0 * elems * blks.element_size(), nb, elems, f32, S,
                                out.data_ptr<float>() + b0 * S, cur_stream()),
             "block_maxdiff");
  }
  return out;
}

// approximate dedup: per-(candidate, split) counts of elements within fp of one query block over its h x w corner
torch::Tensor block_simcount_partial(torch::Tensor pool, torch::Tensor cand, torch::Tensor query, int64_t bc, int64_t h,
                                     int64_t w, double fp) {
  TORCH_CHECK(pool.is_cuda() && pool.is_contiguous() && query.is_contiguous() && cand.is_contiguous(), "device, contiguous");
  TORCH_CHECK(pool.scalar_type() == query.scalar_type(), "pool/query dtype");
  TORCH_CHECK(pool.scalar_type() == torch::kBFloat16 || pool.scalar_type() == torch::kFloat32, "bf16 or f32");
  TORCH_CHECK(cand.scalar_type() == torch::kInt64 && cand.dim() == 1, "cand i64 [n]");
  const int64_t elems = query.numel();
  TORCH_CHECK(pool.dim() >= 1 && pool.size(0) > 0 && pool.numel() == pool.size(0) * elems, "pool rows of query size");
  TORCH_CHECK(elems % bc == 0 && h >= 0 && w >= 0 && h * bc <= elems && w <= bc, "block geometry");
  const int64_t n = cand.size(0);
  const bool f32 = pool.scalar_type() == torch::kFloat32;
  const int S = nsdb_dedup_splits(std::max<int64_t>(n, 1), elems * pool.element_size());
  auto out = torch::empty({n, S}, cand.options().dtype(torch::kInt32));
  for (int64_t b0 = 0; b0 < n; b0 += 65535) {
    const int64_t nb = std::min<int64_t>(65535, n - b0);
    check_rc(nsdb_block_simcount(pool.data_ptr(), (const long long*)cand.data_ptr<int64_t>() + b0, query.data_ptr(), nb,
                                 elems, (int)bc, (int)h, (int)w, (float)fp, f32, S,
                                 reinterpret_cast<unsigned*>(out.data_ptr<int>()) + b0 * S, cur_stream()),
             "block_simcount");
  }
  return out;
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "netsdb_amd CDNA4 (gfx950) HIP kernels";
  register_relops(m);
  register_pipeline(m);
  m.def("gemm_nt", &gemm_nt, "epi(alpha*A@B^T) on MFMA", py::arg("A"), py::arg("B"), py::arg("bias") = py::none(),
        py::arg("bias_mode") = 0, py::arg("act") = 0, py::arg("out_f32") = false, py::arg("alpha") = 1.0,
        py::arg("dropout") = 0.0, py::arg("seed") = 0, py::arg("splits") = 0, py::arg("out") = py::none(),
        py::arg("accumulate") = false, py::arg("cfg") = -1, py::arg("epi") = -1, py::arg("prefetch") = py::none(),
        py::arg("mfma") = 0, py::arg("fixup") = 0);
  m.def("gemm_launch_wgs", [](int64_t M, int64_t N, int64_t K, int64_t batch, int64_t splits, int64_t cfg) {
          return (int64_t)nsdb_gemm_launch_wgs((int)M, (int)N, (int)K, (int)batch, (int)splits, (int)cfg);
        }, "workgroups of the GEMM launch for this shape (splits <= 0: the launcher's choice)",
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("batch") = 1, py::arg("splits") = 0, py::arg("cfg") = -1);
  m.def("prefetch", &prefetch, "warm the caches with a read of each tensor", py::arg("tensors"), py::arg("sink"),
        py::arg("blocks") = 64);
  m.def("gemm_nt_f32", &gemm_nt_f32, "alpha * A.B^T (+C) on the exact-f32 MFMA (16x16x4)", py::arg("A"),
        py::arg("B"), py::arg("alpha") = 1.0, py::arg("out") = py::none(), py::arg("accumulate") = false);
  m.def("gemm_splits", &gemm_splits, py::arg("M"), py::arg("N"), py::arg("K"), py::arg("batch") = 1,
        py::arg("cfg") = -1);
  m.def("gemm_prefetch_eligible", [](int64_t M, int64_t N, int64_t K, int64_t batch, int64_t splits, int64_t cfg) {
          return (bool)nsdb_gemm_prefetch_eligible((int)M, (int)N, (int)K, (int)batch, (int)splits, (int)cfg);
        }, "whether a launch of this shape takes an operand prefetch passed to it (long, one-wave 8-phase GEMM)",
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("batch") = 1, py::arg("splits") = 0, py::arg("cfg") = -1);
  m.def("gemm_nt_softmax", &gemm_nt_softmax, "softmax(alpha A.B^T + bias) fused into the GEMM epilogue",
        py::arg("A"), py::arg("B"), py::arg("bias") = py::none(), py::arg("bias_mode") = 0, py::arg("axis") = 1,
        py::arg("out") = py::none(), py::arg("alpha") = 1.0, py::arg("force_fallback") = false, py::arg("epi") = -1,
        py::arg("stamps") = py::none());
  m.def("conv2d", &conv2d, py::arg("X"), py::arg("W"), py::arg("bias") = py::none(), py::arg("KH") = 1,
        py::arg("KW") = 1, py::arg("stride") = 1, py::arg("pad") = 0, py::arg("dil") = 1, py::arg("act") = 0,
        py::arg("nchw_out") = false, py::arg("out_f32") = false, py::arg("wfrag") = py::none(), py::arg("kernel") = -1,
        py::arg("max_blocks") = -1, py::arg("force_generic") = false, py::arg("variant") = 0, py::arg("contig") = 0);
  m.def("im2col", &im2col);
  m.def("softmax_rows", &softmax_rows, py::arg("X"), py::arg("bias") = py::none(), py::arg("out_f32") = true,
        py::arg("mode") = 0, py::arg("plain_loads") = false);
  m.def("bias_act", &bias_act, py::arg("X"), py::arg("bias") = py::none(), py::arg("bias_mode") = 2,
        py::arg("act") = 0, py::arg("dropout") = 0.0, py::arg("seed") = 0, py::arg("out_f32") = false);
  m.def("gemm_nt_bseg", &gemm_nt_bseg, py::arg("A"), py::arg("Bg"), py::arg("bias") = py::none(),
        py::arg("bias_mode") = 0, py::arg("act") = 0, py::arg("out_f32") = true, py::arg("alpha") = 1.0,
        py::arg("dropout") = 0.0, py::arg("seed") = 0, py::arg("out") = py::none());
  m.def("lstm_ew", &lstm_ew, py::arg("mode"), py::arg("a"), py::arg("b"), py::arg("c") = py::none(),
        py::arg("d") = py::none());
  m.def("lstm_cell", &lstm_cell, py::arg("gates"), py::arg("c_prev") = py::none(), py::arg("h_f32") = true);
  m.def("embedding_bag", &embedding_bag, py::arg("table"), py::arg("idx"), py::arg("offsets"),
        py::arg("weights") = py::none(), py::arg("mode") = 0);
  m.def("block_hash_partial", &block_hash_partial, "dedup: per-(block, split) partial content-hash sums");
  m.def("block_simcount_partial", &block_simcount_partial,
        "approximate dedup: per-(candidate, split) counts of elements within fp of a query block");
  m.def("block_maxdiff_partial", &block_maxdiff_partial, "dedup: per-(block, split) max |pool[cand] - blk|");
  m.def("hash_group_ids", &hash_group_ids, "exact group-by of a device int64 column: (inverse, sorted keys)");
  m.def("str_hash", &str_hash, "64-bit hash per string of a device string column");
  m.def("str_pack", &str_pack, "exact order-preserving int64 code per string of <= 7 bytes");
  m.def("str_like_occ_min_rows", [](int64_t v) { g_like_occ_min_rows = v <= 0 ? (int64_t(1) << 62) : v; },
        "rows from which str_like takes the occurrence-bitmap form (<= 0: never; A/B and tests)");
  m.def("str_like", &str_like, "SQL LIKE over a device string column (segments of the pattern bytes)");
  m.def("str_slice", &str_slice, "SUBSTRING of every row of a device string column (no host read)");
  m.def("str_eq_pairs", &str_eq_pairs, "byte-exact equality of string row pairs a[ia[i]] == b[ib[i]]",
        py::arg("a"), py::arg("sta"), py::arg("ena"), py::arg("ia"), py::arg("b"), py::arg("stb"), py::arg("enb"),
        py::arg("ib"), py::arg("m"));
  m.def("str_gather", &str_gather, "pack rows of a device string column into a new padded byte buffer",
        py::arg("bytes"), py::arg("starts"), py::arg("ends"), py::arg("idx"), py::arg("out_off"), py::arg("out_bytes"));
}
