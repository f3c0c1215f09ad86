// PyTorch bindings of the GEMM STUDY build (module netsdb_amd._hip_study): the diagnostic / rejected
// variants of the block GEMM (csrc/study/gemm_study.hip), kept for A/B scripts; never loaded
// by the product.
// Every op checks device/dtype/shape on the host BEFORE launching (a bad shape must never reach
// the GPU) and launches on the current HIP stream so ops compose with hipGraph capture.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <map>
#include <vector>
#include <mutex>
#include <utility>

extern "C" {
int nsdb_study_gemm_splits(int M, int N, int K, int batch);
void nsdb_study_gemm_force_config(int cfg);
void nsdb_study_gemm_set_stamps(void* ptr);
void nsdb_study_gemm_set_adapt(int on);
void nsdb_study_gemm_steal(int tq, int ch);
void nsdb_study_gemm_set_steal(int on);
void nsdb_study_tail_trigger_arm(void* flag, unsigned value);
int nsdb_study_tail_trigger_consumed();
void nsdb_study_tail_trigger_disarm();
int nsdb_study_stream_wait_value(hipStream_t stream, void* flag, unsigned value);
int nsdb_study_gemm_adapt_state(int M, int N, int K, float* out);
int nsdb_study_gemm_nt_bf16(const void* A, const void* B, void* C, float* ws, const float* bias, int M, int N, int K,
                      long long lda, long long ldb, long long ldc, long long sA, long long sB, long long sC,
                      long long sBias, int batch, int splits, int act, int bias_mode, int out_f32, float alpha,
                      float dropout, unsigned long long seed, int accumulate, long long seg_k, long long seg_stride_b, hipStream_t stream);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

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
torch::Tensor gemm_nt(torch::Tensor A, torch::Tensor B, c10::optional<torch::Tensor> bias, int64_t bias_mode,
                      int64_t act, bool out_f32, double alpha, double dropout, int64_t seed, int64_t splits,
                      c10::optional<torch::Tensor> out, bool accumulate) {
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
  int s = splits > 0 ? (int)splits : nsdb_study_gemm_splits((int)M, (int)N, (int)K, (int)batch);
  torch::Tensor ws;
  float* wsp = nullptr;
  if (s > 1) {
    ws = torch::empty({batch * s * M * N}, A.options().dtype(torch::kFloat32));
    wsp = ws.data_ptr<float>();
  }
  const int rc = nsdb_study_gemm_nt_bf16(
      A.data_ptr(), B.data_ptr(), C.data_ptr(), wsp, bptr, (int)M, (int)N, (int)K, A.stride(-2), B.stride(-2),
      C.stride(-2), batched ? A.stride(0) : 0, batched ? B.stride(0) : 0, batched ? C.stride(0) : 0, sBias,
      (int)batch, s, (int)act, (int)bias_mode, out_f32 ? 1 : 0, (float)alpha, (float)dropout,
      (unsigned long long)seed, accumulate ? 1 : 0, 0, 0, cur_stream());
  check_rc(rc, "gemm_nt");
  return C;
}

// Study path: A/B as K-tiled panels [K/64][ldt][64] bf16 (ldt >= rows, multiple of 256 not required);
// runs the 8-phase kernel's K-tiled variant. C [M,N] f32|bf16.
torch::Tensor gemm_nt_ktiled(torch::Tensor Ap, torch::Tensor Bp, int64_t M, int64_t N, int64_t K, bool out_f32) {
  check_cuda(Ap, "A");
  check_cuda(Bp, "B");
  TORCH_CHECK(Ap.scalar_type() == torch::kBFloat16 && Bp.scalar_type() == torch::kBFloat16, "A,B must be bf16");
  TORCH_CHECK(Ap.dim() == 3 && Bp.dim() == 3 && Ap.is_contiguous() && Bp.is_contiguous(), "A,B [K/64][ld][64]");
  TORCH_CHECK(Ap.size(2) == 64 && Bp.size(2) == 64 && K % 64 == 0 && Ap.size(0) == K / 64 && Bp.size(0) == K / 64,
              "K-tiled panels must hold K/64 slabs of 64");
  TORCH_CHECK(Ap.size(1) >= M && Bp.size(1) >= N, "panel rows < M/N");
  auto C = torch::empty({M, N}, Ap.options().dtype(out_f32 ? torch::kFloat32 : torch::kBFloat16));
  nsdb_study_gemm_force_config(11);
  const int s = nsdb_study_gemm_splits((int)M, (int)N, (int)K, 1);
  torch::Tensor ws;
  float* wsp = nullptr;
  if (s > 1) {
    ws = torch::empty({s * M * N}, Ap.options().dtype(torch::kFloat32));
    wsp = ws.data_ptr<float>();
  }
  const int rc = nsdb_study_gemm_nt_bf16(Ap.data_ptr(), Bp.data_ptr(), C.data_ptr(), wsp, nullptr, (int)M, (int)N, (int)K,
                                   Ap.size(1), Bp.size(1), N, 0, 0, 0, 0, 1, s, 0, 0, out_f32 ? 1 : 0, 1.f, 0.f, 0, 0,
                                   0, 0, cur_stream());
  nsdb_study_gemm_force_config(-1);
  check_rc(rc, "gemm_nt_ktiled");
  return C;
}

int64_t gemm_splits(int64_t M, int64_t N, int64_t K, int64_t batch) {
  return nsdb_study_gemm_splits((int)M, (int)N, (int)K, (int)batch);
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "netsdb_amd GEMM STUDY kernels (diagnostic variants; not part of the product build)";
  m.def("gemm_nt", &gemm_nt, "epi(alpha*A@B^T) under the study launcher (forced config)", py::arg("A"), py::arg("B"),
        py::arg("bias") = py::none(), py::arg("bias_mode") = 0, py::arg("act") = 0, py::arg("out_f32") = false,
        py::arg("alpha") = 1.0, py::arg("dropout") = 0.0, py::arg("seed") = 0, py::arg("splits") = 0,
        py::arg("out") = py::none(), py::arg("accumulate") = false);
  m.def("gemm_splits", &gemm_splits);
  m.def("gemm_force_config", [](int64_t cfg) { nsdb_study_gemm_force_config((int)cfg); },
        "study config (-1 auto; 3-26 8-phase variants / w4 / w4r / steal / fix-up)");
  m.def("gemm_set_stamps", [](int64_t ptr) { nsdb_study_gemm_set_stamps(reinterpret_cast<void*>(ptr)); });
  m.def("gemm_set_adapt", [](int64_t on) { nsdb_study_gemm_set_adapt((int)on); });
  m.def("gemm_adapt_state", [](int64_t M, int64_t N, int64_t K) {
        std::vector<float> buf(128);
        const int n = nsdb_study_gemm_adapt_state((int)M, (int)N, (int)K, buf.data());
        return py::make_tuple(n, buf);
      });
  m.def("gemm_set_steal", [](int64_t on) { nsdb_study_gemm_set_steal((int)on); });
  m.def("gemm_steal", [](int64_t tq, int64_t ch) { nsdb_study_gemm_steal((int)tq, (int)ch); });
  m.def("gemm_nt_ktiled", &gemm_nt_ktiled);
}
