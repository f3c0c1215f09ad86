"""Diagnostic: a START-gated long GEMM leaves 64 CUs free and the fused softmax (228 tiles) is gated on it from a job
lane; prints GEMM / softmax times, the softmax start offset and the tiles' poll / entry spread (phase stamps).
Backs tests/test_softmax_gemm.py::test_softmax_gemm_not_co_resident_gpu."""
import sys, os, torch, json
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from netsdb_amd import _ext, ops
from netsdb_amd.execution.streams import JobStreams, TailTrigger
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(11)
M, N, K = 1000, 14588, 1000
A = torch.empty(M, K, device=dev).uniform_(0, 1, generator=g).to(torch.bfloat16)
B = (torch.empty(N, K, device=dev).uniform_(-1, 1, generator=g) * 0.055).to(torch.bfloat16)
bias = torch.empty(N, device=dev).uniform_(-0.1, 0.1, generator=g)
GA = torch.empty(1024, 1 << 20, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
GB = (torch.empty(1024, 1 << 20, device=dev).uniform_(-1, 1, generator=g) * 1e-3).to(torch.bfloat16)
tiles = 4 * 57
st = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
js = JobStreams(dev, lanes=1)
for rep in range(3):
    torch.cuda.synchronize()
    gate = TailTrigger(dev, mode="start", reserve_cus=64).arm()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[0].record()
    C = ops.gemm_nt(GA, GB, out_dtype=torch.float32)
    e[1].record()
    s = js.stream(0)
    def job():
        e[2].record(s)
        y = _ext.hip().gemm_nt_softmax(A, B, bias, ops.BIAS_COL, 1, None, 1.0, False, -1, st)
        e[3].record(s)
        return y
    h = js.submit(job, independent=True, start_on=gate)
    h.synchronize(); torch.cuda.synchronize()
    s8 = st.view(tiles, 8).cpu()
    poll = (s8[:, 3] - s8[:, 2]) / 100.0
    ent = (s8[:, 0] - s8[:, 0].min()) / 100.0
    print(json.dumps({"gemm_ms": e[0].elapsed_time(e[1]), "soft_ms": e[2].elapsed_time(e[3]),
                      "soft_start_after_gemm_start_ms": e[0].elapsed_time(e[2]),
                      "gated": gate.gated, "flag": int(gate.flag.item()), "count": gate.count,
                      "poll_us_max": float(poll.max()), "entry_spread_us": float(ent.max()),
                      "stream": s.cuda_stream, "default": torch.cuda.current_stream().cuda_stream}), flush=True)
