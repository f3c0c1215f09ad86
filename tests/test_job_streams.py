"""Concurrent jobs on HIP streams (execution/streams.py; reference QuerySchedulerServer job scheduling)."""
import tempfile

import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.execution.streams import JobStreams
from netsdb_amd.models import conv2d as cv
from netsdb_amd.models import ff
from netsdb_amd.models.blocks import to_tensor
from netsdb_amd.objects.record import RecordBatch


def _run(dev, overlap):
    c = PDBClient(root=tempfile.mkdtemp(), device=dev)
    ff.load_model(c, "ff", 64, 1024, 128, 100, 32, 256, seed=0)
    c.create_database("conv2d")
    cv.load_images(c, "conv2d", "img", 4, 3, 32, 32, seed=3)
    w, b = cv.random_kernel(16, 3, 7, 7, seed=5, device=dev)

    def conv():
        cv.conv2d_memfuse_inference(c, "conv2d", "img", "out", w, b)

    for i in range(3):
        if overlap:
            h = c.submit_job(conv, independent=True)
        ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "output", dropout_rate=0.0, seed=i)
        if overlap:
            h.wait()
        else:
            conv()
    c.wait_jobs()
    rb = RecordBatch.concat(c.get_set_batches("conv2d", "out"))
    order = torch.argsort(rb.columns["key"])
    return to_tensor(c, "ff", "output").float().cpu(), rb.columns["data"][order.to(rb.columns["data"].device)].float().cpu()


def test_job_streams_cpu_inline():
    js = JobStreams("cpu")
    h = js.submit(lambda x: x + 1, 41)
    assert h.done() and h.wait() == 42 and h.synchronize() == 42
    js.wait_all()


def test_overlapped_jobs_match_serial_cpu():
    a_ff, a_cv = _run("cpu", False)
    b_ff, b_cv = _run("cpu", True)
    assert torch.equal(a_ff, b_ff) and torch.equal(a_cv, b_cv)


@pytest.mark.gpu
def test_overlapped_jobs_match_serial_gpu():
    a_ff, a_cv = _run("cuda:0", False)
    b_ff, b_cv = _run("cuda:0", True)
    assert torch.equal(a_ff, b_ff)
    assert torch.equal(a_cv, b_cv)


@pytest.mark.gpu
def test_submit_orders_after_caller_stream_gpu():
    js = JobStreams("cuda:0")
    x = torch.zeros(1 << 20, device="cuda:0")
    torch.cuda._sleep(2_000_000)          # long-running producer on the caller's stream
    x.add_(1)
    h = js.submit(lambda: x * 2)          # dependent job: must see x == 1
    out = h.wait()
    torch.cuda.synchronize()
    assert torch.all(out == 2)


def _long_splitk_operands(dev):
    # 1024 x 1024 x 65536: 16 tiles x 16 splits = 256 workgroups of 64 k-tiles (a prefetch-eligible launch)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.empty(1024, 65536, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    B = (torch.empty(1024, 65536, device=dev).uniform_(-1, 1, generator=g) * 0.01).to(torch.bfloat16)
    return A, B


@pytest.mark.gpu
def test_operand_prefetch_is_taken_once_and_exact_gpu():
    """An operand prefetch armed on the stream is taken by the next long 8-phase GEMM only (results bitwise equal
    to an unarmed launch), not by a short GEMM before it, and never by a GEMM on another lane."""
    from netsdb_amd import ops
    from netsdb_amd.execution import streams

    dev = "cuda:0"
    A, B = _long_splitk_operands(dev)
    W2 = torch.randn(14588, 1000, device=dev).to(torch.bfloat16)
    ref = ops.gemm_nt(A, B, out_dtype=torch.float32)
    js = JobStreams(dev, lanes=1)
    assert streams.arm_operand_prefetch(W2)
    a = torch.randn(256, 256, device=dev).to(torch.bfloat16)
    ops.gemm_nt(a, a)                                     # short: does not take it
    other = js.submit(lambda: ops.gemm_nt(A, B, out_dtype=torch.float32), independent=True).synchronize()
    assert streams._armed_pf, "a GEMM on another stream took the prefetch"
    C = ops.gemm_nt(A, B, out_dtype=torch.float32)        # long split-K: takes it
    torch.cuda.synchronize()
    assert not streams._armed_pf
    assert torch.equal(C, ref) and torch.equal(other, ref)


def test_prefetch_api_cpu():
    """CPU: an operand prefetch of a host tensor is refused and nothing is armed."""
    from netsdb_amd.execution import streams

    assert streams.arm_operand_prefetch(torch.zeros(4)) is False
    assert streams.take_operand_prefetch("cpu") is None
