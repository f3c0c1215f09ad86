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


def test_tail_trigger_cpu_is_inert():
    from netsdb_amd.execution.streams import TailTrigger

    t = TailTrigger("cpu").arm()
    assert t.flag is None and not t.gate(None)
    js = JobStreams("cpu")
    assert js.submit(lambda: 7, start_on=t).wait() == 7


def _long_splitk_operands(dev):
    # 1024 x 1024 x 65536: 16 tiles x 16 splits = 256 workgroups of 64 k-tiles (a tail-trigger launch)
    g = torch.Generator(device=dev).manual_seed(0)
    A = torch.empty(1024, 65536, device=dev).uniform_(-1, 1, generator=g).to(torch.bfloat16)
    B = (torch.empty(1024, 65536, device=dev).uniform_(-1, 1, generator=g) * 0.01).to(torch.bfloat16)
    return A, B


@pytest.mark.gpu
def test_tail_gated_job_gpu():
    """A job gated on the tail trigger of a long split-K GEMM runs after the GEMM's first workgroup finishes:
    results of both are exact vs ungated runs, the gate was installed and the flag carries the epoch."""
    from netsdb_amd import ops
    from netsdb_amd.execution.streams import TailTrigger

    dev = "cuda:0"
    A, B = _long_splitk_operands(dev)
    assert ops.gemm_splits(1024, 1024, 65536) == 16
    ref = ops.gemm_nt(A, B, out_dtype=torch.float32)
    x = torch.arange(1 << 20, device=dev, dtype=torch.float32)
    js = JobStreams(dev, lanes=1)
    trig = TailTrigger(dev)
    for it in range(3):
        trig.arm()
        C = ops.gemm_nt(A, B, out_dtype=torch.float32)
        h = js.submit(lambda: x * 2 + it, independent=True, start_on=trig)
        y = h.wait()
        torch.cuda.synchronize()
        assert torch.equal(C, ref)
        assert torch.equal(y, x * 2 + it)
        assert trig.gated == it + 1 and int(trig.flag.item()) == trig.epoch


@pytest.mark.gpu
def test_tail_trigger_unconsumed_does_not_gate_gpu():
    """Armed but no qualifying GEMM launched (short K): the job runs ungated (no wait that could never end)."""
    from netsdb_amd import ops
    from netsdb_amd.execution.streams import TailTrigger

    dev = "cuda:0"
    trig = TailTrigger(dev).arm()
    a = torch.randn(512, 512, device=dev).to(torch.bfloat16)
    ops.gemm_nt(a, a)
    js = JobStreams(dev, lanes=1)
    y = js.submit(lambda: a.float().sum(), independent=True, start_on=trig).synchronize()
    assert trig.gated == 0 and torch.isfinite(y)


@pytest.mark.gpu
def test_tail_trigger_is_per_stream_gpu():
    """A trigger armed on one job lane (its HIP stream) is invisible to a long GEMM enqueued on ANOTHER lane at
    the same time: that GEMM neither takes it nor raises its flag; the armed lane's own GEMM then does. (The
    kernel library holds no process-wide launch state: a forced config or a trigger belongs to one call.)"""
    from netsdb_amd import ops
    from netsdb_amd.execution.streams import TailTrigger

    dev = "cuda:0"
    A, B = _long_splitk_operands(dev)
    ref = ops.gemm_nt(A, B, out_dtype=torch.float32)
    js = JobStreams(dev, lanes=2)
    s_armed, s_other = js.stream(0), js.stream(1)
    trig = TailTrigger(dev)
    with torch.cuda.stream(s_armed):
        trig.arm()
    other = js.submit(lambda: ops.gemm_nt(A, B, out_dtype=torch.float32), lane=1, independent=True)
    C_other = other.synchronize()
    assert not trig.consumed and int(trig.flag.item()) == 0
    assert torch.equal(C_other, ref)
    # a forced config on the other lane's calls does not change this lane's choice either
    C_forced = js.submit(lambda: ops.gemm_nt(A, B, out_dtype=torch.float32, cfg=0), lane=1, independent=True)
    with torch.cuda.stream(s_armed):
        C_armed = ops.gemm_nt(A, B, out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert trig.consumed and int(trig.flag.item()) == trig.epoch
    assert torch.equal(C_armed, ref)
    assert (C_forced.synchronize() - ref).abs().max().item() <= 1e-3 * ref.abs().max().item()


@pytest.mark.gpu
def test_start_gate_reserves_cus_and_gates_job_gpu():
    """A START gate: the long split-K GEMM that takes it leaves reserve_cus CUs free (fewer split-K slices, exact
    result vs an ungated launch with the same splits), every workgroup adds 1 to the flag when it starts, and the
    gated job (sized to the reserved CUs) runs once all have started; over repeated launches the flag carries the
    running workgroup count. Conv2d with a 16-block grid (what bench.py --overlap beside runs) stays exact."""
    from netsdb_amd import _ext, ops
    from netsdb_amd.execution.streams import TailTrigger

    dev = "cuda:0"
    A, B = _long_splitk_operands(dev)
    h = _ext.hip()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    s_res = ops._reserve_cus_splits(h, dev, 1024, 1024, 65536, 1, 0, -1, 16)
    wgs = h.gemm_launch_wgs(1024, 1024, 65536, 1, s_res, -1)
    assert wgs <= cus - 16 and s_res < ops.gemm_splits(1024, 1024, 65536)
    ref = ops.gemm_nt(A, B, out_dtype=torch.float32, splits=s_res)
    X = torch.empty(6, 3, 112, 112, device=dev).uniform_(-1, 1).to(torch.bfloat16)
    Wf = ops.pad_k(torch.empty(64, 147, device=dev).uniform_(-0.1, 0.1)).to(torch.bfloat16).contiguous()
    bias = torch.randn(64, device=dev)
    yref = ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)
    js = JobStreams(dev, lanes=1)
    gate = TailTrigger(dev, mode="start", reserve_cus=16)

    def conv_job():
        with ops.kernel_options(conv_blocks=16):
            return ops.conv2d(X, Wf, bias, 7, 7, 1, 0, nchw_out=True)

    for it in range(3):
        gate.arm()
        C = ops.gemm_nt(A, B, out_dtype=torch.float32)
        y = js.submit(conv_job, independent=True, start_on=gate).wait()
        torch.cuda.synchronize()
        assert torch.equal(C, ref)
        assert torch.equal(y, yref)
        assert gate.gated == it + 1 and int(gate.flag.item()) == gate.count == wgs * (it + 1)


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


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["tail", "start"])
def test_trigger_taken_by_failed_launch_does_not_gate_gpu(mode):
    """A long GEMM takes the armed trigger but its launch is rejected (bad output tensor): the trigger is handed
    back, so the job submitted on it runs ungated instead of waiting on the GPU for a flag no kernel raises."""
    from netsdb_amd import ops
    from netsdb_amd.execution.streams import TailTrigger

    dev = "cuda:0"
    A, B = _long_splitk_operands(dev)
    trig = TailTrigger(dev, mode=mode, reserve_cus=16).arm()
    bad = torch.empty(3, 3, device=dev, dtype=torch.float16)
    with pytest.raises(RuntimeError):
        ops.gemm_nt(A, B, out_dtype=torch.float32, out=bad)
    js = JobStreams(dev, lanes=1)
    y = js.submit(lambda: A[:4, :4].float().sum(), independent=True, start_on=trig).synchronize()
    assert trig.gated == 0 and torch.isfinite(y) and trig.count == 0


def test_start_gate_and_prefetch_api_cpu():
    """CPU: a start gate is inert (no flag, nothing gated), an operand prefetch of a host tensor is refused, and
    an unknown trigger mode is rejected."""
    from netsdb_amd.execution import streams
    from netsdb_amd.execution.streams import TailTrigger

    g = TailTrigger("cpu", mode="start", reserve_cus=16).arm()
    assert g.flag is None and g.gate(None) is False and g.count == 0
    assert streams.arm_operand_prefetch(torch.zeros(4)) is False
    assert streams.take_operand_prefetch("cpu") is None
    with pytest.raises(ValueError):
        TailTrigger("cpu", mode="middle")
