"""Captured jobs (execution/graphs.py): a job's kernels recorded once into a HIP graph and replayed."""
import tempfile
import time

import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.models import conv2d as cv
from netsdb_amd.models import ff
from netsdb_amd.models.blocks import to_tensor


def test_capture_needs_gpu():
    c = PDBClient(root=tempfile.mkdtemp(), device="cpu")
    with pytest.raises(RuntimeError):
        c.capture_job(lambda: None)


def _ff_client(seed):
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    ff.load_model(c, "ff", 64, 1024, 128, 100, 32, 256, seed=seed)
    return c


def _unit(c):
    ff.inference_unit(c, "ff", "w1", "wo", "inputs", "b1", "bo", "output", dropout_rate=0.0, seed=0)


@pytest.mark.gpu
def test_captured_ff_job_replays_exactly_and_reads_inputs_in_place():
    c = _ff_client(0)
    _unit(c)
    eager = to_tensor(c, "ff", "output").float().clone()
    cj = c.capture_job(_unit, c, inputs=[("ff", "inputs")])
    cj.replay()
    torch.cuda.synchronize()
    assert torch.equal(to_tensor(c, "ff", "output").float(), eager)
    # new inputs written into the captured input panel; the replay reads them
    other = _ff_client(0)
    g = torch.Generator(device="cuda:0").manual_seed(5)
    newx = torch.rand(other.storage.get_set("ff", "inputs").panel.shape, device="cuda:0", generator=g).to(
        other.storage.get_set("ff", "inputs").panel.dtype) - 0.5
    other.storage.get_set("ff", "inputs").panel.copy_(newx)
    _unit(other)
    ref = to_tensor(other, "ff", "output").float()
    cj.input("ff", "inputs").copy_(newx)
    cj.replay()
    torch.cuda.synchronize()
    assert torch.equal(to_tensor(c, "ff", "output").float(), ref)
    # launch-bound loop: replay vs the eager engine path (printed; the graph must not be slower)
    n = 20
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        _unit(other)
    torch.cuda.synchronize()
    t_eager = (time.perf_counter() - t0) / n
    t0 = time.perf_counter()
    for _ in range(n):
        cj.replay()
    torch.cuda.synchronize()
    t_graph = (time.perf_counter() - t0) / n
    print(f"small FF inference_unit: eager {t_eager * 1e6:.0f} us/step, graph replay {t_graph * 1e6:.0f} us/step")
    assert t_graph < t_eager


@pytest.mark.gpu
def test_captured_conv_job():
    c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
    c.create_database("conv2d")
    cv.load_images(c, "conv2d", "img", 4, 3, 32, 32, seed=1)
    w, b = cv.random_kernel(16, 3, 7, 7, seed=2, device="cuda:0")

    def job():
        cv.conv2d_memfuse_inference(c, "conv2d", "img", "out", w, b)

    job()
    eager = c.storage.get_set("conv2d", "out").all().columns["data"].float().clone()
    cj = c.capture_job(job)
    cj.replay()
    torch.cuda.synchronize()
    assert torch.equal(c.storage.get_set("conv2d", "out").all().columns["data"].float(), eager)


@pytest.mark.gpu
def test_captured_lstm_sequence():
    """An LSTM time-step job (LSTMTest.cc's graph, lowered to one stacked gate GEMM + lstm_cell) captured once;
    a 6-step recurrence = replays with h_t / c_t copied into the captured h_t_1 / c_t_1 panels in between,
    identical to the eager engine run of the same sequence."""
    from netsdb_amd.models import lstm

    def make():
        c = PDBClient(root=tempfile.mkdtemp(), device="cuda:0")
        lstm.load_lstm_sets(c, "lstm", 256, 64, 128, 64, 64, seed=3, dtype=torch.bfloat16)
        return c

    def step(c):
        lstm.lstm_step_graph(c, "lstm")

    def carry(c):
        for src, dst in (("h_t", "h_t_1"), ("c_t", "c_t_1")):
            c.storage.get_set("lstm", dst).panel.copy_(c.storage.get_set("lstm", src).panel)

    eager = make()
    step(eager)                     # first step untimed (plan compile, derived weights)
    carry(eager)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        step(eager)
        carry(eager)
    torch.cuda.synchronize()
    t_eager = (time.perf_counter() - t0) / 5
    ref = to_tensor(eager, "lstm", "h_t_1").float()

    c = make()
    cj = c.capture_job(step, c, inputs=[("lstm", "h_t_1"), ("lstm", "c_t_1"), ("lstm", "x_t")])
    # capture ran the step twice on the initial state (warmup + recording) without carrying: restart from it
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(6):
        cj.replay()
        carry(c)
    torch.cuda.synchronize()
    t_graph = (time.perf_counter() - t0) / 6
    got = to_tensor(c, "lstm", "h_t_1").float()
    assert torch.equal(got, ref)
    print(f"LSTM step (256 -> 128, batch 64): eager {t_eager * 1e6:.0f} us, graph replay {t_graph * 1e6:.0f} us")
