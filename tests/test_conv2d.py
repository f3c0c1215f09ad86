"""conv2d inference plans vs torch fp32 conv2d (reference: PipelinedConv2dMemFuseTest.cc,
Conv2dProjTest.cc)."""
import pytest
import torch

from netsdb_amd.client import PDBClient
from netsdb_amd.models import conv2d as cv
from netsdb_amd.models.blocks import to_tensor
from netsdb_amd.objects.record import RecordBatch


def _setup(tmp_path, device):
    c = PDBClient(root=str(tmp_path), device=device)
    c.create_database("conv2d")
    cv.load_images(c, "conv2d", "img", 5, 3, 20, 18, page_images=2)
    w, b = cv.random_kernel(8, 3, 7, 7, device=device)
    return c, w, b


def _all_images(c, name):
    bs = c.get_set_batches("conv2d", name)
    rb = RecordBatch.concat(bs)
    order = torch.argsort(rb.columns["key"])
    return rb.columns["data"][order.to(rb.columns["data"].device)].float().cpu()


def _check(c, out_name, w, b):
    x = _all_images(c, "img")
    ref = torch.nn.functional.conv2d(x, w.cpu().to(torch.bfloat16).float(), b.cpu())
    y = _all_images(c, out_name)
    torch.testing.assert_close(y, ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_memfuse(tmp_path, device):
    c, w, b = _setup(tmp_path, device)
    cv.conv2d_memfuse_inference(c, "conv2d", "img", "out", w, b)
    _check(c, "out", w, b)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_conv_proj_spatial(tmp_path, device):
    c, w, b = _setup(tmp_path, device)
    from netsdb_amd.computations import ScanSet, WriteSet
    from netsdb_amd.objects.builtin import Image

    c.create_set("conv2d", "out2", Image)
    sel = cv.Conv2DSelect(w, b, mode="eigen-spatial").set_input(ScanSet("conv2d", "img", Image))
    c.execute_computations(WriteSet("conv2d", "out2").set_input(sel))
    _check(c, "out2", w, b)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda:0", marks=pytest.mark.gpu)])
def test_spatial_rewriting_plan(tmp_path, device):
    c, w, b = _setup(tmp_path, device)
    cv.conv2d_spatial_inference(c, "conv2d", "img", "res", w, b, block_x=16, block_y=16)
    res = to_tensor(c, "conv2d", "res").float().cpu()        # [N*OH*OW, OC]
    x = _all_images(c, "img")
    ref = torch.nn.functional.conv2d(x, w.cpu().to(torch.bfloat16).float(), b.cpu())
    ref = ref.permute(0, 2, 3, 1).reshape(-1, w.shape[0])
    torch.testing.assert_close(res, ref, atol=5e-2, rtol=5e-2)


def test_kernel_options_are_per_thread_and_scoped():
    """Kernel launch options (conv row kernel, grid cap, ...) live in the calling thread's scope and are passed per
    call: another thread (a server request, a job lane on its own thread) never sees them, and they end with the
    block. Unknown options are rejected."""
    import threading

    from netsdb_amd import ops

    seen = {}
    go, done = threading.Event(), threading.Event()

    def other():
        go.wait(10)
        seen["other"] = ops._kopt("conv_kernel", -1)
        done.set()

    t = threading.Thread(target=other)
    t.start()
    with ops.kernel_options(conv_kernel=1, conv_blocks=0):
        with ops.kernel_options(conv_kernel=0):
            seen["nested"] = (ops._kopt("conv_kernel", -1), ops._kopt("conv_blocks", -1))
        seen["outer"] = ops._kopt("conv_kernel", -1)
        go.set()
        done.wait(10)
    t.join(10)
    seen["after"] = ops._kopt("conv_kernel", -1)
    assert seen == {"nested": (0, 0), "outer": 1, "other": -1, "after": -1}
    prev = ops.set_kernel_options(conv_generic=True)
    assert ops._kopt("conv_generic", False) is True
    ops.restore_kernel_options(prev)
    assert ops._kopt("conv_generic", False) is False
    import pytest

    with pytest.raises(ValueError):
        with ops.kernel_options(conv_kernal=5):
            pass
