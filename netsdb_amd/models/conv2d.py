"""Convolution inference as netsDB UDFs.

Reference: src/conv2d_memory_fusion (spatial rewriting: ImageToChunks -> ImageChunksToBlock ->
ImageBlockToMatrix builds the im2col matrix "image_flat" (N*OH*OW x C*KH*KW+1), KernelToChunks
... KernelBiasJoin builds "kernel_flat" with the bias as an extra column, then FFTransposeMult +
FFAggMatrix multiply them; ConvResultToChunks/ConvChunksToImage reshape back) and src/conv2d_proj
(Conv2DSelect: conv as one transformation UDF per image, "aten-conv2d" or "eigen-spatial").
Driver: src/tests/source/PipelinedConv2dMemFuseTest.cc, Conv2dProjTest.cc (100 images 3x112x112,
64 filters 7x7x3, stride 1, no padding).

MI355X-native plans:
  * ``Conv2DMemFuse``  — the memory-fusion idea taken to its end: the im2col rows are never
    materialised; each page of images goes through ONE fused implicit-GEMM MFMA kernel with
    bias (+relu) in the epilogue (csrc/kernels/conv2d.hip).
  * ``ImageToMatrix`` + FFTransposeMult + FFAggMatrix — the reference's materialised spatial
    rewriting (HIP im2col kernel, then the fused split-K block GEMM) for plan parity.
  * ``Conv2DSelect``  — conv_proj's per-image UDF, backed by the same kernel.
"""
from __future__ import annotations

import math
import time
from typing import Optional

import torch

from .. import ops
from ..computations import ScanSet, SelectionComp, WriteSet
from ..lambdas import Literal, make_batch_lambda
from ..objects.builtin import Image
from ..objects.record import RecordBatch
from . import blocks as B
from .ff import FFAggMatrix, FFTransposeMult


def flatten_kernel(weight: torch.Tensor) -> torch.Tensor:
    """[OC, C, KH, KW] -> [OC, ldk] bf16 in im2col (c, kh, kw) order, zero-padded to a multiple of 8
    (KernelToChunks/KernelBiasJoin's kernel_flat; built once per weight tensor, then reused)."""
    oc = weight.shape[0]
    return ops.derived(weight, "conv_wflat",
                       lambda w: ops.pad_k(w.reshape(oc, -1).to(torch.bfloat16)).contiguous())


_CONST_COLS = {}


def _const_col(v: int, n: int, dev) -> torch.Tensor:
    """A length-n int64 column of value v (slice of a cached device buffer: no kernel per call)."""
    key = (v, str(dev))
    buf = _CONST_COLS.get(key)
    if buf is None or buf.numel() < n:
        buf = torch.full((max(n, 1024),), v, dtype=torch.int64, device=dev)
        _CONST_COLS[key] = buf
    return buf[:n]


def images_batch(data: torch.Tensor, first_key: int = 0, keys: Optional[torch.Tensor] = None) -> RecordBatch:
    n, c, h, w = data.shape
    dev = data.device
    if keys is None:
        keys = torch.arange(first_key, first_key + n, device=dev)
    return RecordBatch({"key": keys, "channels": _const_col(c, n, dev), "height": _const_col(h, n, dev),
                        "width": _const_col(w, n, dev), "data": data}, n, Image)


class Conv2DMemFuse(SelectionComp):
    """images -> conv(images, kernel) + bias [-> relu], fused implicit GEMM per page."""

    def __init__(self, weight: torch.Tensor, bias: Optional[torch.Tensor] = None, stride: int = 1, padding: int = 0,
                 dilation: int = 1, act: str = "none", nchw_out: bool = True):
        super().__init__()
        self.kh, self.kw = weight.shape[2], weight.shape[3]
        self.wflat = flatten_kernel(weight)
        self.bias = ops.derived(bias, "bias_f32", lambda t: t.float()) if bias is not None else None
        self.stride, self.padding, self.dilation, self.act, self.nchw_out = stride, padding, dilation, act, nchw_out

    def get_selection(self, img):
        return Literal(True)

    def get_projection(self, img):
        def proj(b: RecordBatch):
            x = b.columns["data"]
            if x.dtype != torch.bfloat16:
                x = x.to(torch.bfloat16)
            w = self.wflat.to(x.device)
            bias = self.bias.to(x.device) if self.bias is not None else None
            y = ops.conv2d(x.contiguous(), w, bias, self.kh, self.kw, self.stride, self.padding, self.dilation,
                           ops.act_code(self.act), nchw_out=True)
            return images_batch(y, keys=b.columns["key"])

        return make_batch_lambda(img, proj, tag="conv2d_igemm")


class Conv2DSelect(Conv2DMemFuse):
    """conv2d_proj Conv2DSelect (per-image transformation UDF)."""

    def __init__(self, weight, bias=None, stride=1, padding=0, mode: str = "aten-conv2d"):
        super().__init__(weight, bias, stride, padding)
        self.mode = mode

    def get_projection(self, img):
        if self.mode == "aten-conv2d":
            return super().get_projection(img)

        def proj(b: RecordBatch):   # "eigen-spatial": explicit im2col + GEMM
            x = b.columns["data"].to(torch.bfloat16).contiguous()
            n, c, h, w = x.shape
            cols = ops.im2col(x, self.kh, self.kw, self.stride, self.padding, 1, self.wflat.shape[1])
            y = ops.gemm_nt(cols, self.wflat.to(x.device), self.bias.to(x.device) if self.bias is not None else None,
                            ops.BIAS_COL)
            oh = (h + 2 * self.padding - self.kh) // self.stride + 1
            ow = (w + 2 * self.padding - self.kw) // self.stride + 1
            y = y.reshape(n, oh, ow, -1).permute(0, 3, 1, 2).contiguous()
            out = images_batch(y)
            out.columns["key"] = b.columns["key"]
            return out

        return make_batch_lambda(img, proj, tag="conv2d_spatial")


class ImageToMatrix(SelectionComp):
    """ImageToChunks+ImageChunksToBlock+ImageBlockToMatrix: an image page -> im2col MatrixBlocks
    (one row-block per image, with the reference's trailing bias column of ones)."""

    def __init__(self, kh, kw, stride=1, padding=0, block_cols: int = 0):
        super().__init__()
        self.kh, self.kw, self.stride, self.padding, self.block_cols = kh, kw, stride, padding, block_cols

    def get_projection(self, img):
        from .ff import mk_blocks

        def proj(b: RecordBatch):
            x = b.columns["data"].to(torch.bfloat16).contiguous()
            n, c, h, w = x.shape
            K = c * self.kh * self.kw
            cols = ops.im2col(x, self.kh, self.kw, self.stride, self.padding, 1, (K + 1 + 7) // 8 * 8)
            cols[:, K] = 1.0                              # bias column (KernelBiasJoin's "+1")
            oh = (h + 2 * self.padding - self.kh) // self.stride + 1
            ow = (w + 2 * self.padding - self.kw) // self.stride + 1
            per = oh * ow
            data = cols.reshape(n, per, -1)
            keys = b.columns["key"]
            tr = int(keys.max().item() + 1) * per if n else 0
            return mk_blocks(keys, torch.zeros_like(keys), data, tr, cols.shape[1])

        return make_batch_lambda(img, proj, tag="im2col")


# ------------------------------------------------------------------------------- drivers
def load_images(client, db: str, name: str, n: int, c: int, h: int, w: int, seed: int = 0, page_images: int = 100,
                partition: bool = True):
    """Synthetic images (reference loads images_100_3_112_112.np)."""
    if client.storage.has_set(db, name):
        client.remove_set(db, name)
    client.create_set(db, name, Image, page_size=1 << 40)
    ws, rank = client.ctx.world_size, client.ctx.rank
    dev = client.device
    g = torch.Generator(device=dev).manual_seed(seed + rank)
    local = n if not partition else n
    key0 = rank * local
    for s in range(0, local, page_images):
        m = min(page_images, local - s)
        x = torch.empty(m, c, h, w, device=dev, dtype=torch.float32).uniform_(-1, 1, generator=g).to(torch.bfloat16)
        client.storage.get_set(db, name).add_batch(images_batch(x, key0 + s))
    return client.storage.get_set(db, name)


def random_kernel(oc, c, kh, kw, seed=0, device="cpu"):
    g = torch.Generator(device=device).manual_seed(seed)
    w = torch.empty(oc, c, kh, kw, device=device).uniform_(-1, 1, generator=g) * (1.0 / math.sqrt(c * kh * kw))
    b = torch.empty(oc, device=device).uniform_(-0.1, 0.1, generator=g)
    return w, b


def conv2d_memfuse_inference(client, db: str, images: str, output: str, weight, bias, stride=1, padding=0,
                             act: str = "none") -> dict:
    """PipelinedConv2dMemFuseTest with the fused plan (kernel 'materialised' once)."""
    if client.storage.has_set(db, output):
        client.clear_set(db, output)
    else:
        client.create_set(db, output, Image, page_size=1 << 40)
    t0 = time.perf_counter()
    sel = Conv2DMemFuse(weight, bias, stride, padding, act=act).set_input(ScanSet(db, images, Image))
    st = client.execute_computations(WriteSet(db, output, Image).set_input(sel), job_name="conv2d")
    return {"seconds": time.perf_counter() - t0, "job": st}


def conv2d_spatial_inference(client, db: str, images: str, output: str, weight, bias, stride=1, padding=0,
                             block_x: int = 32, block_y: int = 32) -> dict:
    """The reference's materialised plan: image_flat (im2col blocks) x kernel_flat^T via the
    block-matmul join + aggregate (fused onto one split-K MFMA GEMM when sets are dense)."""
    oc = weight.shape[0]
    K = weight[0].numel()
    kflat = torch.cat([weight.reshape(oc, K).float(), bias.reshape(oc, 1).float()], 1)
    B.load_tensor(client, db, "kernel_flat", kflat.to(client.device), block_x, block_y)
    if client.storage.has_set(db, "image_flat"):
        client.remove_set(db, "image_flat")
    client.create_set(db, "image_flat", None)
    t0 = time.perf_counter()
    i2m = ImageToMatrix(weight.shape[2], weight.shape[3], stride, padding).set_input(ScanSet(db, images, Image))
    client.execute_computations(WriteSet(db, "image_flat").set_input(i2m), job_name="image_ops")
    # assemble image_flat into a dense matrix set (ImageBlockToMatrix output)
    blocks = client.get_set_batches(db, "image_flat")
    rb = RecordBatch.concat(blocks)
    mat = rb.columns["data"].reshape(-1, rb.columns["data"].shape[-1])[:, : K + 1]
    B.load_tensor(client, db, "image_flat_m", mat, block_x, block_y)
    if client.storage.has_set(db, output):
        client.remove_set(db, output)
    client.create_set(db, output, None, dense=True)
    j = FFTransposeMult()
    j.set_input(0, ScanSet(db, "image_flat_m"))
    j.set_input(1, ScanSet(db, "kernel_flat"))
    agg = FFAggMatrix().set_input(j)
    st = client.execute_computations(WriteSet(db, output).set_input(agg), job_name="conv2d")
    return {"seconds": time.perf_counter() - t0, "job": st}


__all__ = ["Conv2DMemFuse", "Conv2DSelect", "ImageToMatrix", "flatten_kernel", "images_batch", "load_images",
           "random_kernel", "conv2d_memfuse_inference", "conv2d_spatial_inference"]
