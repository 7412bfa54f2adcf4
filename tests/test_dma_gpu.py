"""The all-DMA split implicit GEMM (ig_kernel_x3d: 256 x 192 tiles, eight waves, one block per
CU, activations and the three weight planes staged by LDS-DMA into two stages, A split into three
bf16 terms after its fragment reads) against fp64 torch on the GPU at the fp32 bar, at geometries
that take it (>= 256 tiles of 256 rows): stride-2 convolutions on 64- and 32-wide grids, a ragged
row count, transposed convolutions (four stride-1 phases of 9/6/6/4 taps), their input gradients
and a bias / ReLU epilogue.  Each case checks the plan (the DMA kernel ran) and holds the error
within 1.5x of the native fp32 kernel's own.  GPU only."""
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


def _r(*shape, seed, scale=1.0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(*shape, device=DEV, generator=g) * scale


def _plan(op, a, b, k, s, p):
    from image_compression_amd import _lib
    q = _lib.plan(op, a, b, k, s, p, 2)
    return q["kernel"], q["bm"], q["ksplit"]


def _check(got, native, ref, name):
    got, native, ref = got.double().cpu(), native.double().cpu(), ref.cpu()
    assert_close(got, ref, 1e-4, name)
    es, en = rel_err(got, ref), rel_err(native, ref)
    print(f"{name}: DMA split {es:.2e} native fp32 {en:.2e}")
    assert es <= 1.5 * en + 1e-8, (name, es, en)


# (n, input size, relu): 32 x 64^2 and 128 x 32^2 outputs (512 tiles of 256 rows); 18 x 61^2
# (ragged: 261 full tiles and a partial one)
@pytest.mark.parametrize("n,h,relu", [(32, 128, False), (128, 64, True), (18, 122, False)])
def test_dma_conv_fwd_dgrad(n, h, relu):
    from image_compression_amd import _lib, functional as IF
    ops = _lib.ops()
    x = _r(n, 192, h, h, seed=1).contiguous(memory_format=CL)
    w = _r(192, 192, 5, 5, seed=2, scale=0.03)
    b = _r(192, seed=3, scale=0.1)
    ho = (h + 4 - 5) // 2 + 1
    y = torch.empty(n, 192, ho, ho, device=DEV).contiguous(memory_format=CL)
    assert _plan("conv2d_fwd", x, y, 5, 2, 2) == ("ig_split_dma", 256, 1)
    with torch.no_grad():
        ys = IF.conv2d(x, w, b, 2, 2, act=int(relu), math=2)
        yn = IF.conv2d(x, w, b, 2, 2, act=int(relu), math=0)
        yr = F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=2)
        if relu:
            yr = yr.relu()
    _check(ys, yn, yr, "y")
    del ys, yn, yr
    gy = _r(n, 192, ho, ho, seed=4).contiguous(memory_format=CL)
    assert _plan("conv2d_dgrad", gy, x, 5, 2, 2) == ("ig_split_dma", 256, 1)
    dxs = ops.conv2d_dgrad(gy, w, x, 2, 2, 2)
    dxn = ops.conv2d_dgrad(gy, w, x, 2, 2, 0)
    dxr = torch.nn.grad.conv2d_input(x.shape, w.double(), gy.double(), stride=2, padding=2)
    _check(dxs, dxn, dxr, "dx")


def test_dma_tconv_fwd_dgrad():
    from image_compression_amd import _lib
    ops = _lib.ops()
    n, h = 8, 64
    x = _r(n, 192, h, h, seed=5).contiguous(memory_format=CL)
    w = _r(192, 192, 5, 5, seed=6, scale=0.03)
    y = torch.empty(n, 192, 2 * h, 2 * h, device=DEV).contiguous(memory_format=CL)
    assert _plan("conv_transpose2d_fwd", x, y, 5, 2, 2) == ("ig_split_dma", 256, 1)
    ys = ops.conv_transpose2d_fwd(x, w, None, 2, 2, 1, 0, 2)
    yn = ops.conv_transpose2d_fwd(x, w, None, 2, 2, 1, 0, 0)
    yr = F.conv_transpose2d(x.double(), w.double(), None, stride=2, padding=2, output_padding=1)
    _check(ys, yn, yr, "y")
    del ys, yn, yr
    n = 16  # the input gradient is a stride-2 conv onto 64^2: 256 tiles of 256 rows from 16 images
    x = _r(n, 192, h, h, seed=5).contiguous(memory_format=CL)
    gy = _r(n, 192, 2 * h, 2 * h, seed=7).contiguous(memory_format=CL)
    assert _plan("conv_transpose2d_dgrad", gy, x, 5, 2, 2) == ("ig_split_dma", 256, 1)
    dxs = ops.conv_transpose2d_dgrad(gy, w, x, 2, 2, 2)
    dxn = ops.conv_transpose2d_dgrad(gy, w, x, 2, 2, 0)
    dxr = F.conv2d(gy.double(), w.double(), None, stride=2, padding=2)
    _check(dxs, dxn, dxr, "dx")


# K split across blocks (fewer than 256 tiles of 256 rows, one-phase convs): 8 x 32^2 -> ksplit 8,
# 8 x 64^2 -> 2, 13 x 25^2 (ragged, 32 tiles) -> 8; the partial sums reduced in fixed order
@pytest.mark.parametrize("n,h,ksplit", [(8, 64, 8), (8, 128, 2), (13, 50, 8)])
def test_dma_split_k(n, h, ksplit):
    from image_compression_amd import _lib, functional as IF
    ops = _lib.ops()
    x = _r(n, 192, h, h, seed=21).contiguous(memory_format=CL)
    w = _r(192, 192, 5, 5, seed=22, scale=0.03)
    b = _r(192, seed=23, scale=0.1)
    ho = (h + 4 - 5) // 2 + 1
    y = torch.empty(n, 192, ho, ho, device=DEV).contiguous(memory_format=CL)
    assert _plan("conv2d_fwd", x, y, 5, 2, 2) == ("ig_split_dma", 256, ksplit)
    with torch.no_grad():
        ys = IF.conv2d(x, w, b, 2, 2, math=2)
        yn = IF.conv2d(x, w, b, 2, 2, math=0)
        yr = F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=2)
    _check(ys, yn, yr, "y")
    # deterministic: the same launch twice is bitwise equal
    with torch.no_grad():
        assert torch.equal(ys, IF.conv2d(x, w, b, 2, 2, math=2))
    # a 3x3 stride-1 conv (h_a.0's shape class)
    x1 = _r(n, 192, ho, ho, seed=24).contiguous(memory_format=CL)
    y1 = torch.empty(n, 192, ho, ho, device=DEV).contiguous(memory_format=CL)
    if _plan("conv2d_fwd", x1, y1, 3, 1, 1)[0] == "ig_split_dma":
        with torch.no_grad():
            _check(IF.conv2d(x1, w[:, :, :3, :3].contiguous(), b, 1, 1, math=2),
                   IF.conv2d(x1, w[:, :, :3, :3].contiguous(), b, 1, 1, math=0),
                   F.conv2d(x1.double(), w[:, :, :3, :3].double(), b.double(), stride=1, padding=1), "y3x3")
