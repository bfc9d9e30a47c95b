"""NatureCNN convolutions as hand-written f32 MFMA implicit GEMMs (csrc/conv.hip) against a float64
PyTorch convolution of the same inputs (reference layer: rl_algo_impls/shared/encoder/nature_cnn.py:31-41,
Conv2d -> ReLU).  f32 products with the kernel's own summation order: the tolerance below is a few
f32 ulps of the sum of |products| (K up to 576 terms)."""
import ctypes as C

import pytest
import torch
import torch.nn.functional as F

from rl_algo_impls_amd import _lib

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)

# (Ci, H, Co, k, stride, flatten): the three NatureCNN layers, plus ragged / odd shapes
CASES = [
    (4, 84, 32, 8, 4, False),
    (32, 20, 64, 4, 2, False),
    (64, 9, 64, 3, 1, True),
    (64, 9, 64, 3, 1, False),
    (8, 13, 16, 2, 1, False),
    (32, 11, 48, 3, 2, True),
]


def _inputs(B, Ci, H, Co, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(B, Ci, H, H, generator=g)
    w = torch.randn(Co, Ci, k, k, generator=g) * (2.0 / (Ci * k * k)) ** 0.5
    b = torch.randn(Co, generator=g) * 0.1
    return x, w, b


def _run(x, w, b, stride, flatten, variant=0):
    B, Ci, H, W = x.shape
    Co, _, KH, KW = w.shape
    OH, OW = (H - KH) // stride + 1, (W - KW) // stride + 1
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV).contiguous(memory_format=torch.channels_last)
    bd = b.to(DEV)
    y = torch.full((B, Co * OH * OW), float("nan"), device=DEV)
    rc = _lib.lib().rai_conv2d_bias_relu_fwd_v(xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), B, H, W, Ci, Co, KH, KW,
                                               stride, 1 if flatten else 0, y.data_ptr(), variant,
                                               _lib.stream_handle(DEV))
    _lib.check(rc, "rai_conv2d_bias_relu_fwd")
    torch.cuda.synchronize()
    return y.cpu()


def _reference(x, w, b, stride, flatten):
    xd, wd = x.double(), w.double()
    y = torch.relu(F.conv2d(xd, wd, b.double(), stride))
    bound = F.conv2d(xd.abs(), wd.abs(), b.double().abs(), stride)  # sum of |terms| per output
    if flatten:
        return torch.flatten(y, 1), torch.flatten(bound, 1)
    return y.permute(0, 2, 3, 1).reshape(x.shape[0], -1), bound.permute(0, 2, 3, 1).reshape(x.shape[0], -1)


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(str(v) for v in c[:5]) + ("-flat" if c[5] else ""))
@pytest.mark.parametrize("B", [1, 7, 64])
def test_conv_bias_relu_fwd_matches_fp64(case, B):
    Ci, H, Co, k, s, flat = case
    x, w, b = _inputs(B, Ci, H, Co, k, seed=B)
    y = _run(x, w, b, s, flat)
    ref, bound = _reference(x, w, b, s, flat)
    assert torch.isfinite(y).all()
    err = (y.double() - ref).abs()
    # the worst-case bound of ANY f32 summation order of K = Ci*k*k products plus the bias:
    # gamma_(K+2) * sum|terms| (an indexing error is O(1) relative, far outside it)
    tol = (Ci * k * k + 2) * 2.0 ** -24 * bound + 1e-30
    assert (err <= tol).all(), float((err / tol).max())


@pytest.mark.parametrize("case,B", [((32, 20, 64, 4, 2, False), 256), ((64, 9, 64, 3, 1, True), 256),
                                    ((64, 9, 64, 3, 1, False), 200), ((64, 9, 64, 3, 1, True), 37)])
def test_conv_fwd_splitk_matches_fp64_and_one_pass(case, B, monkeypatch):
    """The split-K forward (rai_conv2d_bias_relu_fwd_splitk, opt-in: conv2 / conv3 of NatureCNN at the
    update's B = 256, where the one-pass tiling leaves CUs idle): two halves of the reduction as separate
    workgroups, raw partial sums, an ordered second pass with the bias and the ReLU (NHWC and the
    flattened NCHW order).  Within the worst-case f32 summation bound of the fp64 convolution, close to
    the one-pass kernel, and deterministic."""
    Ci, H, Co, k, s, flat = case
    monkeypatch.setenv("RAI_CONV_FWD_SPLITK", "1")  # opt-in (measured slower than the one-pass form)
    L = _lib.lib()
    nb = int(L.rai_conv2d_fwd_splitk_bytes(B, H, H, Ci, Co, k, k, s, 1 if flat else 0))
    assert nb > 0, "the shape takes the split"
    x, w, b = _inputs(B, Ci, H, Co, k, seed=B + 3)
    OH = (H - k) // s + 1
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV).contiguous(memory_format=torch.channels_last)
    bd = b.to(DEV)
    outs = []
    for _ in range(2):
        y = torch.full((B, Co * OH * OH), float("nan"), device=DEV)
        part = torch.full((nb // 4,), float("nan"), device=DEV)
        _lib.check(L.rai_conv2d_bias_relu_fwd_splitk(xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), B, H, H, Ci, Co, k, k,
                                                     s, 1 if flat else 0, y.data_ptr(), part.data_ptr(), nb,
                                                     _lib.stream_handle(DEV)), "rai_conv2d_bias_relu_fwd_splitk")
        torch.cuda.synchronize()
        outs.append(y.cpu())
    assert torch.equal(outs[0], outs[1])
    ref, bound = _reference(x, w, b, s, flat)
    err = (outs[0].double() - ref).abs()
    tol = (Ci * k * k + 2) * 2.0 ** -24 * bound + 1e-30
    assert (err <= tol).all(), float((err / tol).max())
    one = _run(x, w, b, s, flat)
    torch.testing.assert_close(outs[0], one, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("variant", list(range(1, 21)))
def test_conv_every_blocking_variant(variant):
    Ci, H, Co, k, s, flat = 32, 20, 64, 4, 2, False
    x, w, b = _inputs(9, Ci, H, Co, k, seed=3)
    ref, bound = _reference(x, w, b, s, flat)
    y = _run(x, w, b, s, flat, variant)
    assert ((y.double() - ref).abs() <= (32 * 16 + 2) * 2.0 ** -24 * bound + 1e-30).all()


def test_conv_relu_keeps_nan_and_zeroes_negatives():
    x, w, b = _inputs(2, 4, 84, 32, 8)
    x[0, 0, 0, 0] = float("nan")  # poisons the first output pixel of sample 0 only
    b[:] = -1e6  # every finite output negative -> 0
    y = _run(x, w, b, 4, False)
    assert torch.isnan(y[0, :32]).all()
    assert (y[0, 32:] == 0).all() and (y[1] == 0).all()


def test_conv_rejects_unsupported_shapes():
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    # Ci % 4, Co % 16, K % 32
    assert L.rai_conv2d_bias_relu_fwd(None, None, None, 1, 8, 8, 3, 16, 2, 2, 1, 0, None, st) == -2
    assert L.rai_conv2d_bias_relu_fwd(None, None, None, 1, 8, 8, 4, 24, 2, 2, 1, 0, None, st) == -2
    assert L.rai_conv2d_bias_relu_fwd(None, None, None, 1, 8, 8, 4, 16, 3, 3, 1, 0, None, st) == -2
    assert L.rai_conv2d_bias_relu_fwd(None, None, None, 0, 8, 8, 8, 16, 2, 2, 1, 0, None, st) == 0
    assert L.rai_conv2d_bias_relu_fwd(None, None, None, 1, 8, 8, 8, 16, 2, 2, 1, 0, None, st) == -1


def _wgrad(x, dz, KH, KW, stride, dw0=None, pf=0):
    """rai_conv2d_wgrad: x (B, Ci, H, W), dz (B, Co, OH, OW) NCHW tensors on the CPU; returns dw in
    (Co, Ci, KH, KW) NCHW order.  dw0: accumulate onto it."""
    B, Ci, H, W = x.shape
    Co = dz.shape[1]
    L = _lib.lib()
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    dzd = dz.to(DEV).contiguous(memory_format=torch.channels_last)
    dw = (dw0 if dw0 is not None else torch.full((Co, Ci, KH, KW), float("nan"))).to(DEV)
    dw = dw.contiguous(memory_format=torch.channels_last)
    nb = int(L.rai_conv2d_wgrad_workspace_bytes(B, H, W, Ci, Co, KH, KW, stride))
    ws = torch.full((max(nb, 16) // 4,), float("nan"), device=DEV)  # needs no zeroing
    rc = L.rai_conv2d_wgrad_v(xd.data_ptr(), dzd.data_ptr(), B, H, W, Ci, Co, KH, KW, stride, dw.data_ptr(),
                              0 if dw0 is None else 1, ws.data_ptr(), nb, 0, pf, _lib.stream_handle(DEV))
    _lib.check(rc, "rai_conv2d_wgrad")
    torch.cuda.synchronize()
    return dw.cpu()


WGRAD_CASES = [  # (Ci, H, Co, k, stride): the three NatureCNN layers + a ragged small one
    (4, 84, 32, 8, 4),
    (32, 20, 64, 4, 2),
    (64, 9, 64, 3, 1),
    (16, 7, 32, 2, 1),
]


@pytest.mark.parametrize("case", WGRAD_CASES, ids=lambda c: "x".join(str(v) for v in c))
@pytest.mark.parametrize("B", [1, 5, 256])
@pytest.mark.parametrize("pf", [0, 104, 108], ids=["default", "buf4", "buf8"])
def test_conv_wgrad_matches_fp64(case, B, pf):
    Ci, H, Co, k, s = case
    if B == 256 and Ci == 4:
        B = 64  # conv1 at 64 samples keeps the fp64 CPU reference fast; 256 runs below at 16
    x, w, _ = _inputs(B, Ci, H, Co, k, seed=B + 11)
    OH = (H - k) // s + 1
    g = torch.Generator().manual_seed(B)
    dz = torch.randn(B, Co, OH, OH, generator=g) * (torch.rand(B, Co, OH, OH, generator=g) > 0.4)
    dw = _wgrad(x, dz, k, k, s, pf=pf)
    xd, dzd = x.double(), dz.double()
    ref = torch.ops.aten.convolution_backward(dzd, xd, w.double(), None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1]
    bound = torch.ops.aten.convolution_backward(dzd.abs(), xd.abs(), w.double(), None, [s, s], [0, 0], [1, 1], False,
                                                [0, 0], 1, [False, True, False])[1]
    M = B * OH * OH
    tol = (M + 2) * 2.0 ** -24 * bound + 1e-30
    assert torch.isfinite(dw).all()
    assert ((dw.double() - ref).abs() <= tol).all(), float(((dw.double() - ref).abs() / tol).max())


def test_conv_wgrad_accumulates_and_is_deterministic():
    Ci, H, Co, k, s = 32, 20, 64, 4, 2
    x, w, _ = _inputs(48, Ci, H, Co, k, seed=5)
    dz = torch.randn(48, Co, 9, 9, generator=torch.Generator().manual_seed(2))
    base = torch.randn(Co, Ci, k, k, generator=torch.Generator().manual_seed(3))
    a = _wgrad(x, dz, k, k, s)
    b = _wgrad(x, dz, k, k, s)
    assert torch.equal(a, b)
    acc = _wgrad(x, dz, k, k, s, dw0=base)
    assert torch.equal(acc, base + a)  # one f32 add per element, after the fixed-order sum


def test_conv_wgrad_full_c3_minibatch_against_miopen():
    """conv1 at the C3 minibatch (B = 256, 102,400 pixels): against MIOpen's f32 weight gradient on the
    same device (both f32 sums of 102,400 terms; the bound is the f32 worst case of their difference)."""
    Ci, H, Co, k, s = 4, 84, 32, 8, 4
    x, w, _ = _inputs(256, Ci, H, Co, k, seed=9)
    dz = torch.randn(256, Co, 20, 20, generator=torch.Generator().manual_seed(4)) * 0.01
    dw = _wgrad(x, dz, k, k, s)
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    dzd = dz.to(DEV).contiguous(memory_format=torch.channels_last)
    ref = torch.ops.aten.convolution_backward(dzd, xd, w.to(DEV).contiguous(memory_format=torch.channels_last), None,
                                              [s, s], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])[1]
    bound = torch.ops.aten.convolution_backward(dzd.abs(), xd, w.to(DEV), None, [s, s], [0, 0], [1, 1], False,
                                                [0, 0], 1, [False, True, False])[1]
    err = (dw.to(DEV) - ref).abs()
    assert (err <= 2 * (256 * 400 + 2) * 2.0 ** -24 * bound + 1e-30).all()
    assert (err <= 1e-4 * bound.max()).all()  # and far tighter in practice


def test_conv_wgrad_partials_and_one_reduce_for_three_layers():
    """The backward's form: each layer's partials, then ONE rai_conv2d_wgrad_reduce over the three
    NatureCNN layers, accumulating into existing gradients -- bit-identical to rai_conv2d_wgrad per
    layer (same plan, same fixed-order sums)."""
    from rl_algo_impls_amd.cnn_ops import _WgradJob
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    jobs, keep, outs, refs = [], [], [], []
    for li, (Ci, H, Co, k, s) in enumerate(WGRAD_CASES[:3]):
        x, w, _ = _inputs(32, Ci, H, Co, k, seed=20 + li)
        OH = (H - k) // s + 1
        dz = torch.randn(32, Co, OH, OH, generator=torch.Generator().manual_seed(li))
        base = torch.randn(Co, Ci, k, k, generator=torch.Generator().manual_seed(40 + li))
        refs.append(_wgrad(x, dz, k, k, s, dw0=base))
        xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
        dzd = dz.to(DEV).contiguous(memory_format=torch.channels_last)
        g = base.to(DEV).contiguous(memory_format=torch.channels_last)
        nb = int(L.rai_conv2d_wgrad_workspace_bytes(32, H, H, Ci, Co, k, k, s))
        ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
        _lib.check(L.rai_conv2d_wgrad_partials(xd.data_ptr(), dzd.data_ptr(), 32, H, H, Ci, Co, k, k, s,
                                               ws.data_ptr(), nb, st), "partials")
        jobs.append(_WgradJob(ws.data_ptr(), g.data_ptr(), None, 32, H, H, Ci, Co, k, k, s, 0))
        keep += [xd, dzd, ws]
        outs.append(g)
    arr = (_WgradJob * 3)(*jobs)
    _lib.check(L.rai_conv2d_wgrad_reduce(C.cast(arr, C.c_void_p), 3, 1, st), "reduce")
    torch.cuda.synchronize()
    for g, ref in zip(outs, refs):
        assert torch.equal(g.cpu(), ref)
    assert L.rai_conv2d_wgrad_reduce(C.cast(arr, C.c_void_p), 5, 1, st) == -2


DGRAD_CASES = [  # (Ci, H, Co, k, stride): NatureCNN conv2 / conv3, odd sizes, a border-only tap case
    (32, 20, 64, 4, 2),
    (64, 9, 64, 3, 1),
    (32, 11, 16, 2, 2),
    (64, 7, 32, 4, 2),
]


@pytest.mark.parametrize("case", DGRAD_CASES, ids=lambda c: "x".join(str(v) for v in c))
@pytest.mark.parametrize("B", [1, 3, 64])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6, 7])
def test_conv_dgrad_matches_fp64(case, B, variant):
    """rai_conv2d_dgrad_v against fp64 autograd.  Variants: 0 = the shipped choice (the per-image
    GEMM + col2im form for NatureCNN conv2 / conv3, else the pixel-class form), 1 / 2 = the pixel-class
    form with LDS-resident weights, 3 = the per-image form only, 4 = the per-image form with the weight
    operand staged through LDS, 5 / 6 / 7 = the per-image form with buffer loads and 2 / 3 / 4 quads in
    flight (3-7: RAI_E_UNSUPPORTED on shapes they have no instantiation for)."""
    Ci, H, Co, k, s = case
    x, w, _ = _inputs(B, Ci, H, Co, k, seed=B + 31)
    OH = (H - k) // s + 1
    dz = torch.randn(B, Co, OH, OH, generator=torch.Generator().manual_seed(B + 7))
    dzd = dz.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV).contiguous(memory_format=torch.channels_last)
    dx = torch.full((B, Ci, H, H), float("nan"), device=DEV).contiguous(memory_format=torch.channels_last)
    rc = _lib.lib().rai_conv2d_dgrad_v(dzd.data_ptr(), wd.data_ptr(), B, H, H, Ci, Co, k, k, s, dx.data_ptr(),
                                       variant, _lib.stream_handle(DEV))
    if variant >= 3 and (Ci, H, Co, k, s) not in ((32, 20, 64, 4, 2), (64, 9, 64, 3, 1)):
        assert rc == -6  # RAI_E_UNSUPPORTED
        return
    _lib.check(rc, "rai_conv2d_dgrad")
    torch.cuda.synchronize()
    ref = torch.ops.aten.convolution_backward(dz.double(), x.double(), w.double(), None, [s, s], [0, 0], [1, 1], False,
                                              [0, 0], 1, [True, False, False])[0]
    bound = torch.ops.aten.convolution_backward(dz.double().abs(), x.double(), w.double().abs(), None, [s, s], [0, 0],
                                                [1, 1], False, [0, 0], 1, [True, False, False])[0]
    got = dx.cpu().double()
    assert torch.isfinite(got).all()
    tol = (Co * k * k + 2) * 2.0 ** -24 * bound + 1e-30
    assert ((got - ref).abs() <= tol).all(), float(((got - ref).abs() / tol).max())


@pytest.mark.parametrize("case", [(4, 84, 32, 8, 4), (32, 20, 64, 4, 2)], ids=["conv1", "conv2"])
def test_conv_wgrad_relu_partials_fold_the_relu_backward_and_bias_gradient(case):
    """rai_conv2d_wgrad_relu_partials + the reduce: dW and db of dz = (y > 0 ? dy : 0) from dy and the
    saved output y, accumulated into existing gradients -- against fp64 (bound as above) and, for dW,
    bit-identical to rai_conv2d_wgrad on the materialized dz."""
    from rl_algo_impls_amd.cnn_ops import _WgradJob
    Ci, H, Co, k, s = case
    B = 24
    x, w, _ = _inputs(B, Ci, H, Co, k, seed=77)
    OH = (H - k) // s + 1
    gen = torch.Generator().manual_seed(5)
    dy = torch.randn(B, Co, OH, OH, generator=gen)
    y = torch.relu(torch.randn(B, Co, OH, OH, generator=gen))  # zeros where the ReLU clipped
    dz = torch.where(y > 0, dy, torch.zeros_like(dy))
    w0 = torch.randn(Co, Ci, k, k, generator=gen)
    b0 = torch.randn(Co, generator=gen)
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    cl = lambda t: t.to(DEV).contiguous(memory_format=torch.channels_last)
    xd, dyd, yd, gw = cl(x), cl(dy), cl(y), cl(w0)
    gb = b0.to(DEV).clone()
    nb = int(L.rai_conv2d_wgrad_workspace_bytes(B, H, H, Ci, Co, k, k, s))
    ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
    _lib.check(L.rai_conv2d_wgrad_relu_partials(dyd.data_ptr(), yd.data_ptr(), xd.data_ptr(), B, H, H, Ci, Co, k, k,
                                                s, ws.data_ptr(), nb, st), "relu_partials")
    job = (_WgradJob * 1)(_WgradJob(ws.data_ptr(), gw.data_ptr(), gb.data_ptr(), B, H, H, Ci, Co, k, k, s, 0))
    _lib.check(L.rai_conv2d_wgrad_reduce(C.cast(job, C.c_void_p), 1, 1, st), "reduce")
    torch.cuda.synchronize()
    assert torch.equal(gw.cpu(), _wgrad(x, dz, k, k, s, dw0=w0))
    db_ref = b0.double() + dz.double().sum(dim=(0, 2, 3))
    bound = b0.double().abs() + dz.double().abs().sum(dim=(0, 2, 3))
    assert ((gb.cpu().double() - db_ref).abs() <= (B * OH * OH + 2) * 2.0 ** -24 * bound).all()


def test_same_conv_twice_in_one_backward_accumulates_both_uses():
    """One conv module applied to two same-shape inputs inside one direct_grads() backward:
    both uses write their weight-gradient partials into the layer's one workspace, so the first use's
    pending reduction must run before the second overwrites it.  One input needs its gradient (partials
    from dz), the other does not (the ReLU backward folded into the partials).  dW, db and dx against
    fp64 autograd of the same graph."""
    from rl_algo_impls_amd import cnn_ops

    torch.manual_seed(3)
    conv = torch.nn.Conv2d(32, 32, 4, stride=2)
    w64, b64 = conv.weight.detach().double(), conv.bias.detach().double()
    x1 = torch.randn(8, 32, 14, 14)
    x2 = torch.randn(8, 32, 14, 14)
    gy = torch.randn(8, 32, 6, 6)
    r1 = x1.double().requires_grad_(True)
    w_r, b_r = w64.clone().requires_grad_(True), b64.clone().requires_grad_(True)
    out = torch.relu(F.conv2d(r1, w_r, b_r, 2)) + torch.relu(F.conv2d(x2.double(), w_r, b_r, 2))
    (out * gy.double()).sum().backward()

    w = conv.weight.detach().to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    b = conv.bias.detach().to(DEV).clone().requires_grad_(True)
    w.grad = torch.zeros_like(w, memory_format=torch.channels_last)
    b.grad = torch.zeros_like(b)
    d1 = x1.to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    d2 = x2.to(DEV).contiguous(memory_format=torch.channels_last)
    with cnn_ops.direct_grads():
        y = cnn_ops.ConvBiasReLU.apply(d1, w, b, 2, 0, conv) + cnn_ops.ConvBiasReLU.apply(d2, w, b, 2, 0, conv)
        (y * gy.to(DEV).contiguous(memory_format=torch.channels_last)).sum().backward()
    torch.cuda.synchronize()
    for got, ref in [(w.grad, w_r.grad), (b.grad, b_r.grad), (d1.grad, r1.grad)]:
        got = got.detach().cpu().double()
        assert torch.isfinite(got).all()
        assert ((got - ref).abs() <= 1e-4 * ref.abs().max() + 1e-6).all(), float((got - ref).abs().max())


@pytest.mark.parametrize("case", [(32, 20, 64, 4, 2), (64, 9, 64, 3, 1)], ids=["conv2", "conv3"])
@pytest.mark.parametrize("B", [3, 256])
def test_conv_dgrad_relu_folds_the_relu_backward(case, B):
    """rai_conv2d_dgrad_relu: the input gradient of dz = (y > 0 ? dy : 0) formed on the fly from dy and the
    saved output y -- against fp64 autograd on the materialised dz (bound as test_conv_dgrad_matches_fp64),
    and bit-identical to rai_conv2d_dgrad on that dz (the same kernel, same summation order).  A shape the
    per-image form has no instantiation for returns RAI_E_UNSUPPORTED."""
    Ci, H, Co, k, s = case
    x, w, _ = _inputs(B, Ci, H, Co, k, seed=B + 3)
    OH = (H - k) // s + 1
    gen = torch.Generator().manual_seed(B + 9)
    dy = torch.randn(B, Co, OH, OH, generator=gen)
    y = torch.relu(torch.randn(B, Co, OH, OH, generator=gen))
    dz = torch.where(y > 0, dy, torch.zeros_like(dy))
    cl = lambda t: t.to(DEV).contiguous(memory_format=torch.channels_last)
    dyd, yd, dzd, wd = cl(dy), cl(y), cl(dz), cl(w)
    dx = torch.full((B, Ci, H, H), float("nan"), device=DEV).contiguous(memory_format=torch.channels_last)
    dx2 = torch.full_like(dx, float("nan"))
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    _lib.check(L.rai_conv2d_dgrad_relu(dyd.data_ptr(), yd.data_ptr(), wd.data_ptr(), B, H, H, Ci, Co, k, k, s,
                                       dx.data_ptr(), st), "rai_conv2d_dgrad_relu")
    _lib.check(L.rai_conv2d_dgrad(dzd.data_ptr(), wd.data_ptr(), B, H, H, Ci, Co, k, k, s, dx2.data_ptr(), st),
               "rai_conv2d_dgrad")
    torch.cuda.synchronize()
    assert torch.equal(dx.cpu(), dx2.cpu())
    ref = torch.ops.aten.convolution_backward(dz.double(), x.double(), w.double(), None, [s, s], [0, 0], [1, 1],
                                              False, [0, 0], 1, [True, False, False])[0]
    bound = torch.ops.aten.convolution_backward(dz.double().abs(), x.double(), w.double().abs(), None, [s, s],
                                                [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])[0]
    got = dx.cpu().double()
    tol = (Co * k * k + 2) * 2.0 ** -24 * bound + 1e-30
    assert ((got - ref).abs() <= tol).all()


def test_conv_dgrad_relu_rejects_shapes_without_an_instantiation():
    """Argument checks only (nothing is launched): a shape the per-image form is not instantiated for
    returns RAI_E_UNSUPPORTED, null pointers RAI_E_NULLPTR, B = 0 is a no-op."""
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    buf = torch.zeros(64, device=DEV)
    p = buf.data_ptr()
    assert L.rai_conv2d_dgrad_relu(p, p, p, 2, 11, 11, 32, 16, 2, 2, 2, p, st) == -6
    assert L.rai_conv2d_dgrad_relu(None, p, p, 2, 20, 20, 32, 64, 4, 4, 2, p, st) == -1
    assert L.rai_conv2d_dgrad_relu(None, None, None, 0, 20, 20, 32, 64, 4, 4, 2, None, st) == 0


def _u8_frames(B, H, seed):
    g = torch.Generator().manual_seed(seed)
    u = torch.randint(0, 256, (B, 4, H, H), generator=g, dtype=torch.uint8)
    u[0, :, :3] = 255  # the table's ends
    u[-1, :, -3:] = 0
    return u


U8_QUOTIENTS = [("fma", 255.0), ("table", 255.0), ("fma", 7.0)]


@pytest.mark.parametrize("quot,divisor", U8_QUOTIENTS)
@pytest.mark.parametrize("B", [1, 7, 256, 1024])
def test_conv1_uint8_forward_is_the_float32_forward_of_the_prescaled_frames(B, quot, divisor, monkeypatch):
    """rai_conv2d_bias_relu_fwd_u8 on uint8 NHWC frames (conv1 of NatureCNN, x = u8 / 255 formed in the
    kernel) is bit-identical to rai_conv2d_bias_relu_fwd on the float32 frames u8 / 255 (IEEE division, as
    the gather's prescale writes them): same blocking and summation order, only the operand load differs.
    Both in-kernel quotients: the multiply + fma correction (default where the host has checked it exact
    for the divisor) and the LDS table (RAI_CONV_U8_LUT=1)."""
    if quot == "table":
        monkeypatch.setenv("RAI_CONV_U8_LUT", "1")
    u = _u8_frames(B, 84, seed=B)
    _, w, b = _inputs(1, 4, 84, 32, 8, seed=3)
    div = torch.tensor(divisor)
    xf = (u.float() / div).to(DEV).contiguous(memory_format=torch.channels_last)
    ud = u.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV).contiguous(memory_format=torch.channels_last)
    bd = b.to(DEV)
    OH = 20
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    y32 = torch.full((B, 32, OH, OH), float("nan"), device=DEV).contiguous(memory_format=torch.channels_last)
    y8 = torch.full_like(y32, float("nan"))
    _lib.check(L.rai_conv2d_bias_relu_fwd(xf.data_ptr(), wd.data_ptr(), bd.data_ptr(), B, 84, 84, 4, 32, 8, 8, 4, 0,
                                          y32.data_ptr(), st), "fwd f32")
    _lib.check(L.rai_conv2d_bias_relu_fwd_u8(ud.data_ptr(), divisor, wd.data_ptr(), bd.data_ptr(), B, 84, 84, 4, 32,
                                             8, 8, 4, 0, y8.data_ptr(), st), "fwd u8")
    torch.cuda.synchronize()
    assert torch.equal(y8.cpu(), y32.cpu())
    if B <= 7:  # and against fp64 (bound as test_conv_bias_relu_fwd_matches_fp64)
        ref, bound = _reference(u.float() / div, w, b, 4, False)
        got = y8.cpu().permute(0, 2, 3, 1).reshape(B, -1).double()
        assert ((got - ref).abs() <= 256 * 2.0 ** -24 * bound + 1e-30).all()


@pytest.mark.parametrize("quot", ["fma", "table"])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("B", [3, 256])
def test_conv1_uint8_weight_gradient_partials_match_the_float32_ones(relu, B, quot, monkeypatch):
    """rai_conv2d_wgrad_partials_u8 / rai_conv2d_wgrad_relu_partials_u8 + the reduce: bit-identical dW (and
    db) to the float32 forms on the prescaled frames, with either in-kernel quotient."""
    from rl_algo_impls_amd.cnn_ops import _WgradJob
    if quot == "table":
        monkeypatch.setenv("RAI_CONV_U8_LUT", "1")
    u = _u8_frames(B, 84, seed=11 + B)
    gen = torch.Generator().manual_seed(B)
    dy = torch.randn(B, 32, 20, 20, generator=gen)
    y = torch.relu(torch.randn(B, 32, 20, 20, generator=gen))
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    cl = lambda t: t.to(DEV).contiguous(memory_format=torch.channels_last)
    xf = cl(u.float() / torch.tensor(255.0))
    ud, dyd, yd = cl(u), cl(dy), cl(y)
    nb = int(L.rai_conv2d_wgrad_workspace_bytes(B, 84, 84, 4, 32, 8, 8, 4))
    outs = []
    for u8 in (False, True):
        ws = torch.empty(nb, dtype=torch.uint8, device=DEV)
        gw = torch.zeros(32, 4, 8, 8, device=DEV).contiguous(memory_format=torch.channels_last)
        gb = torch.zeros(32, device=DEV)
        if relu and u8:
            rc = L.rai_conv2d_wgrad_relu_partials_u8(dyd.data_ptr(), yd.data_ptr(), ud.data_ptr(), 255.0, B, 84, 84, 4,
                                                     32, 8, 8, 4, ws.data_ptr(), nb, st)
        elif relu:
            rc = L.rai_conv2d_wgrad_relu_partials(dyd.data_ptr(), yd.data_ptr(), xf.data_ptr(), B, 84, 84, 4, 32, 8, 8,
                                                  4, ws.data_ptr(), nb, st)
        elif u8:
            rc = L.rai_conv2d_wgrad_partials_u8(ud.data_ptr(), 255.0, dyd.data_ptr(), B, 84, 84, 4, 32, 8, 8, 4,
                                                ws.data_ptr(), nb, st)
        else:
            rc = L.rai_conv2d_wgrad_partials(xf.data_ptr(), dyd.data_ptr(), B, 84, 84, 4, 32, 8, 8, 4, ws.data_ptr(),
                                             nb, st)
        _lib.check(rc, "partials")
        job = (_WgradJob * 1)(_WgradJob(ws.data_ptr(), gw.data_ptr(), gb.data_ptr() if relu else None, B, 84, 84, 4,
                                        32, 8, 8, 4, 0))
        _lib.check(L.rai_conv2d_wgrad_reduce(C.cast(job, C.c_void_p), 1, 0, st), "reduce")
        torch.cuda.synchronize()
        outs.append((gw.cpu(), gb.cpu()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    if B == 3:  # dW against fp64
        dz = torch.where(y > 0, dy, torch.zeros_like(dy)) if relu else dy
        ref = torch.ops.aten.convolution_backward(dz.double(), (u.float() / 255.0).double(),
                                                  torch.zeros(32, 4, 8, 8, dtype=torch.float64), None, [4, 4], [0, 0],
                                                  [1, 1], False, [0, 0], 1, [False, True, False])[1]
        bound = torch.ops.aten.convolution_backward(dz.double().abs(), (u.float() / 255.0).double(),
                                                    torch.zeros(32, 4, 8, 8, dtype=torch.float64), None, [4, 4],
                                                    [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])[1]
        assert ((outs[1][0].double() - ref).abs() <= (B * 400 + 2) * 2.0 ** -24 * bound + 1e-30).all()


def test_conv_uint8_rejects_shapes():
    """The _u8 forms take Ci == 4 only and a positive divisor; misaligned frames are refused."""
    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    u = torch.zeros(2, 84, 84, 8, dtype=torch.uint8, device=DEV)
    w = torch.zeros(32, 8, 8, 8, device=DEV)
    b = torch.zeros(32, device=DEV)
    y = torch.zeros(2, 32, 20, 20, device=DEV)
    assert L.rai_conv2d_bias_relu_fwd_u8(u.data_ptr(), 255.0, w.data_ptr(), b.data_ptr(), 2, 84, 84, 8, 32, 8, 8, 4, 0,
                                         y.data_ptr(), st) == -2
    assert L.rai_conv2d_bias_relu_fwd_u8(u.data_ptr(), 0.0, w.data_ptr(), b.data_ptr(), 2, 84, 84, 4, 32, 8, 8, 4, 0,
                                         y.data_ptr(), st) == -2
    assert L.rai_conv2d_bias_relu_fwd_u8(u.data_ptr() + 1, 255.0, w.data_ptr(), b.data_ptr(), 2, 84, 84, 4, 32, 8, 8,
                                         4, 0, y.data_ptr(), st) == -2
    nb = int(L.rai_conv2d_wgrad_workspace_bytes(2, 84, 84, 8, 32, 8, 8, 4))
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=DEV)
    assert L.rai_conv2d_wgrad_partials_u8(u.data_ptr(), 255.0, y.data_ptr(), 2, 84, 84, 8, 32, 8, 8, 4, ws.data_ptr(),
                                          nb, st) == -2
    torch.cuda.synchronize()


@pytest.mark.parametrize("n,B", [(700, 256), (37, 16)])
def test_gather_uint8_frames_transposed_to_nhwc(n, B):
    """RAI_XFORM_U8_CHW_TO_U8_HWC: every minibatch's frames are the permuted rows' uint8 frames in
    channels_last, byte for byte, next to a copied field; the ragged tail is left untouched.  Shapes
    other than 4 planes are refused."""
    from rl_algo_impls_amd.graphs import GraphedUpdate, gather_next, static_buffers

    g = torch.Generator(device="cpu").manual_seed(n)
    frames = torch.randint(0, 256, (n, 4, 84, 84), generator=g, dtype=torch.uint8)
    fields = [frames.to(DEV), torch.randn(n, generator=g).to(DEV)]
    xforms = [_lib.GatherXform(kind=_lib.RAI_XFORM_U8_CHW_TO_U8_HWC, channels=4, hw=84 * 84, divisor=255.0), None]
    gu = GraphedUpdate(DEV)
    gu.set_rollout(fields, B, True)
    perm = torch.randperm(n, generator=g)
    gu.start_epoch(perm.to(DEV))
    row_bytes = [int(f[0].numel() * f.element_size()) for f in fields]
    for mb in range((n + B - 1) // B):
        rows = min(B, n - mb * B)
        bufs = static_buffers(fields, B, DEV, xforms)
        assert bufs[0].dtype == torch.uint8 and bufs[0].is_contiguous(memory_format=torch.channels_last)
        bufs[0].fill_(7)
        gather_next(DEV, gu.desc, bufs, row_bytes, xforms)
        sel = perm[mb * B: mb * B + rows]
        assert torch.equal(bufs[0][:rows].cpu(), frames[sel])
        assert torch.equal(bufs[1][:rows].cpu(), fields[1][sel.to(DEV)].cpu())
        if rows < B:
            assert (bufs[0][rows:] == 7).all()
    torch.cuda.synchronize()
    out = torch.empty(B, 3, 84, 84, dtype=torch.uint8, device=DEV)
    dst = (C.c_void_p * 1)(out.data_ptr())
    rb = (C.c_int64 * 1)(3 * 84 * 84)
    arr = (_lib.GatherXform * 1)(_lib.GatherXform(kind=_lib.RAI_XFORM_U8_CHW_TO_U8_HWC, channels=3, hw=84 * 84,
                                                  divisor=255.0))
    assert _lib.lib().rai_gather_minibatch_x(gu.desc.data_ptr(), 1, C.cast(dst, C.c_void_p), C.cast(rb, C.c_void_p),
                                             C.cast(arr, C.c_void_p), B, 0, _lib.stream_handle(DEV)) == -2


def test_nature_cnn_encoder_uint8_path_equals_float32_path(monkeypatch):
    """The encoder on uint8 frames: conv1 reading the frames itself (RAI_CONV_U8, default) gives the same
    features, bit for bit, as the float32 prescale path, and -- inside direct_grads(), as in the trainer,
    where conv1's weight gradient runs rai_conv2d_wgrad_relu_partials_u8 -- the same parameter gradients.
    The conv weights are channels_last as the trainer's flat buffer stores them (the MFMA kernels' layout;
    MIOpen's weight gradient would not be bit-reproducible)."""
    import make_golden_networks as nets
    from rl_algo_impls_amd import cnn_ops
    from rl_algo_impls_amd.policy import ActorCritic

    torch.manual_seed(0)
    pol = ActorCritic(nets.pong_env(), activation_fn="relu").to(DEV)
    enc = pol.network._feature_extractor.feature_extractor
    for m in enc.cnn:
        if isinstance(m, torch.nn.Conv2d):
            m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
    g = torch.Generator().manual_seed(9)
    obs = torch.randint(0, 256, (64, 4, 84, 84), generator=g, dtype=torch.uint8).to(DEV)
    assert enc.obs_transform(obs).kind == _lib.RAI_XFORM_U8_CHW_TO_U8_HWC
    outs = []
    for u8 in (False, True, False):  # the first pass settles the fc GEMMs' tuned solutions (TunableOp)
        monkeypatch.setattr(cnn_ops, "_CONV_U8", u8)
        for p in enc.parameters():
            p.grad = torch.zeros_like(p)  # conv weights: channels_last like their data
        with cnn_ops.direct_grads():
            f = enc(obs)
            f.square().sum().backward()
        torch.cuda.synchronize()
        outs.append((f.detach().cpu(), [p.grad.detach().cpu().clone() for p in enc.parameters()]))
    outs = outs[1:]
    assert torch.equal(outs[0][0], outs[1][0])
    for (name, _), a, b in zip(enc.named_parameters(), outs[0][1], outs[1][1]):
        assert torch.equal(a, b), name
    monkeypatch.setattr(cnn_ops, "_CONV_U8", False)
    assert enc.obs_transform(obs).kind == _lib.RAI_XFORM_U8_CHW_TO_F32_HWC


def test_conv_dgrad_shape_gates_fall_back_instead_of_raising():
    """A valid convolution shape the MFMA input-gradient kernels are not instantiated for (Ci < 16, Co not a
    multiple of 16, kernel not a multiple of the stride) returns RAI_E_UNSUPPORTED (not RAI_E_SHAPE), so
    cnn_ops falls back (MIOpen for dx, the materialised dz for the ReLU fold) instead of raising; an
    impossible shape stays RAI_E_SHAPE."""
    from rl_algo_impls_amd import cnn_ops

    L = _lib.lib()
    st = _lib.stream_handle(DEV)
    p = torch.zeros(64, device=DEV).data_ptr()
    assert L.rai_conv2d_dgrad_relu(p, p, p, 2, 20, 20, 8, 64, 4, 4, 2, p, st) == -6  # Ci < 16
    assert L.rai_conv2d_dgrad_relu(p, p, p, 2, 20, 20, 32, 24, 4, 4, 2, p, st) == -6  # Co % 16
    assert L.rai_conv2d_dgrad_v(p, p, 2, 20, 20, 32, 24, 4, 4, 2, p, 0, st) == -6
    assert L.rai_conv2d_dgrad_v(p, p, 2, 20, 20, 16, 64, 4, 4, 2, p, 0, st) == -6  # Ci not 32 / 64
    assert L.rai_conv2d_dgrad_v(p, p, 2, 3, 3, 32, 64, 4, 4, 2, p, 0, st) == -2  # kernel larger than the input
    # the Python paths: None (fold skipped) and MIOpen's dx, equal to fp64 autograd within f32 bounds
    B, Ci, H, Co, k, s = 3, 8, 20, 24, 4, 2
    x, w, _ = _inputs(B, Ci, H, Co, k, seed=5)
    OH = (H - k) // s + 1
    dz = torch.randn(B, Co, OH, OH, generator=torch.Generator().manual_seed(9))
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV).contiguous(memory_format=torch.channels_last)
    dzd = dz.to(DEV).contiguous(memory_format=torch.channels_last)
    y = torch.rand_like(dzd)
    assert cnn_ops._conv_dgrad_relu(xd, dzd, y, wd, s) is None
    dx = cnn_ops._conv_dgrad(xd, dzd, wd, s)
    ref = torch.ops.aten.convolution_backward(dz.double(), x.double(), w.double(), None, [s, s], [0, 0], [1, 1], False,
                                              [0, 0], 1, [True, False, False])[0]
    torch.testing.assert_close(dx.cpu().double(), ref, rtol=1e-4, atol=1e-4)
