"""Detection kernels (ops/csrc/detection.hip, K28): device NMS against the host greedy scan over
the fp32 IoU matrix, and ROI align forward / backward against the torch gather formulation
(reference nn/Nms.scala, nn/RoiAlign.scala)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def N():
    from bigdl.ops import native
    from bigdl.utils.engine import Engine
    Engine.init(device="cuda:0")
    assert native.status()["loaded"] and native.has("nms") and native.has("roi_align")
    return native


def _boxes(n, seed=0, span=200.0):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(n, 2, generator=g) * span
    wh = torch.rand(n, 2, generator=g) * 60 + 2
    return torch.cat([xy, xy + wh], 1), torch.rand(n, generator=g)


def _host_nms(boxes, scores, thresh, plus_one, max_keep=-1):
    from bigdl.nn.layers.detection import box_iou
    order = torch.argsort(scores, descending=True)
    b = boxes[order].float()
    over = (box_iou(b, b, plus_one) > thresh).numpy()
    keep, removed = [], np.zeros(len(b), bool)
    for i in range(len(b)):
        if removed[i]:
            continue
        keep.append(i)
        if 0 < max_keep <= len(keep):
            break
        removed |= over[i]
    return order[keep]


@pytest.mark.parametrize("n,thresh,plus_one", [(1, 0.5, 1.0), (63, 0.5, 1.0), (64, 0.3, 0.0), (65, 0.7, 1.0),
                                               (1000, 0.5, 1.0), (6000, 0.7, 1.0)])
def test_nms_matches_host_scan(N, n, thresh, plus_one):
    from bigdl.nn.layers.detection import nms
    boxes, scores = _boxes(n, seed=n)
    ref = _host_nms(boxes, scores, thresh, plus_one)
    got = nms(boxes.cuda(), scores.cuda(), thresh, plus_one=plus_one).cpu()
    assert torch.equal(got, ref), (got[:20], ref[:20])
    assert N.fallback_counts() == {} or not any(k[0] == "nms" for k in N.fallback_counts())


def test_nms_max_keep(N):
    from bigdl.nn.layers.detection import nms
    boxes, scores = _boxes(3000, seed=7)
    ref = _host_nms(boxes, scores, 0.5, 1.0, max_keep=100)
    got = nms(boxes.cuda(), scores.cuda(), 0.5, max_keep=100).cpu()
    assert len(got) == 100 and torch.equal(got, ref)


def _rois(K, N_, H, W, seed=0):
    g = torch.Generator().manual_seed(seed)
    x1 = torch.rand(K, generator=g) * W * 6
    y1 = torch.rand(K, generator=g) * H * 6
    w = torch.rand(K, generator=g) * W * 4 + 1
    h = torch.rand(K, generator=g) * H * 4 + 1
    b = torch.randint(0, N_, (K,), generator=g).float()
    return torch.stack([b, x1, y1, x1 + w, y1 + h], 1)


def _ref_roi_align(data, rois, scale, oh, ow, sr, aligned):
    from bigdl.nn.layers import pooling
    # the torch gather path (run on the host so the native path cannot be taken)
    return pooling.roi_align(data.detach().float().cpu(), rois.cpu(), scale, oh, ow, sr, aligned)


@pytest.mark.parametrize("sr,aligned", [(2, True), (2, False), (0, False), (0, True)])
@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
def test_roi_align_forward(N, sr, aligned, layout):
    from bigdl.nn.layers.pooling import roi_align
    data = torch.randn(2, 16, 20, 24)
    rois = _rois(37, 2, 20, 24)
    ref = _ref_roi_align(data, rois, 0.125, 7, 7, sr, aligned)
    d = data.cuda()
    if layout == "nhwc":
        d = d.contiguous(memory_format=torch.channels_last)
    got = roi_align(d, rois.cuda(), 0.125, 7, 7, sr, aligned)
    assert got.shape == ref.shape
    torch.testing.assert_close(got.cpu(), ref, rtol=1e-4, atol=1e-5)


def test_roi_align_bf16_input(N):
    from bigdl.nn.layers.pooling import roi_align
    data = torch.randn(1, 32, 14, 14).to(torch.bfloat16)
    rois = _rois(20, 1, 14, 14, seed=3)
    ref = _ref_roi_align(data.float(), rois, 0.25, 5, 5, 2, False)
    got = roi_align(data.cuda(), rois.cuda(), 0.25, 5, 5, 2, False)
    assert got.dtype == torch.bfloat16
    torch.testing.assert_close(got.float().cpu(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("sr,aligned", [(2, False), (0, True)])
def test_roi_align_backward(N, sr, aligned):
    from bigdl.nn.layers.pooling import roi_align
    data = torch.randn(2, 8, 12, 16, dtype=torch.float32)
    rois = _rois(25, 2, 12, 16, seed=5)
    gout = torch.randn(25, 8, 4, 4)
    xr = data.clone().requires_grad_(True)
    from bigdl.nn.layers import pooling
    yr = pooling.roi_align(xr, rois, 0.25, 4, 4, sr, aligned)
    yr.backward(gout)
    xd = data.cuda().requires_grad_(True)
    yd = roi_align(xd, rois.cuda(), 0.25, 4, 4, sr, aligned)
    yd.backward(gout.cuda())
    torch.testing.assert_close(xd.grad.cpu(), xr.grad, rtol=1e-4, atol=1e-4)


def test_roialign_layer_on_device(N):
    from bigdl.nn.layers.pooling import RoiAlign
    from bigdl.utils.table import T
    data = torch.randn(1, 4, 10, 10)
    rois = torch.tensor([[1.0, 1.0, 30.0, 30.0], [5.0, 8.0, 60.0, 70.0]])
    m = RoiAlign(0.125, 2, 3, 3)
    host = m.forward(T(data, rois)).clone()
    dev = RoiAlign(0.125, 2, 3, 3).forward(T(data.cuda(), rois.cuda()))
    torch.testing.assert_close(dev.cpu().float(), host.float(), rtol=1e-4, atol=1e-5)
