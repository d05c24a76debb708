"""Detection layers: golden values from the reference specs (RoiAlignSpec, PoolerSpec, NmsSpec,
PriorBoxSpec — numbers extracted into tests/fixtures/detection_golden.json) plus shape/semantics
tests for Anchor, Proposal, RegionProposal, DetectionOutputSSD/Frcnn, FPN, BoxHead, MaskHead."""
import json
import os

import numpy as np
import pytest
import torch

from bigdl.nn import (Anchor, Nms, Proposal, RegionProposal, PriorBox, DetectionOutputSSD, DetectionOutputFrcnn,
                      Pooler, FPN, BoxHead, MaskHead, RoiAlign, nms)
from bigdl.utils.table import Table

FX = json.load(open(os.path.join(os.path.dirname(__file__), "fixtures", "detection_golden.json")))


def test_roialign_golden():
    g = FX["roialign"]
    data = torch.tensor(g["data"]).view(1, 2, 6, 8)
    rois = torch.tensor(g["rois"]).view(4, 4)
    out = RoiAlign(1.0, 3, 2, 2).forward(Table(data, rois))
    np.testing.assert_allclose(out.flatten().numpy(), g["expectedRes"], atol=1e-6)


def test_roialign_backward_matches_autograd_shape():
    data = torch.randn(2, 3, 9, 9)
    rois = torch.tensor([[0, 1.0, 1.0, 6.0, 7.0], [1, 0.0, 2.0, 8.0, 5.0]])
    m = RoiAlign(1.0, 2, 3, 3)
    y = m.forward(Table(data, rois))
    gi = m.backward(Table(data, rois), torch.ones_like(y))
    assert gi[1].shape == data.shape
    assert abs(float(gi[1].sum()) - y.numel()) < 1e-3  # bilinear weights of each sample sum to 1


def test_pooler_golden():
    g = FX["pooler"]
    feats = Table(torch.tensor(g["feature1"]).view(1, 2, 8, 8), torch.tensor(g["feature2"]).view(1, 2, 4, 4),
                  torch.tensor(g["feature3"]).view(1, 2, 2, 2))
    rois = torch.tensor([[0, 0, 10, 10], [0, 0, 60, 60], [0, 0, 500, 500]], dtype=torch.float32)
    out = Pooler(2, [0.125, 0.0625, 0.03125], 2).forward(Table(feats, Table(rois)))
    np.testing.assert_allclose(out.flatten().numpy(), g["expectedRes"], atol=1e-6)


@pytest.mark.parametrize("thresh,key", [(0.4, "expected_04"), (0.1, "expected_01")])
def test_nms_golden(thresh, key):
    d = torch.tensor(FX["nms"]["dets"]).view(112, 5)
    idx = np.zeros(112, dtype=np.int64)
    n = Nms().nms(d[:, 4].contiguous(), d[:, :4].contiguous(), thresh, idx)
    assert idx[:n].tolist() == FX["nms"][key]


def test_nms_matches_bruteforce():
    g = torch.Generator().manual_seed(0)
    xy = torch.rand(200, 2, generator=g) * 100
    wh = torch.rand(200, 2, generator=g) * 30 + 1
    boxes = torch.cat([xy, xy + wh], 1)
    scores = torch.rand(200, generator=g)
    keep = nms(boxes, scores, 0.5).tolist()
    order = torch.argsort(scores, descending=True).tolist()
    ref, alive = [], set(order)
    for i in order:
        if i not in alive:
            continue
        ref.append(i)
        for j in order:
            if j in alive and j != i:
                a, b = boxes[i], boxes[j]
                iw = max(0.0, float(min(a[2], b[2]) - max(a[0], b[0]) + 1))
                ih = max(0.0, float(min(a[3], b[3]) - max(a[1], b[1]) + 1))
                inter = iw * ih
                ua = float((a[2] - a[0] + 1) * (a[3] - a[1] + 1) + (b[2] - b[0] + 1) * (b[3] - b[1] + 1)) - inter
                if inter / ua > 0.5:
                    alive.discard(j)
        alive.discard(i)
    assert keep == ref


def test_priorbox_golden():
    layer = PriorBox([460.8], [537.6], [2.0], is_flip=True, is_clip=False, variances=[0.1, 0.1, 0.2, 0.2],
                     offset=0.5, img_h=512, img_w=512)
    out = layer.forward(torch.zeros(8, 256, 1, 1))
    assert out.shape == (1, 2, 16)
    np.testing.assert_allclose(out.flatten().numpy(), FX["priorbox"], atol=1e-5)


def test_anchor_basic_values():
    a = Anchor([0.5, 1.0, 2.0], [8.0, 16.0, 32.0])
    b = a.basic_anchors(16)
    assert b[0].tolist() == [-84.0, -40.0, 99.0, 55.0]
    assert b[4].tolist() == [-120.0, -120.0, 135.0, 135.0]
    full = a.generate_anchors(3, 2, 16)
    assert full.shape == (3 * 2 * 9, 4)
    # second cell in x is the first cell shifted by the stride
    assert torch.equal(full[9:18], b + torch.tensor([16.0, 0, 16.0, 0]))


def test_proposal_shapes_and_order():
    torch.manual_seed(0)
    A, H, W = 9, 6, 8
    scores = torch.rand(1, 2 * A, H, W)
    deltas = torch.randn(1, 4 * A, H, W) * 0.1
    info = torch.tensor([[96.0, 128.0, 1.0, 1.0]])
    p = Proposal(300, 50, [0.5, 1.0, 2.0], [8.0, 16.0, 32.0], 600, 100)
    p.evaluate()
    out = p.forward(Table(scores, deltas, info))
    assert out.shape[1] == 5 and 0 < out.shape[0] <= 50
    assert (out[:, 0] == 0).all()
    assert (out[:, 1] >= 0).all() and (out[:, 3] <= 127).all() and (out[:, 4] <= 95).all()


def test_region_proposal_batch():
    torch.manual_seed(0)
    rp = RegionProposal(8, [32, 64], [0.5, 1.0, 2.0], [4, 8], 100, 20, 100, 20, 0.7, 0)
    rp.evaluate()
    feats = Table(torch.randn(2, 8, 16, 16), torch.randn(2, 8, 8, 8))
    out = rp.forward(Table(feats, torch.tensor([64.0, 64.0])))
    assert len(out) == 2
    for i in (1, 2):
        assert out[i].shape[1] == 4 and 0 < out[i].shape[0] <= 20


def test_detection_output_ssd():
    torch.manual_seed(0)
    pri = PriorBox([30.0], [60.0], [2.0], img_h=300, img_w=300).forward(torch.zeros(1, 4, 5, 5))
    P = pri.shape[-1] // 4
    loc = torch.zeros(2, P * 4)
    conf = torch.randn(2, P * 21) * 3
    d = DetectionOutputSSD(21, keep_top_k=50, conf_thresh=0.3)
    d.evaluate()
    out = d.forward(Table(loc, conf, pri))
    assert out.shape[0] == 2
    for b in range(2):
        n = int(out[b, 0])
        assert 0 < n <= 50
        dets = out[b, 1:1 + 6 * n].view(n, 6)
        assert (dets[:, 0] >= 1).all() and (dets[:, 1] > 0.3).all()
        assert torch.equal(dets[:, 0], dets[:, 0].sort().values)  # grouped by label


def test_detection_output_frcnn():
    torch.manual_seed(0)
    K, C = 30, 5
    rois = torch.cat([torch.zeros(K, 1), torch.rand(K, 2) * 50, torch.rand(K, 2) * 50 + 60], 1)
    d = DetectionOutputFrcnn(n_classes=C, max_per_image=10)
    d.evaluate()
    out = d.forward(Table(torch.tensor([[200.0, 200.0, 1.0, 1.0]]), rois, torch.zeros(K, 4 * C),
                          torch.softmax(torch.randn(K, C) * 3, 1)))
    n = int(out[0])
    assert 0 < n <= 10 and out.numel() == 1 + 6 * n


def test_fpn_and_heads():
    torch.manual_seed(0)
    fpn = FPN([8, 16, 32], 8, top_blocks=1)
    c = Table(torch.randn(1, 8, 32, 32), torch.randn(1, 16, 16, 16), torch.randn(1, 32, 8, 8))
    p = fpn.forward(c)
    assert [tuple(p[i].shape) for i in range(1, 5)] == [(1, 8, 32, 32), (1, 8, 16, 16), (1, 8, 8, 8), (1, 8, 4, 4)]
    feats = Table(p[1], p[2], p[3])
    props = torch.tensor([[0.0, 0.0, 40.0, 40.0], [10.0, 10.0, 120.0, 100.0], [5.0, 5.0, 20.0, 30.0]])
    bh = BoxHead(8, 4, [0.25, 0.125, 0.0625], 2, 0.0, 0.5, 10, 32, 4)
    bh.evaluate()
    out = bh.forward(Table(feats, props, torch.tensor([128.0, 128.0])))
    assert out[1].shape == (3, 32)
    labels, boxes, scores = out[2][1], out[2][2][1], out[2][3]
    assert labels.shape[0] == boxes.shape[0] == scores.shape[0] <= 10
    mh = MaskHead(8, 4, [0.25, 0.125, 0.0625], 2, [8, 8], 1, 4)
    mh.evaluate()
    mo = mh.forward(Table(feats, boxes, labels))
    assert mo[2].shape == (boxes.shape[0], 1, 8, 8)
    assert ((mo[2] >= 0) & (mo[2] <= 1)).all()


def test_maskrcnn_inference_smoke():
    from bigdl.models import MaskRCNN, MaskRCNNParams
    torch.manual_seed(0)
    cfg = MaskRCNNParams(preNmsTopNTest=50, postNmsTopNTest=20, outputSize=64, boxScoreThresh=0.0,
                         maxPerImage=5, layers=[16, 16])
    m = MaskRCNN(in_channels=32, out_channels=16, num_classes=5, config=cfg)
    m.evaluate()
    img = torch.randn(1, 3, 64, 64)
    out = m.forward(Table(img, torch.tensor([[64.0, 64.0, 128.0, 96.0]])))
    r = out[1]
    n = r["bboxes"].shape[0]
    assert 0 < n <= 5 and len(r["masks"]) == n and r["classes"].shape[0] == n
    assert r["masks"][0].height == 128 and r["masks"][0].width == 96
