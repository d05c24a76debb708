"""Data layer: vision ImageFeature/ImageFrame transforms, legacy BGR pipeline, text pipeline,
COCO RLE masks (MaskApi.c encoding), datamining RowTransformer, and the K25 device kernel."""
import io

import numpy as np
import pytest
import torch

from bigdl.transform.vision.image import (ImageFeature, ImageFrame, BytesToMat, Resize, CenterCrop, RandomCrop,
                                          HFlip, ChannelNormalize, MatToTensor, ImageFrameToSample, ColorJitter,
                                          Expand, RoiLabel, RoiNormalize, RoiHFlip, RoiProject, FixedCrop,
                                          MTImageFeatureToBatch, RandomAlterAspect, BboxUtil, bgr_to_hsv,
                                          hsv_to_bgr, Filler, ImageFeatureToMiniBatch)


def _png(h=40, w=50, seed=0):
    from PIL import Image
    rng = np.random.RandomState(seed)
    img = (rng.rand(h, w, 3) * 255).astype(np.uint8)
    buf = io.BytesIO()
    Image.fromarray(img).save(buf, format="PNG")
    return buf.getvalue(), img


def test_bytes_to_mat_is_bgr():
    b, rgb = _png()
    f = BytesToMat().transform(ImageFeature(b))
    m = f.opencv_mat()
    assert m.shape == (40, 50, 3)
    assert torch.equal(m[..., 0].to(torch.uint8), torch.from_numpy(rgb[..., 2]))


def test_geometry_and_normalize():
    b, _ = _png()
    f = ImageFeature(b, 2.0)
    pipe = BytesToMat() >> Resize(30, 36) >> CenterCrop(20, 10) >> HFlip()
    pipe.transform(f)
    assert f.get_size() == (10, 20, 3)
    m = f.opencv_mat().clone()
    ChannelNormalize(10.0, 20.0, 30.0, 2.0, 4.0, 5.0).transform(f)
    torch.testing.assert_close(f.opencv_mat()[..., 0], (m[..., 0] - 30.0) / 5.0)  # B channel uses meanB
    MatToTensor(to_rgb=True).transform(f)
    assert f[ImageFeature.imageTensor].shape == (3, 10, 20)


def test_hsv_roundtrip_and_jitter_finite():
    x = torch.rand(8, 8, 3) * 255
    torch.testing.assert_close(hsv_to_bgr(bgr_to_hsv(x)), x, rtol=1e-4, atol=1e-3)
    b, _ = _png()
    f = (BytesToMat() >> ColorJitter(random_order_prob=0.5) >> RandomAlterAspect(crop_length=16)).transform(
        ImageFeature(b))
    assert f.get_size() == (16, 16, 3) and torch.isfinite(f.opencv_mat()).all()


def test_roi_transforms():
    b, _ = _png(40, 40)
    f = BytesToMat().transform(ImageFeature(b))
    f[ImageFeature.label] = RoiLabel(torch.tensor([1.0, 2.0]), torch.tensor([[0, 0, 20, 20], [20, 20, 40, 40.]]))
    RoiNormalize().transform(f)
    torch.testing.assert_close(f.get_label().bboxes[1], torch.tensor([0.5, 0.5, 1.0, 1.0]))
    RoiHFlip().transform(f)
    torch.testing.assert_close(f.get_label().bboxes[0], torch.tensor([0.5, 0.0, 1.0, 0.5]))
    FixedCrop(0.0, 0.0, 0.5, 0.5, True).transform(f)
    RoiProject().transform(f)
    assert f.get_label().size() == 0 or f.get_label().bboxes.max() <= 1
    a = torch.tensor([[0, 0, 10, 10.]])
    bb = torch.tensor([[5, 5, 15, 15.], [20, 20, 30, 30]])
    torch.testing.assert_close(BboxUtil.iou(a, bb), torch.tensor([[25 / 175, 0.0]]))
    pri = torch.tensor([[0, 0, 10, 10.], [5, 5, 25, 15]])
    boxes = torch.tensor([[1, 1, 9, 11.], [6, 4, 20, 16]])
    torch.testing.assert_close(BboxUtil.decode(BboxUtil.encode(boxes, pri), pri), boxes, rtol=1e-5, atol=1e-4)


def test_frame_and_minibatch():
    fr = ImageFrame.array([ImageFeature(_png(seed=i)[0], float(i + 1)) for i in range(5)])
    fr = fr.transform(BytesToMat() >> Resize(16, 16) >> MatToTensor() >> ImageFrameToSample(target_keys=["label"]))
    batches = list(ImageFeatureToMiniBatch(2)(fr.array))
    assert [b.size() for b in batches] == [2, 2, 1]
    assert batches[0].getInput().shape == (2, 3, 16, 16)
    dfr = fr.to_distributed(rank=1, world=2)
    assert len(dfr) == 2


def test_mt_batch_cpu_matches_reference():
    feats = [BytesToMat().transform(ImageFeature(_png(seed=i)[0], float(i + 1))) for i in range(3)]
    mt = MTImageFeatureToBatch(24, 20, 4, mean=(1, 2, 3), std=(2, 3, 4), device="cpu")
    b = next(iter(mt(feats)))
    x = b.getInput()
    assert x.shape == (3, 3, 20, 24)
    m = feats[0].opencv_mat()
    crop = m[10:30, 13:37].flip(2)  # center crop, BGR→RGB
    ref = (crop - torch.tensor([1.0, 2.0, 3.0])) / torch.tensor([2.0, 3.0, 4.0])
    torch.testing.assert_close(x[0].permute(1, 2, 0), ref)
    assert b.getTarget().tolist() == [1.0, 2.0, 3.0]


def test_legacy_bgr_pipeline():
    from bigdl.dataset.image import (ByteRecord, BytesToBGRImg, BGRImgCropper, BGRImgNormalizer, HFlip as LH,
                                     BGRImgToBatch, Lighting, ColorJitter as LCJ, BGRImgRdmCropper, BGRImgToSample)
    recs = [ByteRecord(_png(seed=i)[0], float(i + 1)) for i in range(3)]
    chain = BytesToBGRImg() >> BGRImgCropper(32, 32, "center") >> LH(0.5) >> LCJ() >> Lighting() >> \
        BGRImgNormalizer((0.4, 0.4, 0.4), (0.2, 0.2, 0.2)) >> BGRImgToBatch(2)
    batches = list(chain(iter(recs)))
    assert batches[0].getInput().shape == (2, 3, 32, 32) and batches[1].size() == 1
    s = next((BytesToBGRImg() >> BGRImgRdmCropper(32, 32, 4) >> BGRImgToSample())(iter(recs)))
    assert s.feature().shape == (3, 32, 32)


def test_text_pipeline(tmp_path):
    from bigdl.dataset.text import (Dictionary, SentenceSplitter, SentenceTokenizer, SentenceBiPadding,
                                    TextToLabeledSentence, LabeledSentenceToSample)
    text = ["The cat sat. The dog ran! A cat ran."]
    sents = list(SentenceSplitter()(iter(text)))[0]
    assert len(sents) == 3
    padded = list(SentenceBiPadding()(iter(sents)))
    toks = list(SentenceTokenizer()(iter(padded)))
    d = Dictionary(toks, 100)
    assert d.get_vocab_size() == len({w for t in toks for w in t})
    assert d.get_index("zzz-unknown") == d.get_vocab_size()
    d.save(str(tmp_path))
    d2 = Dictionary(directory=str(tmp_path))
    assert d2.word2index() == d.word2index()
    ls = list(TextToLabeledSentence(d)(iter(toks)))
    assert ls[0].dataLength() == len(toks[0]) - 1
    samples = list(LabeledSentenceToSample(d.get_vocab_size() + 1, 8, 8)(iter(ls)))
    assert samples[0].feature().shape == (8, d.get_vocab_size() + 1)
    assert samples[0].feature().sum() == 8 and samples[0].label().min() >= 1


def test_coco_rle_string_roundtrip_and_iou():
    from bigdl.dataset.segmentation import MaskUtils, RLEMasks, PolyMasks
    m = torch.zeros(6, 5, dtype=torch.uint8)
    m[1:4, 1:3] = 1
    m[5, 4] = 1
    r = MaskUtils.binary_to_rle(m)
    assert MaskUtils.rle_area(r) == int(m.sum())
    assert torch.equal(MaskUtils.rle_to_binary(r), m)
    s = MaskUtils.rle2string(r)
    assert MaskUtils.string2rle(s, 6, 5) == r
    # known COCO compact string: counts [3, 2, 5] → "32;" style round trip on large deltas too
    big = RLEMasks([100000, 7, 3, 250000, 1], 600, 600)
    assert MaskUtils.string2rle(MaskUtils.rle2string(big), 600, 600) == big
    m2 = torch.zeros(6, 5, dtype=torch.uint8)
    m2[1:4, 1:2] = 1
    iou = MaskUtils.rle_iou(MaskUtils.binary_to_rle(m2), r, False)
    assert abs(iou - 3 / 7) < 1e-6
    pm = PolyMasks([[1, 1, 8, 1, 8, 8, 1, 8]], 10, 10)
    assert MaskUtils.rle_area(pm.to_rle()) >= 49
    assert MaskUtils.bbox_iou((0, 0, 2, 2), (1, 1, 3, 3), False) == pytest.approx(1 / 7)


def test_row_transformer():
    from bigdl.dataset.datamining import RowTransformer
    rows = [{"a": 1, "b": 2.5, "c": 3}, {"a": 4, "b": 5, "c": 6}]
    t = list(RowTransformer.numeric({"x": ["a", "b"], "y": ["c"]})(iter(rows)))
    assert t[0]["x"].tolist() == [1.0, 2.5] and t[1]["y"].tolist() == [6.0]
    t2 = list(RowTransformer.atomic(["a", "c"], schema=["a", "b", "c"])(iter([(7, 8, 9)])))
    assert t2[0]["c"].tolist() == [9.0]


@pytest.mark.gpu
def test_image_kernel_matches_reference():
    from bigdl.ops import native_ops as NO, reference as R, native_status
    assert native_status()["loaded"]
    src = (torch.rand(3, 20, 30, 3) * 255).to(torch.uint8).cuda()
    oy, ox, fl = torch.tensor([0, 3, 5]), torch.tensor([1, 0, 7]), torch.tensor([0, 1, 1])
    for to_rgb in (True, False):
        for dt in (torch.float32, torch.bfloat16):
            out = NO.image_crop_flip_norm(src, oy, ox, fl, 12, 16, (1, 2, 3), (2, 3, 4), to_rgb, dt)
            ref = R.image_crop_flip_norm(src, oy, ox, fl, 12, 16, (1, 2, 3), (2, 3, 4), to_rgb, dt)
            torch.testing.assert_close(out.float(), ref.float(), rtol=1e-2, atol=1e-2)


def test_pyspark_dataset_modules(tmp_path):
    """``bigdl.dataset.{mnist,movielens,news20,sentence,base}`` on synthetic local files."""
    import gzip
    import struct
    import numpy as np
    from bigdl.dataset import mnist, movielens, news20, sentence, base
    imgs = (np.arange(3 * 28 * 28) % 256).astype(np.uint8)
    with gzip.open(tmp_path / "train-images-idx3-ubyte.gz", "wb") as f:
        f.write(struct.pack(">IIII", 2051, 3, 28, 28) + imgs.tobytes())
    with gzip.open(tmp_path / "train-labels-idx1-ubyte.gz", "wb") as f:
        f.write(struct.pack(">II", 2049, 3) + bytes([7, 0, 9]))
    x, y = mnist.read_data_sets(str(tmp_path), "train")
    assert x.shape == (3, 28, 28, 1) and list(y) == [7, 0, 9]
    with open(tmp_path / "train-images-idx3-ubyte.gz", "rb") as f:
        assert mnist.extract_images(f).shape == (3, 28, 28, 1)
    (tmp_path / "ml-1m").mkdir()
    (tmp_path / "ml-1m" / "ratings.dat").write_text("1::10::5::978\n2::20::3::979\n")
    assert movielens.get_id_ratings(str(tmp_path)).tolist() == [[1, 10, 5], [2, 20, 3]]
    d = tmp_path / "news" / "20news-18828"
    for c, docs in (("alt.atheism", ["1", "2"]), ("sci.space", ["5"])):
        (d / c).mkdir(parents=True)
        for n in docs:
            (d / c / n).write_text(f"text {c} {n}")
    texts = news20.get_news20(str(tmp_path / "news"))
    assert [t[1] for t in texts] == [1, 1, 2]
    assert sentence.sentences_split("Hi there. How are you? Fine!") == ["Hi there.", "How are you?", "Fine!"]
    assert sentence.sentence_tokenizer("a, b") == ["a", ",", "b"]
    with pytest.raises(FileNotFoundError):
        base.maybe_download("nope.gz", str(tmp_path), "http://example/nope.gz")


def test_sequence_file_roundtrip_and_seqfilefolder(tmp_path):
    """Hadoop SequenceFile container (Text key "name\\nlabel", Text value w/h + BGR bytes) as the
    reference's ``BGRImgToLocalSeqFile`` writes it, read back by ``SeqFileFolder``."""
    import numpy as np
    from bigdl.dataset.seqfile import (BGRImgToLocalSeqFile, SeqFileFolder, read_sequence_file, write_vlong,
                                       read_vlong)
    import io
    for v in (0, 5, -7, 127, -112, 128, 300, -1000, 2 ** 31, -(2 ** 40)):
        b = io.BytesIO()
        write_vlong(b, v)
        b.seek(0)
        assert read_vlong(b) == v
    rng = np.random.RandomState(0)
    items = [(rng.randint(0, 256, (5 + i, 7, 3)).astype(np.uint8), i % 3 + 1, f"img{i}") for i in range(9)]
    files = BGRImgToLocalSeqFile(4, str(tmp_path / "part"), has_name=True)(items)
    assert len(files) == 3
    recs = list(SeqFileFolder.read(str(tmp_path)))
    assert len(recs) == 9
    for (img, lab, name), (i0, l0, n0) in zip(recs, items):
        assert np.array_equal(img, i0) and lab == l0 and name == n0
    frame = SeqFileFolder.files_to_image_frame(str(tmp_path), None, 3)
    assert len(list(frame)) == 9
    assert sum(1 for _ in read_sequence_file(files[0])) == 4


def test_ssd_random_sampler():
    import torch
    from bigdl.transform.vision.image import ImageFeature, RandomSampler, RoiProject
    from bigdl.transform.vision.image.label import RoiLabel
    from bigdl.utils.random import RNG
    RNG.setSeed(3)
    for _ in range(10):
        f = ImageFeature(image=torch.rand(60, 80, 3) * 255)
        f[ImageFeature.label] = RoiLabel(torch.tensor([1.0]), torch.tensor([[0.2, 0.2, 0.6, 0.7]]))
        RandomSampler().transform(f)
        h, w = f.get_height(), f.get_width()
        assert 1 <= h <= 60 and 1 <= w <= 80
        assert ImageFeature.cropBbox in f
