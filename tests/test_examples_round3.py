"""The reference's remaining example programs, run end to end on small synthetic inputs (CPU):
``example/lenetLocal`` (train → checkpoint → test → predict), ``example/tensorflow/loadandsave``
(save the reference LeNet Graph as a GraphDef, load it back, same output),
``example/tensorflow/transferlearning`` (features from a TF graph's own input pipeline — the
reference's ``lenet_batch_2.pbtxt`` / ``mnist_train.tfrecord`` fixtures), ``example/dlframes``
(image inference + Pipeline transfer learning over a Caffe model written by the Caffe persister),
``example/mkldnn/int8`` (GenerateInt8Scales → quantized ImageNet inference on sequence files) and
``example/treeLSTMSentiment`` (SST-format trees, GloVe vocabulary, Tree-LSTM training)."""
import os
import random
import struct

import numpy as np
import pytest
import torch

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "tf")


def _mnist(d, n_train=120, n_test=36):
    rng = np.random.default_rng(0)

    def write(pre, n):
        y = rng.integers(0, 10, n).astype(np.uint8)
        x = np.zeros((n, 28, 28), np.uint8)
        for i in range(n):
            x[i, 2 * y[i]:2 * y[i] + 6, 4:24] = 200
        x += rng.integers(0, 30, x.shape).astype(np.uint8)
        with open(os.path.join(d, f"{pre}-images-idx3-ubyte"), "wb") as f:
            f.write(struct.pack(">IIII", 2051, n, 28, 28) + x.tobytes())
        with open(os.path.join(d, f"{pre}-labels-idx1-ubyte"), "wb") as f:
            f.write(struct.pack(">II", 2049, n) + y.tobytes())
    write("train", n_train)
    write("t10k", n_test)


def test_lenet_local_train_test_predict(tmp_path):
    from bigdl.example import lenetLocal as L
    d = str(tmp_path)
    _mnist(d)
    ck = os.path.join(d, "ck")
    L.main(["train", "-f", d, "-b", "12", "-e", "2", "-r", "0.1", "--checkpoint", ck])
    snaps = sorted((os.path.join(r, f) for r, _, fs in os.walk(ck) for f in fs if f.startswith("model.")),
                   key=lambda p: int(p.rsplit(".", 1)[1]))
    assert snaps, "no model checkpoint written"
    res = L.main(["test", "-f", d, "--model", snaps[-1], "-b", "16"])
    acc = res[0][0].result()[0]
    assert acc > 0.5, acc  # the class-dependent synthetic pattern is learnable in 2 epochs
    classes = L.main(["predict", "-f", d, "--model", snaps[-1]])
    assert len(classes) == 36 and classes.min() >= 1 and classes.max() <= 10


def test_tensorflow_save_then_load(tmp_path):
    from bigdl.example.tensorflow import loadandsave as LS
    p = str(tmp_path / "bigdl.pb")
    m = LS.save(p)
    x = torch.rand(1, 1, 28, 28)
    y0 = m.forward(x)
    _, y1 = LS.load(p, ["input"], ["output"], x)
    torch.testing.assert_close(y1.reshape(y0.shape), y0, atol=1e-5, rtol=1e-5)


def test_tensorflow_transfer_learning_on_graph_pipeline(tmp_path):
    from bigdl.example.tensorflow import transferlearning as TL
    src = open(os.path.join(FIX, "lenet_batch_2.pbtxt")).read()
    src = src.replace("/home/yang/sources/models/slim/data/mnist_train.tfrecord",
                      os.path.join(FIX, "mnist_train.tfrecord"))
    (tmp_path / "model.pbtxt").write_text(src)
    recs = TL.get_data(str(tmp_path), "LeNet/Flatten/Reshape", "fifo_queue_Dequeue:1", 32, "model.pbtxt")
    assert len(recs) == 10 and recs[0].feature().shape == (3136,)
    assert all(1 <= float(r.label()) <= 10 for r in recs)
    model = TL.main(["-t", str(tmp_path), "-v", str(tmp_path), "--graphFile", "model.pbtxt",
                     "--featureNode", "LeNet/Flatten/Reshape", "--labelNode", "fifo_queue_Dequeue:1",
                     "--featureSize", "3136", "--classNum", "10", "--graphBatch", "32", "-b", "5", "-e", "2"])
    assert model.forward(torch.stack([r.feature() for r in recs[:3]])).shape == (3, 10)


def _images(d, n=10):
    from PIL import Image
    rng = np.random.default_rng(0)
    os.makedirs(d, exist_ok=True)
    for i in range(n):
        arr = (rng.random((40, 48, 3)) * 120).astype(np.uint8)
        if i % 2 == 0:
            arr[..., 0] = 250
        Image.fromarray(arr).save(os.path.join(d, ("cat" if i % 2 == 0 else "dog") + f"_{i}.jpg"))


def test_dlframes_image_inference_and_transfer_learning(tmp_path):
    from bigdl.example import dlframes as E
    from bigdl.nn import Linear, ReLU, Reshape, Sequential, SoftMax, SpatialAveragePooling, SpatialConvolution
    from bigdl.serialization.caffe_persister import save_caffe
    img = str(tmp_path / "img")
    _images(img)
    torch.manual_seed(0)
    m = (Sequential().add(SpatialConvolution(3, 8, 3, 3, 2, 2)).add(ReLU())
         .add(SpatialAveragePooling(15, 15, 15, 15)).add(Reshape([8])).add(Linear(8, 20)).add(SoftMax()))
    proto, weights = str(tmp_path / "deploy.prototxt"), str(tmp_path / "m.caffemodel")
    save_caffe(m, proto, weights, overwrite=True)
    common = ["--caffeDefPath", proto, "--modelPath", weights, "--folder", img, "--imageSize", "32", "--resize", "36",
              "-b", "4"]
    out = E.main(["inference"] + common)
    assert len(out) == 10 and set(out["prediction"]) <= set(float(c) for c in range(1, 21))
    pred, score = E.main(["transfer"] + common + ["--featureSize", "20", "--maxEpoch", "3"])
    assert len(pred) > 0 and 0.0 <= score <= 1.0


def test_int8_generate_scales_then_quantized_inference(tmp_path):
    from bigdl.dataset.seqfile import BGRImgToLocalSeqFile
    from bigdl.example import int8 as E
    from bigdl.models.resnet import ResNet, DatasetType, model_init
    from bigdl.nn.module import Module
    from bigdl.utils.random import RNG
    rng = np.random.default_rng(0)
    (tmp_path / "val").mkdir()
    items = []
    for i in range(16):
        lab = i % 4 + 1
        img = (rng.random((40, 40, 3)) * 60).astype(np.uint8)
        img[:, :, lab % 3] += 150
        items.append((img, lab))
    BGRImgToLocalSeqFile(10, str(tmp_path / "val" / "part"))(items)
    RNG.setSeed(1)
    m = model_init(ResNet(4, depth=18, dataset=DatasetType.ImageNet, image_size=32))
    m.evaluate()
    path = str(tmp_path / "r18.bigdl")
    m.saveModule(path, over_write=True)
    q = E.main(["genscales", "-f", str(tmp_path), "-m", path, "-b", "8", "--imageSize", "32"])
    assert q.endswith(".quantized.bigdl") and os.path.exists(q)
    loaded = Module.loadModule(q)
    assert any(getattr(x, "hasInt8Scales", lambda: False)() for x in loaded.flattened_modules())
    res = E.main(["inference", "-f", str(tmp_path), "-m", q, "-b", "8", "--imageSize", "32"])
    assert res[0][0].result()[1] == 16
    # the int8 model agrees with the float one on these inputs
    batches = E.val_batches(str(tmp_path), 32, 16)
    x = batches[0].getInput()
    fl = loaded.forward(x).argmax(1)
    qm = loaded.quantize()
    assert float((qm.forward(x).argmax(1) == fl).float().mean()) >= 0.75


def _sst(d):
    random.seed(0)
    words = ["good", "bad", "movie", "great", "awful", "plot", "fun", "boring", "the", "a"]
    pos, neg = {"good", "great", "fun"}, {"bad", "awful", "boring"}
    os.makedirs(os.path.join(d, "glove"), exist_ok=True)
    with open(os.path.join(d, "glove", "g.txt"), "w") as f:
        for w in words[:-1]:
            f.write(w + " " + " ".join(f"{random.uniform(-1, 1):.4f}" for _ in range(8)) + "\n")
    os.makedirs(os.path.join(d, "sst"), exist_ok=True)
    with open(os.path.join(d, "sst", "vocab-cased.txt"), "w") as f:
        f.write("\n".join(words) + "\n")

    def sent():
        n = random.randint(2, 5)
        ws = [random.choice(words) for _ in range(n)]
        root = max(-2, min(2, sum(w in pos for w in ws) - sum(w in neg for w in ws)))
        parents = [n + 1 if i <= 2 else n + i - 1 for i in range(1, n + 1)]
        parents += [k + 1 if k < 2 * n - 1 else 0 for k in range(n + 1, 2 * n)]
        return ws, parents, [0] * (2 * n - 2) + [root]
    for split, N in (("train", 40), ("dev", 12)):
        S = [sent() for _ in range(N)]
        sd = os.path.join(d, "sst", split)
        os.makedirs(sd, exist_ok=True)
        open(os.path.join(sd, "sents.txt"), "w").write("\n".join(" ".join(s[0]) for s in S) + "\n")
        open(os.path.join(sd, "parents.txt"), "w").write("\n".join(" ".join(map(str, s[1])) for s in S) + "\n")
        open(os.path.join(sd, "labels.txt"), "w").write("\n".join(" ".join(map(str, s[2])) for s in S) + "\n")


def test_tree_lstm_sentiment_example(tmp_path):
    from bigdl.example import treeLSTMSentiment as E
    from bigdl.nn.layers.tree_lstm import TensorTree
    # "a b c" with ((a b) c): SST parents [4 4 5 5 0] → node 1 = root, node k+1 = SST node k
    t = TensorTree(E.read_tree([4, 4, 5, 5, 0]))
    assert t.getRoot() == 1 and sorted(c for c in t.children(1) if c > 0) == [4, 5]
    assert [t.leafIndex(i) for i in (2, 3, 4)] == [1, 2, 3]
    assert E.rotate([1, 2, 3, 9], 1) == [9, 1, 2, 3]
    d = str(tmp_path)
    _sst(d)
    model = E.main(["-b", d, "--glove", "glove/g.txt", "-i", "8", "-h", "16", "-e", "2", "-p", "0.0", "-l", "0.1"])
    assert model is not None


def _ptb(d):
    rng = random.Random(0)
    words = [f"w{i}" for i in range(40)]
    for split, n in (("train", 120), ("valid", 30), ("test", 30)):
        with open(os.path.join(d, f"ptb.{split}.txt"), "w") as f:
            for _ in range(n):
                f.write(" " + " ".join(rng.choice(words[:25] if split == "train" else words) for _ in range(8)) + " \n")


def test_languagemodel_ptbwordlm_example(tmp_path):
    from bigdl.example import languagemodel as E
    d = str(tmp_path)
    _ptb(d)
    train, valid, test, dic = E.sequence_preprocess(d, 20)
    assert dic.get_vocab_size() == 19 and min(train) >= 1.0 and max(train) <= 20.0
    assert E.reader([1.0, 2.0, 3.0, 4.0, 5.0, 6.0], 2) == [[1.0, 2.0, 3.0], [3.0, 4.0, 5.0]]
    mb = next(iter(E.to_dataset(train, 5, 4).data(train=False)))
    x, y = mb.getInput(), mb.getTarget()
    assert x.shape == (4, 5) and torch.equal(x[0, 1:], y[0, :-1])  # next-word targets, ids unchanged
    model, loss = E.main(["-f", d, "-b", "4", "--vocab", "20", "-h", "16", "--numLayers", "1", "--numSteps", "5",
                          "-e", "1", "--test"])
    assert model is not None and 0 < loss < 1e4


def _val_seq(d, n=12, size=40):
    from bigdl.dataset.seqfile import BGRImgToLocalSeqFile
    rng = np.random.default_rng(3)
    items = []
    for i in range(n):
        img = (rng.random((size, size, 3)) * 200).astype(np.uint8)
        items.append((img, i % 5 + 1))
    os.makedirs(os.path.join(d, "val"), exist_ok=True)
    BGRImgToLocalSeqFile(6, os.path.join(d, "val", "part"))(items)


def test_loadmodel_example_models_and_validator(tmp_path):
    from bigdl.example import loadmodel as L
    from bigdl.nn import Linear, LogSoftMax, Reshape, Sequential, SpatialAveragePooling, SpatialConvolution
    from bigdl.serialization.caffe_persister import save_caffe
    for f, s in ((L.AlexNet_OWT, 224), (L.AlexNet_OWT_graph, 224), (L.AlexNet, 227)):
        m = f(7)
        m.evaluate()
        assert m.forward(torch.randn(2, 3, s, s)).shape == (2, 7)
    d = str(tmp_path)
    _val_seq(d)
    # bigdl vgg16 / resnet paths with a small 224-input network
    net = (Sequential().add(SpatialConvolution(3, 8, 3, 3, 2, 2)).add(SpatialAveragePooling(111, 111, 111, 111))
           .add(Reshape([8])).add(Linear(8, 1000)).add(LogSoftMax()))
    mp = str(tmp_path / "m.bigdl")
    net.saveModule(mp, over_write=True)
    for name in ("vgg16", "resnet"):
        res = L.main(["-t", "bigdl", "-m", name, "-f", d, "--modelPath", mp, "-b", "4"])
        assert res[0][0].result()[1] == 12
    # caffe alexnet path: mean file of 256·256·3 pixel means, 227 crop
    cnet = (Sequential().add(SpatialConvolution(3, 4, 3, 3, 2, 2)).add(SpatialAveragePooling(113, 113, 113, 113))
            .add(Reshape([4])).add(Linear(4, 1000)).add(LogSoftMax()))
    proto, weights = str(tmp_path / "a.prototxt"), str(tmp_path / "a.caffemodel")
    save_caffe(cnet, proto, weights, overwrite=True)
    mean = tmp_path / "mean.txt"
    mean.write_text("\n".join(["100.0"] * (256 * 256 * 3)) + "\n")
    res = L.main(["-t", "caffe", "-m", "alexnet", "-f", d, "--caffeDefPath", proto, "--modelPath", weights,
                  "--meanFile", str(mean), "-b", "5"])
    assert res[0][0].result()[1] == 12
