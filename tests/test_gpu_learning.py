"""The native GPU training path learns (not only "runs"): VGG-CIFAR, ResNet-20 and the PTB LSTM
reduce their loss on a learnable synthetic task and classify it above chance — on the bf16 HIP
kernels with zero torch fallbacks."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True)
def _deterministic():
    """Bit-reproducible kernels (no split-K float atomics): with them these short, high-learning-rate
    runs are chaotic — the same seed gave VGG-CIFAR eval accuracies from 0.12 to 0.64 across runs
    (tools/vgg_flaky.py) — and a learning check must not depend on the reduction order."""
    from bigdl.utils import config
    prev = config.get_property("bigdl.deterministic")
    config.set_property("bigdl.deterministic", True)
    yield
    config.set_property("bigdl.deterministic", prev)


def _setup():
    from bigdl.utils.engine import Engine
    from bigdl.ops import native
    Engine.init(device="cuda:0")
    native.reset_fallbacks()


def _images(n, classes=10, seed=0):
    from bigdl.models.train.common import synthetic_images
    imgs, labels = synthetic_images(n, 32, 32, 3, classes, seed)
    x = torch.from_numpy(imgs).float().permute(0, 3, 1, 2).div(255.0).sub(0.5).div(0.25)
    return x, torch.from_numpy(labels)


def _train(model, crit, method, batches, epochs):
    from bigdl.dataset import MiniBatch
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.utils.engine import Engine
    dt = Engine.compute_dtype()
    mbs = [MiniBatch(x.to(dev).to(dt).contiguous(memory_format=torch.channels_last) if x.dim() == 4
                     else x.to(dev), y.to(dev)) for x, y in batches]
    opt = LocalOptimizer(model, mbs, crit, method, batch_size=mbs[0].size())
    opt.prepare()
    losses = []
    for _ in range(epochs):
        for b in mbs:
            losses.append(float(opt.train_step(b)))
    torch.cuda.synchronize()
    return losses, mbs


def _accuracy(model, mbs):
    model.evaluate()
    correct = total = 0
    with torch.no_grad():
        for b in mbs:
            out = model.forward(b.getInput()).float()
            correct += int((out.argmax(1) + 1 == b.getTarget().long()).sum())
            total += b.size()
    model.training()
    return correct / total


def _assert_learns(losses, acc, chance):
    from bigdl import ops
    first, last = np.mean(losses[:4]), np.mean(losses[-4:])
    # (float-atomic reduction order varies run to run: margins sized for that spread)
    assert last < 0.65 * first, (first, last)
    assert acc > 2.5 * chance, acc
    assert ops.fallback_counts() == {}, ops.fallback_counts()


def test_vgg_cifar_learns_on_gpu():
    _setup()
    from bigdl.models.vgg import VggForCifar10
    from bigdl.nn import ClassNLLCriterion
    from bigdl.optim import SGD
    torch.manual_seed(0)
    x, y = _images(512)
    batches = [(x[i:i + 64], y[i:i + 64]) for i in range(0, 512, 64)]
    model = VggForCifar10(10).to(device=dev)
    losses, mbs = _train(model, ClassNLLCriterion(), SGD(learningrate=0.02, momentum=0.9, dampening=0.0), batches, 20)
    _assert_learns(losses, _accuracy(model, mbs), 0.1)


def test_resnet20_learns_on_gpu():
    _setup()
    from bigdl.models.resnet import ResNet, model_init
    from bigdl.nn import CrossEntropyCriterion
    from bigdl.optim import SGD
    torch.manual_seed(0)
    x, y = _images(512, seed=1)
    batches = [(x[i:i + 64], y[i:i + 64]) for i in range(0, 512, 64)]
    model = ResNet(10, depth=20)
    model_init(model)
    model = model.to(device=dev)
    losses, mbs = _train(model, CrossEntropyCriterion(), SGD(learningrate=0.05, momentum=0.9, dampening=0.0),
                         batches, 16)
    _assert_learns(losses, _accuracy(model, mbs), 0.1)


def test_ptb_lstm_learns_on_gpu():
    """The 2-layer LSTM language model memorises a periodic token stream."""
    _setup()
    from bigdl.models.rnn import PTBModel
    from bigdl.nn import TimeDistributedCriterion, CrossEntropyCriterion
    from bigdl.optim import Adagrad
    torch.manual_seed(0)
    vocab, T, B = 50, 20, 20
    stream = (np.arange(T * B * 8 + 1) * 7 % vocab) + 1
    batches = []
    for k in range(8):
        seg = stream[k * T * B:(k + 1) * T * B + 1]
        xs = torch.tensor(seg[:-1].reshape(B, T), dtype=torch.float32)
        ys = torch.tensor(seg[1:].reshape(B, T), dtype=torch.float32)
        batches.append((xs, ys))
    model = PTBModel.lstm(vocab, 64, vocab, 2).to(device=dev)
    crit = TimeDistributedCriterion(CrossEntropyCriterion(), size_average=True)
    losses, mbs = _train(model, crit, Adagrad(learningrate=0.5), batches, 10)
    first, last = np.mean(losses[:4]), np.mean(losses[-4:])
    assert last < 0.3 * first, (first, last)
    from bigdl import ops
    assert ops.fallback_counts() == {}, ops.fallback_counts()
