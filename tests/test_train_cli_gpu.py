"""The training entry points on the GPU path: native C++ loader → pinned H2D → bf16 HIP kernels,
checkpoint and validation, with zero torch fallbacks (reference models/*/Train.scala,
models/resnet/TrainImageNet.scala)."""
import pytest

pytestmark = pytest.mark.gpu


def _clean():
    from bigdl import ops
    assert ops.fallback_counts() == {}, ops.fallback_counts()


def test_imagenet_resnet50_cli_on_gpu(tmp_path):
    from bigdl import ops
    from bigdl.models.train import imagenet
    ops.reset_fallbacks()
    out = imagenet.main(["--synthetic", "256", "-b", "64", "-e", "1", "--maxIteration", "3", "--depth", "50",
                         "--classes", "1000", "--imageSize", "224", "--warmupEpoch", "1", "--maxLr", "0.4",
                         "--threads", "4", "--checkpoint", str(tmp_path / "ck")])
    assert out["neval"] == 4
    _clean()


def test_cifar_vgg_cli_on_gpu():
    from bigdl import ops
    from bigdl.models.train import cifar
    ops.reset_fallbacks()
    out = cifar.main(["--synthetic", "512", "-b", "128", "-e", "1", "--maxIteration", "4", "--net", "vgg",
                      "--threads", "4"])
    assert out["neval"] == 5
    _clean()


def test_lenet_cli_on_gpu(tmp_path):
    from bigdl import ops
    from bigdl.models.train import lenet
    ops.reset_fallbacks()
    out = lenet.main(["--synthetic", "512", "-b", "128", "-e", "1", "--threads", "2",
                      "--checkpoint", str(tmp_path / "ck")])
    assert out["neval"] == 5
    _clean()
