"""The model-zoo training CLIs (reference models/*/Train.scala, Test.scala) end to end on CPU with
synthetic data: optimize → per-epoch checkpoint + validation + summaries → saved model →
Test (evaluate the saved model); and the distributed launch path (gloo, world 2)."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "bigdl-1_amd")


def test_lenet_train_checkpoint_summary_then_test(tmp_path):
    from bigdl.models.train import lenet
    ck, sm, mf = str(tmp_path / "ck"), str(tmp_path / "sum"), str(tmp_path / "lenet.bigdl")
    out = lenet.main(["--synthetic", "512", "-b", "64", "-e", "4", "--checkpoint", ck, "--summary", sm,
                      "--saveModel", mf, "--dtype", "fp32", "--threads", "2"])
    assert out["epoch"] == 5 and out["neval"] == 33
    assert glob.glob(os.path.join(ck, "*", "model.*")) and glob.glob(os.path.join(ck, "*", "optimMethod-*"))
    assert glob.glob(os.path.join(sm, "*", "train", "*tfevents*"))
    assert glob.glob(os.path.join(sm, "*", "validation", "*tfevents*"))
    res = lenet.main(["--synthetic", "512", "-b", "64", "--test", "--model", mf, "--dtype", "fp32"])
    # the synthetic classes are separable by their mean intensity: 4 epochs must beat chance (0.1) clearly
    assert res["Top1Accuracy"] > 0.25, res


def test_cifar_vgg_and_resnet_train_short():
    from bigdl.models.train import cifar
    out = cifar.main(["--synthetic", "256", "-b", "32", "-e", "1", "--maxIteration", "3", "--net", "vgg",
                      "--dtype", "fp32", "--threads", "2"])
    assert out["neval"] == 4
    out = cifar.main(["--synthetic", "256", "-b", "32", "-e", "1", "--maxIteration", "2", "--net", "resnet",
                      "--depth", "20", "--dtype", "fp32", "--threads", "2"])
    assert out["neval"] == 3


def test_imagenet_resnet_warmup_schedule_short(tmp_path):
    from bigdl.models.train import imagenet
    out = imagenet.main(["--synthetic", "32", "-b", "8", "-e", "1", "--maxIteration", "2", "--depth", "18",
                         "--classes", "10", "--imageSize", "224", "--warmupEpoch", "1", "--maxLr", "0.4",
                         "--dtype", "fp32", "--threads", "2", "--checkpoint", str(tmp_path / "ck")])
    assert out["neval"] == 3
    assert imagenet.imagenet_decay(29) == 0 and imagenet.imagenet_decay(30) == 1 and imagenet.imagenet_decay(85) == 3


def test_ptb_rnn_train_short():
    from bigdl.models.train import rnn
    out = rnn.main(["--synthetic", "4000", "-b", "4", "-e", "1", "--maxIteration", "3", "--vocabSize", "50",
                    "--hiddenSize", "16", "--numSteps", "5", "--dtype", "fp32"])
    assert out["neval"] == 4 and out["perplexity"] > 1


def test_autoencoder_train_short():
    from bigdl.models.train import autoencoder
    out = autoencoder.main(["--synthetic", "300", "-b", "50", "-e", "1", "--dtype", "fp32"])
    assert out["neval"] == 7


def test_lenet_under_launcher_gloo_world2(tmp_path):
    """python -m bigdl.launch --nproc 2 -m bigdl.models.train.lenet (CPU ranks → gloo)."""
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get("PYTHONPATH", ""), CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, "-m", "bigdl.launch", "--nproc", "2", "--no-numa-bind", "-m",
                        "bigdl.models.train.lenet", "--synthetic", "256", "-b", "64", "-e", "1", "--dtype", "fp32",
                        "--threads", "1"], env=env, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "DistriOptimizer: world=2" in r.stdout + r.stderr
