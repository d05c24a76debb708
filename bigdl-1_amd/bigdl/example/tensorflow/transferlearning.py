"""Transfer learning on features computed by a TensorFlow graph
(``DL/example/tensorflow/transferlearning/TransferLearning.scala``).

The TF graph (``model.pb`` + variables ``model.bin``, e.g. dumped by the reference's
``dump_model_example.py`` from a slim InceptionV1 with its input pipeline) is opened as a session
(``TensorflowLoader.checkpoints``); ``getRDD([featureNode, labelNode])`` runs the graph's own input
pipeline through it and yields one (feature, one-hot label) record per example; a BigDL
``Squeeze → Linear(featureSize, classNum)`` head is trained on those with CrossEntropy and
RMSprop(lr 0.001, decay 0.9), validated with Top-1 every epoch when a validation model is given.

    python -m bigdl.example.tensorflow.transferlearning -t <training model dir> [-v <validation dir>]
        [-b 16] [-e 10] [--featureNode InceptionV1/Logits/AvgPool_0a_7x7/AvgPool]
        [--labelNode OneHotEncoding/one_hot] [--featureSize 1024] [--classNum 5]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch


def get_data(model_dir: str, feature_node: str, label_node: str, graph_batch=None, graph_file="model.pb",
             bin_file="model.bin"):
    """[Sample(feature, 1-based class)] from the graph's pipeline (``getData``)."""
    from ...dataset.core import Sample
    from ...utils.tf.loader import TensorflowLoader
    g = os.path.join(model_dir, graph_file)
    b = os.path.join(model_dir, bin_file)
    if os.path.exists(b):
        sess = TensorflowLoader.checkpoints(g, b)
    else:
        from ...utils.tf.session import Session
        sess = Session(TensorflowLoader.parse(g))
    recs = sess.getRDD([feature_node, label_node], batch_size=graph_batch)
    out = []
    for t in recs:
        feature = torch.as_tensor(t[1]).float()
        label = float(torch.as_tensor(t[2]).float().reshape(-1).argmax()) + 1.0
        out.append(Sample(feature, torch.tensor([label])))
    return out


def build_model(feature_size: int, class_num: int):
    from ...nn import Linear, Sequential, Squeeze
    return Sequential().add(Squeeze(None, batch_mode=True)).add(Linear(feature_size, class_num))


def main(argv=None):
    ap = argparse.ArgumentParser(description="BigDL TensorFlow transfer learning example")
    ap.add_argument("-t", "--trainingModelDir", required=True)
    ap.add_argument("-v", "--validationModelDir", default=None)
    ap.add_argument("-b", "--batchSize", type=int, default=16)
    ap.add_argument("-e", "--nEpochs", type=int, default=10)
    ap.add_argument("--featureNode", default="InceptionV1/Logits/AvgPool_0a_7x7/AvgPool")
    ap.add_argument("--labelNode", default="OneHotEncoding/one_hot")
    ap.add_argument("--featureSize", type=int, default=1024)
    ap.add_argument("--classNum", type=int, default=5)
    ap.add_argument("--graphBatch", type=int, default=None, help="batch the TF graph runs at (fixed-shape graphs)")
    ap.add_argument("--graphFile", default="model.pb")
    a = ap.parse_args(argv)
    from ...dataset.core import DataSet, SampleToMiniBatch
    from ...nn import CrossEntropyCriterion
    from ...optim import RMSprop
    from ...optim.optimizer import Optimizer
    from ...optim.trigger import Trigger
    from ...optim.validation import Top1Accuracy
    from ...utils.engine import Engine
    Engine.init()
    train = get_data(a.trainingModelDir, a.featureNode, a.labelNode, a.graphBatch, a.graphFile)
    model = build_model(a.featureSize, a.classNum)
    opt = Optimizer(model, DataSet.array(train) >> SampleToMiniBatch(a.batchSize), CrossEntropyCriterion(),
                    batch_size=a.batchSize)
    opt.setEndWhen(Trigger.maxEpoch(a.nEpochs))
    opt.setOptimMethod(RMSprop(learningrate=0.001, decayrate=0.9))
    if a.validationModelDir:
        val = get_data(a.validationModelDir, a.featureNode, a.labelNode, a.graphBatch, a.graphFile)
        opt.setValidation(Trigger.everyEpoch(), DataSet.array(val) >> SampleToMiniBatch(a.batchSize), [Top1Accuracy()],
                          a.batchSize)
    return opt.optimize()


if __name__ == "__main__":
    main(sys.argv[1:])
