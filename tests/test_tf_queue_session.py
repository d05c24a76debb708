"""TensorFlow queue-fed graphs (``DL/utils/tf/Session.scala``; reference test
``spark/dl/src/test/scala/.../utils/tf/SessionSpec.scala:96-140``) on the reference's own fixtures
(``lenet_batch_2.pbtxt`` / ``lenet_with_batch_3.pbtxt`` + ``mnist_train.tfrecord``):

* the graph's input pipeline (file-name queue → 4 TFRecord readers → shuffle queue → ParseExample /
  decode_image cond → batch queue → one-hot → prefetch queue) yields the reference's numbers:
  10 records, Σ features = −6009.5, Σ labels = 10, per-record shapes (28, 28, 1) / (10,), also at
  batch 3 (the final partial batch is kept);
* ``train_graph`` trains the TF TRAINING graph through TF's own backward ops
  (``Conv2DBackpropInput/Filter``, ``MaxPoolGrad``, ``ReluGrad``, ``BiasAddGrad``,
  ``BroadcastGradientArgs`` …): the gradients match finite differences of the graph's loss and
  SGD drives the loss down."""
import os

import pytest
import torch

from bigdl.utils.tf.loader import TensorflowLoader
from bigdl.utils.tf.session import Session

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "tf")


def _nodes(name):
    nodes = TensorflowLoader.parse(os.path.join(FIX, name))
    for n in nodes:
        if n.name == "parallel_read/filenames/Const":
            t = n.attr["value"].tensor
            del t.string_val[:]
            t.string_val.append(os.path.join(FIX, "mnist_train.tfrecord").encode())
    return nodes


def test_input_pipeline_records_match_reference():
    recs = Session(_nodes("lenet_batch_2.pbtxt")).get_records(["fifo_queue_Dequeue"])
    assert len(recs) == 10
    assert abs(sum(float(r[1].sum()) for r in recs) - (-6009.5)) < 1e-3
    assert sum(float(r[2].sum()) for r in recs) == 10


def test_input_pipeline_arbitrary_batch_size():
    recs = Session(_nodes("lenet_with_batch_3.pbtxt")).get_records(["fifo_queue_Dequeue"])
    assert len(recs) == 10
    for r in recs:
        assert tuple(r[1].shape) == (28, 28, 1)
        assert tuple(r[2].shape) == (10,)


def test_train_tf_training_graph_gradients_and_loss():
    from bigdl.optim import SGD
    from bigdl.optim.trigger import MaxIteration
    from bigdl.utils.tf.executor import GraphExecutor
    sess = Session(_nodes("lenet_batch_2.pbtxt"))
    ex = GraphExecutor(sess.nodes, variables=sess.context, seed=0)
    ex.initialize_variables()
    recs = ex.records("fifo_queue_Dequeue")
    batch = [recs[i % len(recs)] for i in range(32)]  # the graph's reshapes bake in batch 32
    feeds = {"fifo_queue_Dequeue": (torch.stack([r[1] for r in batch]), torch.stack([r[2] for r in batch]))}
    var, grad_ref = "LeNet/fc4/biases", "gradients/LeNet/fc4/BiasAdd_grad/tuple/control_dependency_1"

    def run(refs):  # the graph has dropout (RandomUniform): same mask on every evaluation
        torch.manual_seed(123)
        return ex.run(refs, feeds=feeds)
    loss0, g = run(["total_loss", grad_ref])
    v = sess.context[var]
    for i in (0, 3, 7):
        eps = 1e-2
        v[i] += eps
        lp = float(run(["total_loss"])[0])
        v[i] -= 2 * eps
        lm = float(run(["total_loss"])[0])
        v[i] += eps
        fd = (lp - lm) / (2 * eps)
        assert abs(fd - float(g[i])) < 2e-2 * max(1.0, abs(fd)), (i, fd, float(g[i]))
    # a conv weight: its TF gradient runs through MaxPoolGrad / ReluGrad / Conv2DBackpropInput of
    # the layers above and Conv2DBackpropFilter (+ the L2 regulariser's gradient, AddN)
    (gw,) = run(["gradients/AddN_3"])
    w = sess.context["LeNet/conv1/weights"]
    for idx in ((0, 0, 0, 0), (2, 3, 0, 17)):
        eps = 2e-3  # small: ReLU / max-pool switches make the loss only piecewise smooth
        w[idx] += eps
        lp = float(run(["total_loss"])[0])
        w[idx] -= 2 * eps
        lm = float(run(["total_loss"])[0])
        w[idx] += eps
        fd = (lp - lm) / (2 * eps)
        assert abs(fd - float(gw[idx])) < 5e-2 * max(1.0, abs(fd)), (idx, fd, float(gw[idx]))
    losses = Session(_nodes("lenet_batch_2.pbtxt")).train_graph(["train_op"], SGD(learningrate=0.01),
                                                                 MaxIteration(6), batch_size=32)
    assert len(losses) == 6 and all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < 0.5 * losses[0], losses
