"""Observability + inference drivers: TrainSummary/ValidationSummary event files, LocalPredictor,
Evaluator/Validator, PredictionService (bytes protocol of PredictionService.scala:184-281)."""
import numpy as np
import torch

from bigdl.dataset import Sample
from bigdl.nn import Sequential, Linear, LogSoftMax, ReLU, ClassNLLCriterion
from bigdl.optim import SGD
from bigdl.optim.evaluator import Evaluator, Validator
from bigdl.optim.optimizer import LocalOptimizer
from bigdl.optim.predictor import LocalPredictor, PredictionService, serialize_activity, deserialize_activity
from bigdl.optim.trigger import MaxIteration, SeveralIteration, EveryEpoch
from bigdl.optim.validation import Top1Accuracy, Loss
from bigdl.utils.table import Table
from bigdl.visualization import TrainSummary, ValidationSummary, crc32c, read_records


def _data(n=64):
    rng = np.random.RandomState(0)
    xs = rng.randn(n, 4).astype(np.float32)
    ys = (xs[:, 0] > 0).astype(np.float32) + 1
    return [Sample(x, np.array([y], np.float32)) for x, y in zip(xs, ys)]


def _model():
    return Sequential().add(Linear(4, 8)).add(ReLU()).add(Linear(8, 2)).add(LogSoftMax())


def test_crc32c_known_vector():
    assert crc32c(b"123456789") == 0xE3069283


def test_train_and_validation_summary(tmp_path):
    data = _data()
    opt = LocalOptimizer(_model(), data, ClassNLLCriterion(), SGD(learningrate=0.1), end_trigger=MaxIteration(6),
                         batch_size=16)
    ts = TrainSummary(str(tmp_path), "app")
    ts.set_summary_trigger("Parameters", SeveralIteration(3))
    vs = ValidationSummary(str(tmp_path), "app")
    opt.setTrainSummary(ts)
    opt.setValidationSummary(vs)
    opt.setValidation(SeveralIteration(2), data, [Top1Accuracy()], 16)
    opt.optimize()
    loss = ts.read_scalar("Loss")
    assert [s for s, _, _ in loss] == list(range(1, 7))
    assert all(np.isfinite(v) for _, v, _ in loss)
    assert len(ts.read_scalar("Throughput")) == 6
    assert len(ts.read_scalar("LearningRate")) == 6
    acc = vs.read_scalar("Top1Accuracy")
    assert len(acc) == 3 and all(0 <= v <= 1 for _, v, _ in acc)
    ts.close()
    vs.close()
    files = [p for p in (tmp_path / "app" / "train").iterdir()]
    assert files and sum(1 for _ in read_records(str(files[0]))) > 6  # crc-checked read


def test_local_predictor_and_evaluator():
    m = _model()
    data = _data(20)
    out = LocalPredictor(m, batch_size=8).predict(data)
    assert len(out) == 20 and out[0].shape == (2,)
    cls = m.predict_class(data)
    assert cls.shape == (20,) and set(cls.tolist()) <= {1, 2}
    ref = m.forward(torch.stack([s.feature() for s in data])).argmax(1) + 1
    assert cls.tolist() == ref.tolist()
    res = Evaluator(m).test(data, [Top1Accuracy(), Loss()], 8)
    assert res[0][0].result()[1] == 20
    res2 = Validator(m, data).test([Top1Accuracy()])
    assert res2[0][0].result()[0] == res[0][0].result()[0]
    r3 = m.evaluate(data, [Top1Accuracy()], 5)
    assert r3[0][0].result()[0] == res[0][0].result()[0]


def test_prediction_service_bytes_and_errors():
    m = _model()
    ps = PredictionService(m, 3)
    x = torch.randn(5, 4)
    y = deserialize_activity(ps.predict(serialize_activity(x)))
    torch.testing.assert_close(y, m.forward(x))
    assert isinstance(ps.predict(torch.randn(2, 4)), torch.Tensor)
    err = deserialize_activity(ps.predict(serialize_activity(torch.randn(2, 7))))
    assert isinstance(err, str) and "running forward" in err
    bad = deserialize_activity(ps.predict(b"\xff\xff\xff"))
    assert isinstance(bad, str) and "DeSerialize" in bad
    t = Table()
    t[1] = torch.arange(6.0).reshape(2, 3)
    t[2] = torch.tensor([1, 2, 3])
    t2 = deserialize_activity(serialize_activity(t))
    torch.testing.assert_close(t2[1], t[1])
    assert t2[2].tolist() == [1, 2, 3]


def test_prediction_service_concurrent():
    import threading
    m = _model()
    ps = PredictionService(m, 2)
    xs = [torch.randn(3, 4) for _ in range(8)]
    outs = [None] * 8

    def work(i):
        outs[i] = ps.predict(xs[i])
    th = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for x, o in zip(xs, outs):
        torch.testing.assert_close(o, m.forward(x))


def test_convert_model_cli_roundtrips(tmp_path):
    """``ConvertModel`` CLI: bigdl → caffe → bigdl (+quantize) → torch, outputs preserved."""
    import torch
    from bigdl.nn import Sequential, SpatialConvolution, ReLU, SpatialMaxPooling, View, Linear
    from bigdl.nn.module import Module
    from bigdl.utils.convert_model import main
    torch.manual_seed(0)
    m = (Sequential().add(SpatialConvolution(3, 8, 3, 3)).add(ReLU()).add(SpatialMaxPooling(2, 2, 2, 2))
         .add(View(8 * 3 * 3)).add(Linear(72, 5)))
    m.evaluate()
    x = torch.randn(2, 3, 8, 8)
    ref = m.forward(x).clone()
    src = str(tmp_path / "m.bigdl")
    m.saveModule(src, over_write=True)
    cm = str(tmp_path / "m.caffemodel")
    assert main(["--from", "bigdl", "--to", "caffe", "--input", src, "--output", cm]) == 0
    back = str(tmp_path / "back.bigdl")
    assert main(["--from", "caffe", "--to", "bigdl", "--prototxt", str(tmp_path / "m.prototxt"), "--input", cm,
                 "--output", back]) == 0
    m2 = Module.loadModule(back)
    m2.evaluate()
    torch.testing.assert_close(m2.forward(x), ref, rtol=1e-5, atol=1e-5)
    t7 = str(tmp_path / "m.t7")
    assert main(["--from", "bigdl", "--to", "torch", "--input", back, "--output", t7]) == 0
    m3 = Module.loadTorch(t7)
    m3.evaluate()
    torch.testing.assert_close(m3.forward(x), ref, rtol=1e-5, atol=1e-5)
    q = str(tmp_path / "q.bigdl")
    assert main(["--from", "bigdl", "--to", "bigdl", "--input", src, "--output", q, "--quantize", "true"]) == 0
    mq = Module.loadModule(q)
    mq.evaluate()
    assert (mq.forward(x) - ref).abs().max() < 0.1


def test_precision_recall_auc_and_evaluate_methods():
    import torch
    from bigdl.optim import PrecisionRecallAUC, EvaluateMethods
    # perfect ranking → AUC 1; reference PRAUCResult semantics (trapezoids from (0, 1))
    r = PrecisionRecallAUC()(torch.tensor([0.9, 0.8, 0.3, 0.1]), torch.tensor([1.0, 1.0, 0.0, 0.0]))
    assert abs(r.result()[0] - 1.0) < 1e-6 and r.result()[1] == 4
    r2 = PrecisionRecallAUC()(torch.tensor([0.9, 0.8, 0.3]), torch.tensor([0.0, 1.0, 1.0]))
    # steps: (P=0, R=0) → (1/2, 1/2) → (2/3, 1): 0.5·(0 + 1)/2 ... computed by hand:
    # i1 neg: p=0, r=0 → area += 0; i2 pos: p=.5, r=.5 → += .5·(.5+0); i3 pos: p=2/3, r=1 → += .5·(2/3+.5)
    exp = (0.5 * 0.5 + 0.5 * (2 / 3 + 0.5)) / 2
    assert abs(r2.result()[0] - exp) < 1e-6
    merged = r + r2
    assert merged.result()[1] == 7
    out = torch.tensor([[0.1, 0.7, 0.2], [0.5, 0.2, 0.3]])
    assert EvaluateMethods.calcAccuracy(out, torch.tensor([2.0, 3.0])) == (1, 2)
    assert EvaluateMethods.calcTop5Accuracy(out, torch.tensor([2.0, 3.0])) == (2, 2)


def test_retry_from_checkpoint_after_injected_fault(tmp_path):
    """an injected failure mid-training is retried from the latest checkpoint
    (``DistriOptimizer.scala:881-963`` retry loop; fault injection = ``ExceptionTest``)."""
    import torch
    from bigdl.nn import Sequential, Linear, ReLU, LogSoftMax, ClassNLLCriterion, FaultInject
    from bigdl.optim import SGD, MaxIteration, SeveralIteration
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import Sample
    FaultInject.reset("retry_test")
    torch.manual_seed(0)
    m = (Sequential().add(Linear(4, 8)).add(FaultInject(fail_at=5, key="retry_test")).add(ReLU())
         .add(Linear(8, 3)).add(LogSoftMax()))
    data = [Sample(torch.randn(4), torch.tensor(float(i % 3 + 1))) for i in range(32)]
    opt = LocalOptimizer(m, data, ClassNLLCriterion(), SGD(learningrate=0.1), MaxIteration(8), batch_size=8)
    opt.setCheckpoint(str(tmp_path), SeveralIteration(1))
    trained = opt.optimize()
    assert opt.state["neval"] >= 8
    assert FaultInject._counts["retry_test"] >= 8  # the failure happened and training went on
    assert trained is not None


def test_util_thread_pool_model_utils(tmp_path):
    import time
    import numpy as np
    from bigdl.utils.util import kthLargest
    from bigdl.utils.thread_pool import ThreadPool
    arr = [5, 1, 9, 3, 7, 7, 2]
    assert kthLargest(list(arr), 0, len(arr) - 1, 1) == 9
    assert kthLargest(list(arr), 0, len(arr) - 1, 3) == 7
    assert kthLargest(list(arr), 0, len(arr) - 1, 7) == 1
    pool = ThreadPool(4)
    assert pool.invokeAndWait([lambda i=i: i * i for i in range(5)]) == [0, 1, 4, 9, 16]
    futs = pool.invokeAndWait2([lambda: 1, lambda: time.sleep(2) or 2], timeout=0.3)
    assert futs[0].done() and futs[0].result() == 1
    assert not futs[1].done() or futs[1].cancelled()  # the straggler did not finish within the timeout
    pool.shutdown()
    # seq file generator over a tiny image folder
    from PIL import Image
    from bigdl.models.utils.seqfile_generator import main as gen
    from bigdl.dataset.seqfile import SeqFileFolder
    for c in ("cat", "dog"):
        (tmp_path / "img" / c).mkdir(parents=True)
        Image.fromarray(np.full((6, 9, 3), 100, np.uint8)).save(tmp_path / "img" / c / "a.png")
    assert gen(["-f", str(tmp_path / "img"), "-o", str(tmp_path / "seq"), "-b", "1", "-r", "4", "--hasName"]) == 0
    recs = list(SeqFileFolder.read(str(tmp_path / "seq")))
    assert [r[1] for r in recs] == [1.0, 2.0] and recs[0][0].shape == (4, 6, 3) and recs[0][2] == "a.png"


def test_perf_harness_runs_cpu(capsys):
    from bigdl.models.utils.perf import main
    assert main(["--model", "lenet5", "--batch", "8", "--iteration", "2", "--warmup", "1", "--dtype", "fp32"]) == 0
    assert "records/second" in capsys.readouterr().out


def test_async_checkpoint_matches_sync_and_is_atomic(tmp_path):
    """trigger-driven checkpoints snapshot on the training thread and serialise/write on
    the writer thread; the files equal a synchronous save, temp files are never picked up as the
    latest checkpoint, and writer errors surface on the next wait."""
    import os
    import pytest
    import torch
    from bigdl.nn import Sequential, Linear, ReLU
    from bigdl.optim import SGD
    from bigdl.serialization import checkpoint as ck
    torch.manual_seed(0)
    m = Sequential().add(Linear(16, 32)).add(ReLU()).add(Linear(32, 4))
    sgd = SGD(learningrate=0.1, momentum=0.9)
    sgd.state["buf"] = torch.randn(100)
    state = {"epoch": 1, "neval": 3, "Loss": 0.5}
    a, b = str(tmp_path / "sync"), str(tmp_path / "async")
    ck.save_checkpoint(a, m, {"sgd": sgd}, state)
    ck.save_checkpoint(b, m, {"sgd": sgd}, state, asynchronous=True)
    # mutate right away: the async snapshot must not see it
    with torch.no_grad():
        for w in m.parameters()[0]:
            w.add_(1.0)
    ck.wait_checkpoints()
    for f in ("model.2", "optimMethod-sgd.2", "state.2"):
        assert open(os.path.join(a, f), "rb").read() == open(os.path.join(b, f), "rb").read(), f
    open(os.path.join(b, "model.9.tmp123"), "wb").write(b"partial")
    assert ck._latest(os.path.join(b, "model*")).endswith("model.2")

    def boom():
        raise IOError("disk full")
    ck._submit(boom)
    with pytest.raises(RuntimeError):
        ck.wait_checkpoints()
    ck.wait_checkpoints()  # the error is reported once
