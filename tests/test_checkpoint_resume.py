"""Checkpoint consistency and OptimMethod matching on resume (CPU).

* A crash between the model file and the state file of a checkpoint must not mix checkpoints: the
  newest complete ``state<sfx>`` fixes the suffix of the model / optimMethod files that are loaded.
* Several OptimMethods keyed by default module names (``get_name`` carries a per-process postfix,
  like the reference's) are matched on resume by the arena slice each owns, not by sorted key
  position; an unmatched method raises instead of receiving another method's state."""
import os

import pytest
import torch


def _opt(tmp_path, names=("a", "b")):
    from bigdl.nn import Sequential, Linear, ReLU, LogSoftMax, ClassNLLCriterion
    from bigdl.optim import SGD, Adam
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.utils.engine import Engine
    Engine.init(device="cpu")
    torch.manual_seed(0)
    l1, l2 = Linear(6, 8), Linear(8, 3)
    l1.setName(names[0])
    l2.setName(names[1])
    m = Sequential().add(l1).add(ReLU()).add(l2).add(LogSoftMax())
    x = torch.randn(5, 6)
    y = (torch.randint(0, 3, (5,)) + 1).float()
    opt = LocalOptimizer(m, [MiniBatch(x, y)], ClassNLLCriterion())
    opt.setOptimMethods({names[0]: SGD(learningrate=0.1, momentum=0.9), names[1]: Adam(learningrate=0.01)})
    opt.setCheckpoint(str(tmp_path), None, is_overwrite=False)
    opt.prepare()
    return opt, MiniBatch(x, y)


def test_resume_matches_methods_by_arena_slice_not_key(tmp_path, monkeypatch):
    monkeypatch.setenv("BIGDL_CKPT_FLAT", "1")
    opt, b = _opt(tmp_path, ("layerA_123", "layerB_456"))
    for _ in range(3):
        opt.train_step(b)
    opt.state["neval"] = 4
    opt.checkpoint()
    sgd_buf = opt.optim_methods["layerA_123"].state["dfdx"].clone()
    adam_s = opt.optim_methods["layerB_456"].state["s"].clone()
    # a "restarted process": same layers, different default-name postfixes, and keys whose sorted
    # order is reversed relative to the checkpoint's
    opt2, b2 = _opt(tmp_path, ("zzz_layerA", "aaa_layerB"))
    opt2._restore_latest()
    torch.testing.assert_close(opt2.optim_methods["zzz_layerA"].state["dfdx"], sgd_buf)
    torch.testing.assert_close(opt2.optim_methods["aaa_layerB"].state["s"], adam_s)


def test_unmatched_method_raises(tmp_path, monkeypatch):
    monkeypatch.setenv("BIGDL_CKPT_FLAT", "1")
    opt, b = _opt(tmp_path, ("x1", "x2"))
    opt.train_step(b)
    opt.state["neval"] = 2
    opt.checkpoint()
    opt2, _ = _opt(tmp_path, ("y1", "y2"))
    opt2._method_slices = {"y1": (0, 1), "y2": (1, 10 ** 6)}  # layout no longer matches
    with pytest.raises(ValueError, match="matches no live OptimMethod"):
        opt2._restore_latest()


def test_torn_checkpoint_loads_complete_set(tmp_path):
    """model.3 exists but its state file was never written (crash mid-write): the loader takes
    checkpoint 2 as a whole."""
    from bigdl.serialization.checkpoint import save_checkpoint, load_latest_checkpoint
    from bigdl.nn import Linear
    from bigdl.optim import SGD
    m = Linear(3, 2)
    sgd = SGD(learningrate=0.1, momentum=0.9)
    for n in (2, 3):
        m.weight.fill_(float(n))
        sgd.state["dfdx"] = torch.full((8,), float(n))
        save_checkpoint(str(tmp_path), m, {"sgd": sgd}, {"neval": n + 1, "epoch": 1})
    os.remove(tmp_path / "state.3")
    # make the torn model/optimizer files the newest by mtime, as an interrupted write would
    for f in ("model.3", "optimMethod-sgd.3"):
        os.utime(tmp_path / f, None)
    model, methods, state = load_latest_checkpoint(str(tmp_path))
    assert state["neval"] == 3
    assert float(model.weight.flatten()[0]) == 2.0
    assert float(methods["sgd"].state["dfdx"][0]) == 2.0


def test_sharded_checkpoint_missing_shard_falls_back(tmp_path, monkeypatch):
    """A crash after rank 0's state file but before another rank's ``.rank<r>`` shard landed: every
    rank must resume from the previous COMPLETE checkpoint (not raise, and not disagree on which)."""
    from bigdl.serialization.checkpoint import save_checkpoint, save_shard_state, load_latest_checkpoint
    from bigdl.nn import Linear
    from bigdl.optim import SGD
    m = Linear(3, 2)
    sgd = SGD(learningrate=0.1, momentum=0.9)
    slices = {"sgd": (0, 8)}
    for n in (2, 3):
        m.weight.fill_(float(n))
        for r in range(2):
            sgd.state["dfdx"] = torch.full((4,), float(10 * n + r))
            save_shard_state(str(tmp_path), {"sgd": sgd}, {"neval": n + 1}, rank=r, slices=slices)
        save_checkpoint(str(tmp_path), m, {"sgd": sgd}, {"neval": n + 1, "epoch": 1}, world_size=2, sharded=True,
                        slices=slices)
    os.remove(tmp_path / "optimMethod-@0.3.rank1")
    for rank in (0, 1):
        monkeypatch.setenv("RANK", str(rank))
        model, methods, state = load_latest_checkpoint(str(tmp_path), world_size=2, sharded=True)
        assert state["neval"] == 3
        assert float(model.weight.flatten()[0]) == 2.0
        assert float(methods["sgd"].state["dfdx"][0]) == 20.0 + rank
