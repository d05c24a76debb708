"""Native C++ batch loader (``bigdl/runtime``): the reference's multi-threaded batch assembly
(``MTLabeledBGRImgToBatch``) — deterministic per (seed, batch) independent of thread count,
epoch permutations cover the data, eval mode equals a numpy center-crop/normalise oracle."""
import numpy as np
import torch

from bigdl.runtime import NativeBatchLoader


def _data(n=50, h=12, w=10, c=3):
    rng = np.random.RandomState(0)
    x = rng.randint(0, 256, size=(n, h, w, c)).astype(np.uint8)
    y = np.arange(n, dtype=np.float32) + 1
    return x, y


def test_eval_mode_matches_numpy_oracle():
    x, y = _data()
    mean, std = [10.0, 20.0, 30.0], [2.0, 4.0, 8.0]
    ld = NativeBatchLoader(x, y, 8, crop=(8, 6), pad=0, flip=False, train=False, mean=mean, std=std,
                           shuffle=False, drop_last=True, threads=3, device="cpu")
    b = ld.next_batch()
    ref = (x[:8, 2:10, 2:8, :].astype(np.float32) - np.array(mean)) / np.array(std)
    np.testing.assert_allclose(b.getInput().numpy(), ref.transpose(0, 3, 1, 2), rtol=1e-6)
    np.testing.assert_array_equal(b.getTarget().numpy(), y[:8])
    ld.close()


def test_train_mode_deterministic_across_threads_and_covers_epoch():
    x, y = _data()
    outs = []
    for t in (1, 4):
        ld = NativeBatchLoader(x, y, 10, crop=(12, 10), pad=2, flip=True, train=True, shuffle=True, seed=7,
                               threads=t, prefetch=3, device="cpu")
        assert ld.batches_per_epoch() == 5
        bs = [ld.next_batch() for _ in range(10)]
        outs.append(bs)
        labels = torch.cat([b.getTarget() for b in bs[:5]])
        assert sorted(labels.tolist()) == list(range(1, 51))  # one epoch = a permutation
        assert not torch.equal(torch.cat([b.getTarget() for b in bs[5:]]), labels)  # new epoch, new order
        ld.close()
    for a, b in zip(*outs):
        assert torch.equal(a.getInput(), b.getInput()) and torch.equal(a.getTarget(), b.getTarget())
    # every sample is a padded crop (+ optional flip) of its source image
    b0 = outs[0][0]
    for i in range(3):
        src = x[int(b0.getTarget()[i]) - 1].astype(np.float32)
        pad = np.zeros((16, 14, 3), np.float32)
        pad[2:14, 2:12] = src
        img = b0.getInput()[i].numpy().transpose(1, 2, 0)
        ok = any(np.array_equal(img, cand) for oy in range(5) for ox in range(5)
                 for cand in (pad[oy:oy + 12, ox:ox + 10], pad[oy:oy + 12, ox:ox + 10][:, ::-1]))
        assert ok


def test_bf16_nhwc_output():
    x, y = _data()
    a = NativeBatchLoader(x, y, 5, train=False, shuffle=False, dtype=torch.float32, layout="NHWC", device="cpu")
    b = NativeBatchLoader(x, y, 5, train=False, shuffle=False, dtype=torch.bfloat16, layout="NHWC", device="cpu")
    xa, xb = a.next_batch().getInput(), b.next_batch().getInput()
    assert xb.dtype == torch.bfloat16 and xa.shape == (5, 3, 12, 10)
    assert torch.equal(xa.to(torch.bfloat16), xb)
    a.close()
    b.close()


def test_loader_thread_sanitizer_stress(tmp_path):
    """The C++ loader under ThreadSanitizer and ASan/UBSan (SURVEY §5.2 race detection): 6 workers,
    3 slots, 4 epochs, each epoch a permutation — no data race or memory error reported."""
    import os
    import shutil
    import subprocess
    import pytest
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    srcs = [os.path.join(root, "tools", "native_tests", "loader_stress.cpp"),
            os.path.join(root, "bigdl-1_amd", "bigdl", "runtime", "csrc", "batch_loader.cpp")]
    for san in ("thread", "address,undefined"):
        exe = str(tmp_path / ("stress_" + san.split(",")[0]))
        subprocess.run([gxx, "-O1", "-g", f"-fsanitize={san}", "-pthread"] + srcs + ["-o", exe], check=True,
                       capture_output=True, timeout=240)
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and "loader stress ok" in r.stdout, r.stderr[-3000:]
        assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
