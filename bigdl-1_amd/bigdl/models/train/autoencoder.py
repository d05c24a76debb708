"""MNIST autoencoder (``DL/models/autoencoder/Train.scala``): 784 → 32 → 784 with MSE, Adagrad
(lr 0.01, decay 0.0, weightDecay 5e-4), batch 150.  ``--folder`` MNIST idx files or
``--synthetic N``."""
from __future__ import annotations

import sys

import numpy as np
import torch

from .common import assemble, base_parser, finish, init_engine, load_model_or, optim_or, per_rank_batch


def main(argv=None):
    ap = base_parser("Train the MNIST autoencoder", batch=150, epochs=10, lr=0.01)
    args = ap.parse_args(argv)
    init_engine(args)
    from ...dataset import MiniBatch
    from ...models.autoencoder import Autoencoder
    from ...nn import MSECriterion
    from ...optim import Adagrad
    batch = per_rank_batch(args)
    if args.synthetic:
        x = np.random.default_rng(args.seed).integers(0, 256, (args.synthetic, 28, 28, 1)).astype(np.uint8)
    else:
        if not args.folder:
            raise SystemExit("--folder (MNIST idx files) or --synthetic N is required")
        from ...dataset.mnist import read_data_sets
        x, _ = read_data_sets(args.folder, "train")
    flat = torch.from_numpy(x.reshape(x.shape[0], -1).astype(np.float32) / 255.0)
    data = [MiniBatch(flat[i:i + batch], flat[i:i + batch]) for i in range(0, flat.shape[0] - batch + 1, batch)]
    model = load_model_or(args, lambda: Autoencoder(32))
    optim = optim_or(args, lambda: Adagrad(learningrate=args.learningRate, learningrate_decay=0.0, weightdecay=5e-4))
    opt = assemble(model, data, MSECriterion(), optim, args, None, None, batch, app="autoencoder")
    opt.optimize()
    return finish(opt, model, args)


if __name__ == "__main__":
    main(sys.argv[1:])
