"""PTB-model training curves on a learnable synthetic language: tokens follow a fixed random sparse
Markov chain (each of V tokens has 4 possible successors with fixed probabilities), so the
2-layer LSTM LM (PTBModel.lstm, hidden 200, 20 steps, batch 20, Adagrad lr 0.01 decay 0.001 — the
reference's PTB defaults) can drive its per-token cross-entropy from ln V towards the chain's
entropy (ln 4 or lower).  Same init and token stream per arm: bf16 native, fp32 native (bf16x3 step
kernels), fp32 on torch (bigdl.fp32.native=false).

    python tools/convergence_ptb.py --dtype fp32 --steps 1500
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "bigdl-1_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=1500)
    ap.add_argument("--vocab", type=int, default=10000)
    ap.add_argument("--log-every", type=int, default=100)
    args = ap.parse_args()
    from bigdl.utils import config
    config.set_property("bigdl.compute.dtype", args.dtype)
    from bigdl.utils.engine import Engine
    Engine.init()
    from bigdl.models.rnn import PTBModel
    from bigdl.nn import CrossEntropyCriterion, TimeDistributedCriterion
    from bigdl.optim import Adagrad
    from bigdl.optim.optimizer import LocalOptimizer
    from bigdl.dataset import MiniBatch
    from bigdl.utils.random import RNG
    dev = torch.device("cuda")
    V, B, T = args.vocab, 20, 20
    g0 = torch.Generator().manual_seed(11)
    succ = torch.randint(0, V, (V, 4), generator=g0)
    prob = torch.tensor([0.55, 0.25, 0.15, 0.05])
    entropy = float(-(prob * prob.log()).sum())
    succ, prob = succ.to(dev), prob.to(dev)

    def batch(step):
        g = torch.Generator(device=dev).manual_seed(5000 + step)
        toks = torch.empty(B, T + 1, dtype=torch.long, device=dev)
        toks[:, 0] = torch.randint(0, V, (B,), generator=g, device=dev)
        for t in range(T):
            pick = torch.multinomial(prob.expand(B, 4), 1, generator=g).squeeze(1)
            toks[:, t + 1] = succ[toks[:, t], pick]
        return MiniBatch((toks[:, :T] + 1).float(), (toks[:, 1:] + 1).float())

    RNG.setSeed(42)
    torch.manual_seed(42)
    model = PTBModel.lstm(V, 200, V, 2)
    crit = TimeDistributedCriterion(CrossEntropyCriterion(), size_average=False)
    ada = Adagrad(learningrate=0.01, learningrate_decay=0.001)
    first = batch(0)
    opt = LocalOptimizer(model, [first], crit, ada, batch_size=B)
    opt.prepare()
    t0 = time.perf_counter()
    for step in range(args.steps):
        loss = opt.train_step(batch(step))
        if step % args.log_every == 0 or step == args.steps - 1:
            # TimeDistributedCriterion(size_average=False) sums over the T steps: per-token nats = loss / T
            print(json.dumps({"dtype": args.dtype, "step": step, "nats_per_token": round(float(loss) / T, 4),
                              "t": round(time.perf_counter() - t0, 1)}), flush=True)
    print(json.dumps({"dtype": args.dtype, "final": True, "steps": args.steps, "ln_vocab": round(math.log(V), 3),
                      "chain_entropy": round(entropy, 3), "train_s": round(time.perf_counter() - t0, 1)}),
          flush=True)


if __name__ == "__main__":
    main()
