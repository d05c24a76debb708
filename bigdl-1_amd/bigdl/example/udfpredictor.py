"""DataFrame UDF prediction (``DL/example/udfpredictor/DataframePredictor.scala``): train (or load)
the text classifier, wrap it as a row-wise prediction function and use it to add a prediction
column to a pandas DataFrame and to filter rows by predicted class (the Spark SQL ``udf`` /
``filter(classifierUDF($"text") === k)`` calls of the reference).  Predictions are batched on the
device rather than one row at a time."""
from __future__ import annotations

import argparse
import sys

import torch

from .textclassification import synthetic_corpus, train, vectorize


def make_udf(model, w2v, dim, seq_len, batch=256):
    model.evaluate()
    params = model.parameters()[0]
    dev = params[0].device if params else torch.device("cpu")

    def predict(texts):
        out = []
        for i in range(0, len(texts), batch):
            x = vectorize(list(texts[i:i + batch]), w2v, dim, seq_len).to(dev)  # rows go to the model's device
            with torch.no_grad():
                out += (model.forward(x).argmax(-1) + 1).cpu().tolist()
        return out
    return predict


def main(argv=None):
    ap = argparse.ArgumentParser(description="text-classifier UDF over a DataFrame")
    ap.add_argument("--synthetic", type=int, default=400)
    ap.add_argument("--seqLen", type=int, default=40)
    ap.add_argument("--filterClass", type=int, default=1)
    a = ap.parse_args(argv)
    import pandas as pd
    from ..utils.engine import Engine
    Engine.init()
    docs, labels, w2v = synthetic_corpus(a.synthetic, 4)
    model, acc = train(docs, labels, w2v, 20, a.seqLen, 4, 32, 3)
    udf = make_udf(model, w2v, 20, a.seqLen)
    df = pd.DataFrame({"filename": [f"doc{i}" for i in range(len(docs))], "text": docs, "textLabel": labels})
    df["textType"] = udf(df["text"].tolist())
    picked = df[df["textType"] == a.filterClass]
    print(picked.head())
    return df, picked


if __name__ == "__main__":
    main(sys.argv[1:])
