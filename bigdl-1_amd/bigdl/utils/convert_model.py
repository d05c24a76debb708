"""Model format converter CLI (``DL/utils/ConvertModel.scala:25-133``).

    python -m bigdl.utils.convert_model --from caffe --to bigdl --prototxt deploy.prototxt \\
        --input net.caffemodel --output net.bigdl [--quantize true]

``--from``: bigdl | caffe | torch | tensorflow (``--tf_inputs a,b --tf_outputs c``);
``--to``: bigdl | caffe | torch | tensorflow.  ``--quantize`` (only with ``--to bigdl``) swaps
Linear / SpatialConvolution / SpatialDilatedConvolution for their int8 versions (inference only).
"""
from __future__ import annotations

import argparse
import sys

FROM = ("bigdl", "caffe", "torch", "tensorflow")
TO = ("bigdl", "caffe", "torch", "tensorflow")


def _bool(s: str) -> bool:
    if s.lower() in ("true", "1", "yes"):
        return True
    if s.lower() in ("false", "0", "no"):
        return False
    raise argparse.ArgumentTypeError(f"expected a boolean, got {s!r}")


def parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="convert_model", description="Convert models between different dl frameworks")
    p.add_argument("--from", dest="src", required=True, type=str.lower, choices=FROM,
                   help=f"type of the origin model ({', '.join(FROM)})")
    p.add_argument("--to", dest="dst", required=True, type=str.lower, choices=TO,
                   help=f"type of the model to write ({', '.join(TO)})")
    p.add_argument("--input", required=True, help="origin model file")
    p.add_argument("--output", required=True, help="output model file (caffe: the .caffemodel; the prototxt "
                                                    "is written next to it with a .prototxt suffix)")
    p.add_argument("--prototxt", default="", help="caffe deploy prototxt (required with --from caffe)")
    p.add_argument("--quantize", type=_bool, default=False, help="quantize the model (only with --to bigdl)")
    p.add_argument("--tf_inputs", default="", help="comma-separated TensorFlow input names")
    p.add_argument("--tf_outputs", default="", help="comma-separated TensorFlow output names")
    return p


def load(src: str, path: str, prototxt: str = "", tf_inputs=(), tf_outputs=()):
    from ..nn.module import Module
    if src == "bigdl":
        return Module.loadModule(path)
    if src == "torch":
        return Module.loadTorch(path)
    if src == "caffe":
        return Module.loadCaffeModel(prototxt, path)
    if src == "tensorflow":
        return Module.loadTF(path, list(tf_inputs), list(tf_outputs))
    raise ValueError(src)


def save(model, dst: str, path: str):
    if dst == "bigdl":
        model.saveModule(path, over_write=True)
    elif dst == "torch":
        model.saveTorch(path, over_write=True)
    elif dst == "caffe":
        proto = path[:-len(".caffemodel")] + ".prototxt" if path.endswith(".caffemodel") else path + ".prototxt"
        model.saveCaffe(proto, path, over_write=True)
    elif dst == "tensorflow":
        from .tf import TensorflowSaver
        TensorflowSaver.save_graph(model, [("input", [-1])], path)
    else:
        raise ValueError(dst)


def main(argv=None) -> int:
    a = parser().parse_args(argv)
    if a.src == "caffe" and not a.prototxt:
        parser().error("If model is converted from caffe, the prototxt should be given with --prototxt.")
    if a.src == "tensorflow" and (not a.tf_inputs or not a.tf_outputs):
        parser().error("If model is converted from tensorflow, inputs and outputs should be given")
    if a.quantize and a.dst != "bigdl":
        parser().error("Only support quantizing models to BigDL model now.")
    model = load(a.src, a.input, a.prototxt, [s for s in a.tf_inputs.split(",") if s],
                 [s for s in a.tf_outputs.split(",") if s])
    if a.quantize:
        model = model.quantize()
    save(model, a.dst, a.output)
    print(f"converted {a.src}:{a.input} -> {a.dst}:{a.output}")
    return 0


ConvertModel = main

if __name__ == "__main__":
    sys.exit(main())
