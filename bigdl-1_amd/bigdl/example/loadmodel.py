"""Load a pre-trained model and validate it (``DL/example/loadmodel/ModelValidator.scala``):
``--modelType caffe|torch|bigdl``, ``--modelPath``, ``--caffeDefPath``, ``--folder`` of labelled
images; the Top-1/Top-5 evaluation is :mod:`bigdl.models.utils.model_validator`."""
import sys

from ..models.utils.model_validator import main

if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
