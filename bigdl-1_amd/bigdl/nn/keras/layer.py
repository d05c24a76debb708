"""pyspark module path ``bigdl.nn.keras.layer`` (``PY/nn/keras/layer.py``)."""
from .layers import *  # noqa: F401,F403
from .topology import *  # noqa: F401,F403
