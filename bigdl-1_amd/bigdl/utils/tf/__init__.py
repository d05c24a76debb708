"""TensorFlow interop: GraphDef loader/saver, TFRecord I/O (``DL/utils/tf/``)."""
from .loader import TensorflowLoader  # noqa: F401
from .saver import TensorflowSaver  # noqa: F401
from .tfrecord import TFRecordIterator, TFRecordWriter  # noqa: F401
