"""TensorBoard observability (``DL/visualization``): TrainSummary, ValidationSummary, event I/O."""
from .summary import Summary, TrainSummary, ValidationSummary, scalar, histogram
from .tensorboard import FileWriter, FileReader, RecordWriter, EventWriter, crc32c, masked_crc32c, read_records

__all__ = ["Summary", "TrainSummary", "ValidationSummary", "scalar", "histogram", "FileWriter", "FileReader",
           "RecordWriter", "EventWriter", "crc32c", "masked_crc32c", "read_records"]
