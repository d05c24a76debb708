from .core import (Sample, MiniBatch, PaddingParam, Transformer, ChainedTransformer, FnTransformer, SampleToMiniBatch,
                   AbstractDataSet, LocalArrayDataSet, DistributedDataSet, TransformedDataSet, SyntheticDataSet, DataSet,
                   DevicePrefetcher)
