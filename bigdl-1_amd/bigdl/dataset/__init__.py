from .core import (Sample, MiniBatch, ArrayTensorMiniBatch, SparseMiniBatch, DefaultPadding, PaddingParam, Transformer, ChainedTransformer, FnTransformer, SampleToMiniBatch,
                   AbstractDataSet, LocalArrayDataSet, DistributedDataSet, TransformedDataSet, SyntheticDataSet, DataSet,
                   DevicePrefetcher)
