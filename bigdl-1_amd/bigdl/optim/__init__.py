from .optim_method import (OptimMethod, SGD, Adam, ParallelAdam, Adamax, Adagrad, Adadelta, RMSprop, Ftrl, LBFGS,
                           LarsSGD, LearningRateSchedule, Default, Step, MultiStep, EpochStep, EpochDecay, Regime,
                           EpochSchedule, Poly, NaturalExp, Exponential, Plateau, Warmup, SequentialSchedule,
                           EpochDecayWithWarmUp)
from .trigger import (Trigger, EveryEpoch, SeveralIteration, MaxEpoch, MaxIteration, MaxScore, MinLoss, TriggerAnd,
                      TriggerOr)
from .validation import (ValidationMethod, ValidationResult, AccuracyResult, LossResult, Top1Accuracy, Top5Accuracy,
                         TreeNNAccuracy, Loss, MAE, HitRatio, NDCG, MeanAveragePrecision,
                         MeanAveragePrecisionObjectDetection, PrecisionRecallAUC, PRAUCResult, EvaluateMethods)
from .regularizer import Regularizer, L1L2Regularizer, L1Regularizer, L2Regularizer
from .metrics import Metrics
from .optimizer import BaseOptimizer, LocalOptimizer, Optimizer


def __getattr__(name):
    if name == "DistriOptimizer":
        from ..parallel.distri_optimizer import DistriOptimizer
        return DistriOptimizer
    if name == "ParallelOptimizer":
        from ..parallel.distri_optimizer import ParallelOptimizer
        return ParallelOptimizer
    raise AttributeError(name)
from .line_search import LineSearch, LswolfeLineSearch  # noqa: E402,F401
