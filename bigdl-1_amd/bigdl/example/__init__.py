"""Runnable examples (the reference's ``DL/example/*`` mains).

* ``textclassification`` — News20 + GloVe CNN text classifier (TextClassifier.scala);
* ``languagemodel``      — PTB word LM (PTBWordLM.scala; the model-zoo trainer ``models.train.rnn``);
* ``udfpredictor``       — a trained text classifier applied as a DataFrame UDF (DataframePredictor.scala);
* ``mlpipeline``         — DLClassifier / DLEstimator pipelines (DLClassifierLeNet / LogisticRegression /
  DLEstimatorMultiLabelLR .scala);
* ``loadmodel``          — load a Caffe / Torch / BigDL model and validate it (loadmodel/ModelValidator.scala);
* ``imageclassification``— batch prediction over an image folder with a saved model (ImagePredictor.scala);
* ``keras``              — LeNet through the Keras-style API (example/keras/Train.scala).

Each is ``python -m bigdl.example.<name> --help``; without datasets (no network) they run on
``--synthetic`` data of the right shape.
"""
