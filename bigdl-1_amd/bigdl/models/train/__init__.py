"""Model-zoo training / evaluation entry points (the reference's ``models/*/Train.scala`` and
``Test.scala`` mains, ``DL/models/{resnet,lenet,vgg,rnn,inception,autoencoder}``).

Every module is a CLI (``python -m bigdl.models.train.<name> --help``) and runs single-process or
one process per GPU under the launcher::

    python -m bigdl.launch --nproc 8 -m bigdl.models.train.imagenet -f /data/imagenet-seq \
        --batchSize 2048 --nEpochs 90 --warmupEpoch 5 --maxLr 3.2 --checkpoint /ckpt

* ``imagenet``  — ResNet (TrainImageNet.scala) / Inception-v1 / VGG-16 on ImageNet sequence files
  through the native batch loader; ``--test`` = TestImageNet (Top-1 / Top-5 of a saved model);
* ``cifar``     — VggForCifar10 / ResNet-20…110 (vgg/Train.scala, resnet/TrainCIFAR10.scala);
* ``lenet``     — LeNet-5 on MNIST idx files (lenet/Train.scala, lenet/Test.scala);
* ``rnn``       — PTB language model (rnn/Train.scala: LSTM LM, perplexity);
* ``autoencoder`` — MNIST autoencoder (autoencoder/Train.scala).

Datasets are never downloaded (no network): point ``--folder`` at local files, or pass
``--synthetic N`` to train on N random records of the right shape (used by the CI tests).
"""
