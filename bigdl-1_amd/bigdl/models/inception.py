"""GoogLeNet builders (``DL/models/inception/Inception_v1.scala:106,193``, ``Inception_v2.scala``).

Layer names follow the Caffe bvlc_googlenet naming of the reference (``conv1/7x7_s2``,
``inception_3a/1x1`` …) so Caffe weights load by name (config 5).  v1 convs use Xavier weights
and constant-0.1 biases; v2 (BN-Inception) puts SpatialBatchNormalization(eps=1e-3) after every
conv.  Each builder has a Sequential form and a ``.graph`` form (Graph of ModuleNodes)."""
from __future__ import annotations

from ..nn import (Concat, ConstInitMethod, Dropout, Graph, Input, JoinTable, Linear, LogSoftMax, ReLU, Sequential,
                  SpatialAveragePooling, SpatialBatchNormalization, SpatialConvolution, SpatialCrossMapLRN,
                  SpatialMaxPooling, View, Xavier, Zeros)

# (1x1, (3x3 reduce, 3x3), (5x5 reduce, 5x5), pool proj) per v1 module
_V1 = {
    "3a": (192, 64, (96, 128), (16, 32), 32), "3b": (256, 128, (128, 192), (32, 96), 64),
    "4a": (480, 192, (96, 208), (16, 48), 64), "4b": (512, 160, (112, 224), (24, 64), 64),
    "4c": (512, 128, (128, 256), (24, 64), 64), "4d": (512, 112, (144, 288), (32, 64), 64),
    "4e": (528, 256, (160, 320), (32, 128), 128), "5a": (832, 256, (160, 320), (32, 128), 128),
    "5b": (832, 384, (192, 384), (48, 128), 128),
}


def _xconv(cin, cout, k, s=1, p=0, name=None, propagate_back=True):
    c = SpatialConvolution(cin, cout, k, k, s, s, p, p, 1, propagate_back)
    c.setInitMethod(Xavier(), ConstInitMethod(0.1))
    return c.set_name(name) if name else c


def _relu(name):
    return ReLU(True).set_name(name)


def _v1_branches(cin, c1, c3, c5, cp, pre):
    """The four v1 branches as lists of modules (consumed by both builders)."""
    return [
        [_xconv(cin, c1, 1, name=pre + "1x1"), _relu(pre + "relu_1x1")],
        [_xconv(cin, c3[0], 1, name=pre + "3x3_reduce"), _relu(pre + "relu_3x3_reduce"),
         _xconv(c3[0], c3[1], 3, 1, 1, name=pre + "3x3"), _relu(pre + "relu_3x3")],
        [_xconv(cin, c5[0], 1, name=pre + "5x5_reduce"), _relu(pre + "relu_5x5_reduce"),
         _xconv(c5[0], c5[1], 5, 1, 2, name=pre + "5x5"), _relu(pre + "relu_5x5")],
        [SpatialMaxPooling(3, 3, 1, 1, 1, 1).ceil().set_name(pre + "pool"),
         _xconv(cin, cp, 1, name=pre + "pool_proj"), _relu(pre + "relu_pool_proj")],
    ]


def Inception_Layer_v1(input_size, config, name_prefix=""):
    """config = ((c1,), (c3r, c3), (c5r, c5), (cp,)) as the reference's T(T(..), ...)."""
    c1, c3, c5, cp = config[0][0], tuple(config[1]), tuple(config[2]), config[3][0]
    cat = Concat(2)
    for br in _v1_branches(input_size, c1, c3, c5, cp, name_prefix):
        cat.add(Sequential(*br))
    return cat.set_name(name_prefix + "output")


def _v1_node(x, key):
    cin, c1, c3, c5, cp = _V1[key]
    outs = []
    for br in _v1_branches(cin, c1, c3, c5, cp, f"inception_{key}/"):
        n = x
        for m in br:
            n = m(n)
        outs.append(n)
    return JoinTable(2, 0)(*outs)


def _v1_layer(key):
    cin, c1, c3, c5, cp = _V1[key]
    return Inception_Layer_v1(cin, ((c1,), c3, c5, (cp,)), f"inception_{key}/")


def _v1_stem():
    return [_xconv(3, 64, 7, 2, 3, "conv1/7x7_s2", propagate_back=False), _relu("conv1/relu_7x7"),
            SpatialMaxPooling(3, 3, 2, 2).ceil().set_name("pool1/3x3_s2"),
            SpatialCrossMapLRN(5, 0.0001, 0.75).set_name("pool1/norm1"),
            _xconv(64, 64, 1, name="conv2/3x3_reduce"), _relu("conv2/relu_3x3_reduce"),
            _xconv(64, 192, 3, 1, 1, "conv2/3x3"), _relu("conv2/relu_3x3"),
            SpatialCrossMapLRN(5, 0.0001, 0.75).set_name("conv2/norm2"),
            SpatialMaxPooling(3, 3, 2, 2).ceil().set_name("pool2/3x3_s2")]


def _pool(name):
    return SpatialMaxPooling(3, 3, 2, 2).ceil().set_name(name)


def _v1_head(class_num, has_dropout):
    mods = [SpatialAveragePooling(7, 7, 1, 1).set_name("pool5/7x7_s1")]
    if has_dropout:
        mods.append(Dropout(0.4).set_name("pool5/drop_7x7_s1"))
    fc = Linear(1024, class_num).set_name("loss3/classifier")
    fc.setInitMethod(Xavier(), Zeros())
    mods += [View(1024).setNumInputDims(3), fc, LogSoftMax().set_name("loss3/loss3")]
    return mods


def _v1_aux(idx, cin, class_num, has_dropout, ceil):
    ap = SpatialAveragePooling(5, 5, 3, 3)
    if ceil:
        ap = ap.ceil()
    mods = [ap.set_name(f"loss{idx}/ave_pool"), SpatialConvolution(cin, 128, 1, 1, 1, 1).set_name(f"loss{idx}/conv"),
            _relu(f"loss{idx}/relu_conv"), View(128 * 4 * 4).setNumInputDims(3),
            Linear(128 * 4 * 4, 1024).set_name(f"loss{idx}/fc"), _relu(f"loss{idx}/relu_fc")]
    if has_dropout:
        mods.append(Dropout(0.7).set_name(f"loss{idx}/drop_fc"))
    mods += [Linear(1024, class_num).set_name(f"loss{idx}/classifier"), LogSoftMax().set_name(f"loss{idx}/loss")]
    return mods


def Inception_v1_NoAuxClassifier(class_num=1000, has_dropout=True):
    m = Sequential(*_v1_stem())
    for key in ("3a", "3b"):
        m.add(_v1_layer(key))
    m.add(_pool("pool3/3x3_s2"))
    for key in ("4a", "4b", "4c", "4d", "4e"):
        m.add(_v1_layer(key))
    m.add(_pool("pool4/3x3_s2"))
    for key in ("5a", "5b"):
        m.add(_v1_layer(key))
    for mod in _v1_head(class_num, has_dropout):
        m.add(mod)
    return m


def _v1_noaux_graph(class_num=1000, has_dropout=True):
    inp = Input()
    x = inp
    for mod in _v1_stem():
        x = mod(x)
    for key in ("3a", "3b"):
        x = _v1_node(x, key)
    x = _pool("pool3/3x3_s2")(x)
    for key in ("4a", "4b", "4c", "4d", "4e"):
        x = _v1_node(x, key)
    x = _pool("pool4/3x3_s2")(x)
    for key in ("5a", "5b"):
        x = _v1_node(x, key)
    for mod in _v1_head(class_num, has_dropout):
        x = mod(x)
    return Graph(inp, x)


Inception_v1_NoAuxClassifier.graph = _v1_noaux_graph


def Inception_v1(class_num=1000, has_dropout=True):
    """Three-headed GoogLeNet; output = concat(loss3, loss2, loss1) log-probs along dim 2."""
    feature1 = Sequential(*_v1_stem())
    for key in ("3a", "3b"):
        feature1.add(_v1_layer(key))
    feature1.add(_pool("pool3/3x3_s2")).add(_v1_layer("4a"))
    output1 = Sequential(*_v1_aux(1, 512, class_num, has_dropout, True))
    feature2 = Sequential(_v1_layer("4b"), _v1_layer("4c"), _v1_layer("4d"))
    output2 = Sequential(*_v1_aux(2, 528, class_num, has_dropout, False))
    output3 = Sequential(_v1_layer("4e"), _pool("pool4/3x3_s2"), _v1_layer("5a"), _v1_layer("5b"),
                         *_v1_head(class_num, has_dropout))
    split2 = Concat(2).set_name("split2").add(output3).add(output2)
    main = Sequential(feature2, split2)
    split1 = Concat(2).set_name("split1").add(main).add(output1)
    return Sequential(feature1, split1)


def _v1_graph(class_num=1000, has_dropout=True):
    inp = Input()
    x = inp
    for mod in _v1_stem():
        x = mod(x)
    for key in ("3a", "3b"):
        x = _v1_node(x, key)
    x = _v1_node(_pool("pool3/3x3_s2")(x), "4a")
    o1 = x
    for mod in _v1_aux(1, 512, class_num, has_dropout, True):
        o1 = mod(o1)
    for key in ("4b", "4c", "4d"):
        x = _v1_node(x, key)
    o2 = x
    for mod in _v1_aux(2, 528, class_num, has_dropout, False):
        o2 = mod(o2)
    x = _v1_node(x, "4e")
    x = _pool("pool4/3x3_s2")(x)
    for key in ("5a", "5b"):
        x = _v1_node(x, key)
    for mod in _v1_head(class_num, has_dropout):
        x = mod(x)
    return Graph(inp, JoinTable(2, 0)(x, o2, o1))


Inception_v1.graph = _v1_graph


# ------------------------------------------------------------------------------------------- v2
# (c1, (c3r, c3), (cd_r, cd), (pool kind, pool proj)); c1 == 0 drops the branch, pool proj 0 with
# "max" makes the module a stride-2 reduction
_V2 = {
    "3a": (192, 64, (64, 64), (64, 96), ("avg", 32)), "3b": (256, 64, (64, 96), (64, 96), ("avg", 64)),
    "3c": (320, 0, (128, 160), (64, 96), ("max", 0)), "4a": (576, 224, (64, 96), (96, 128), ("avg", 128)),
    "4b": (576, 192, (96, 128), (96, 128), ("avg", 128)), "4c": (576, 160, (128, 160), (128, 160), ("avg", 96)),
    "4d": (576, 96, (128, 192), (160, 192), ("avg", 96)), "4e": (576, 0, (128, 192), (192, 256), ("max", 0)),
    "5a": (1024, 352, (192, 320), (160, 224), ("avg", 128)),
    "5b": (1024, 352, (192, 320), (192, 224), ("max", 128)),
}


def _cbr(cin, cout, k, s, p, name):
    return [SpatialConvolution(cin, cout, k, k, s, s, p, p).set_name(name),
            SpatialBatchNormalization(cout, 1e-3).set_name(name + "/bn"), ReLU(True).set_name(name + "/bn/sc/relu")]


def _v2_branches(cin, c1, c3, cd, pool, pre):
    kind, proj = pool
    reduce_ = kind == "max" and proj == 0
    s = 2 if reduce_ else 1
    brs = []
    if c1 != 0:
        brs.append(_cbr(cin, c1, 1, 1, 0, pre + "1x1"))
    brs.append(_cbr(cin, c3[0], 1, 1, 0, pre + "3x3_reduce") + _cbr(c3[0], c3[1], 3, s, 1, pre + "3x3"))
    brs.append(_cbr(cin, cd[0], 1, 1, 0, pre + "double3x3_reduce") + _cbr(cd[0], cd[1], 3, 1, 1, pre + "double3x3a")
               + _cbr(cd[1], cd[1], 3, s, 1, pre + "double3x3b"))
    if kind == "max":
        pl = (SpatialMaxPooling(3, 3, 1, 1, 1, 1) if proj != 0 else SpatialMaxPooling(3, 3, 2, 2)).ceil()
    elif kind == "avg":
        pl = SpatialAveragePooling(3, 3, 1, 1, 1, 1).ceil()
    else:
        raise ValueError(kind)
    pbr = [pl.set_name(pre + "pool")]
    if proj != 0:
        pbr += _cbr(cin, proj, 1, 1, 0, pre + "pool_proj")
    brs.append(pbr)
    return brs


def Inception_Layer_v2(input_size, config, name_prefix):
    c1 = config[0][0]
    cat = Concat(2)
    for br in _v2_branches(input_size, c1, tuple(config[1]), tuple(config[2]), tuple(config[3]), name_prefix):
        cat.add(Sequential(*br))
    return cat.set_name(name_prefix + "output")


def _v2_layer(key):
    cin, c1, c3, cd, pool = _V2[key]
    return Inception_Layer_v2(cin, ((c1,), c3, cd, pool), f"inception_{key}/")


def _v2_node(x, key):
    cin, c1, c3, cd, pool = _V2[key]
    outs = []
    for br in _v2_branches(cin, c1, c3, cd, pool, f"inception_{key}/"):
        n = x
        for m in br:
            n = m(n)
        outs.append(n)
    return JoinTable(2, 0)(*outs)


def _v2_stem():
    return (_cbr(3, 64, 7, 2, 3, "conv1/7x7_s2") + [SpatialMaxPooling(3, 3, 2, 2).ceil().set_name("pool1/3x3_s2")]
            + _cbr(64, 64, 1, 1, 0, "conv2/3x3_reduce") + _cbr(64, 192, 3, 1, 1, "conv2/3x3")
            + [SpatialMaxPooling(3, 3, 2, 2).ceil().set_name("pool2/3x3_s2")])


def _v2_head(class_num):
    return [SpatialAveragePooling(7, 7, 1, 1).ceil().set_name("pool5/7x7_s1"), View(1024).setNumInputDims(3),
            Linear(1024, class_num).set_name("loss3/classifier"), LogSoftMax().set_name("loss3/loss")]


def _v2_aux(idx, cin, pool_name, spatial, class_num):
    return ([SpatialAveragePooling(5, 5, 3, 3).ceil().set_name(pool_name)] + _cbr(cin, 128, 1, 1, 0, f"loss{idx}/conv")
            + [View(128 * spatial * spatial).setNumInputDims(3),
               Linear(128 * spatial * spatial, 1024).set_name(f"loss{idx}/fc"),
               ReLU(True).set_name(f"loss{idx}/fc/bn/sc/relu"),
               Linear(1024, class_num).set_name(f"loss{idx}/classifier"), LogSoftMax().set_name(f"loss{idx}/loss")])


def Inception_v2_NoAuxClassifier(class_num=1000):
    m = Sequential(*_v2_stem())
    for key in ("3a", "3b", "3c", "4a", "4b", "4c", "4d", "4e", "5a", "5b"):
        m.add(_v2_layer(key))
    for mod in _v2_head(class_num):
        m.add(mod)
    return m


def _v2_noaux_graph(class_num=1000):
    inp = Input()
    x = inp
    for mod in _v2_stem():
        x = mod(x)
    for key in ("3a", "3b", "3c", "4a", "4b", "4c", "4d", "4e", "5a", "5b"):
        x = _v2_node(x, key)
    for mod in _v2_head(class_num):
        x = mod(x)
    return Graph(inp, x)


Inception_v2_NoAuxClassifier.graph = _v2_noaux_graph


def Inception_v2(class_num=1000):
    features1 = Sequential(*_v2_stem(), _v2_layer("3a"), _v2_layer("3b"), _v2_layer("3c"))
    output1 = Sequential(*_v2_aux(1, 576, "pool3/5x5_s3", 4, class_num))
    features2 = Sequential(*[_v2_layer(k) for k in ("4a", "4b", "4c", "4d", "4e")])
    output2 = Sequential(*_v2_aux(2, 1024, "pool4/5x5_s3", 2, class_num))
    output3 = Sequential(_v2_layer("5a"), _v2_layer("5b"), *_v2_head(class_num))
    split2 = Concat(2).add(output3).add(output2)
    split1 = Concat(2).add(Sequential(features2, split2)).add(output1)
    return Sequential(features1, split1)


def _v2_graph(class_num=1000):
    inp = Input()
    x = inp
    for mod in _v2_stem():
        x = mod(x)
    for key in ("3a", "3b", "3c"):
        x = _v2_node(x, key)
    o1 = x
    for mod in _v2_aux(1, 576, "pool3/5x5_s3", 4, class_num):
        o1 = mod(o1)
    for key in ("4a", "4b", "4c", "4d", "4e"):
        x = _v2_node(x, key)
    o2 = x
    for mod in _v2_aux(2, 1024, "pool4/5x5_s3", 2, class_num):
        o2 = mod(o2)
    for key in ("5a", "5b"):
        x = _v2_node(x, key)
    for mod in _v2_head(class_num):
        x = mod(x)
    return Graph(inp, JoinTable(2, 0)(x, o2, o1))


Inception_v2.graph = _v2_graph
