"""ResNet family (BASELINE.json config "raw-tf ResNet-50 MultiWorkerMirroredStrategy -> RCCL
all-reduce on 8xMI355X").  Not in the reference repo (SURVEY.md §0 finding 6): the architecture is
Keras' ``keras.applications.ResNet50`` (v1 bottlenecks, stride on the first 1x1 conv of a stage,
conv bias + BatchNormalization(epsilon=1.001e-5), ZeroPadding2D + 7x7/2 stem, 3x3/2 max-pool,
GAP + Dense(classes, softmax)), with Keras' layer names (``conv2_block1_1_conv`` ...), built on the
functional :class:`~pyspark_tf_gke_amd.nn.Model`.  ResNet-50 has 25,636,712 parameters
(25,583,592 trainable), identical to Keras.
"""
from __future__ import annotations

from .. import nn
from ..nn import layers as L

BN_EPS = 1.001e-5


def _block1(x, filters, kernel_size=3, stride=1, conv_shortcut=True, name=None, expansion=4):
    if conv_shortcut:
        shortcut = nn.Conv2D(expansion * filters, 1, strides=stride, name=name + "_0_conv")(x)
        shortcut = nn.BatchNormalization(epsilon=BN_EPS, name=name + "_0_bn")(shortcut)
    else:
        shortcut = x
    x = nn.Conv2D(filters, 1, strides=stride, name=name + "_1_conv")(x)
    x = nn.BatchNormalization(epsilon=BN_EPS, name=name + "_1_bn")(x)
    x = nn.Activation("relu", name=name + "_1_relu")(x)
    x = nn.Conv2D(filters, kernel_size, padding="same", name=name + "_2_conv")(x)
    x = nn.BatchNormalization(epsilon=BN_EPS, name=name + "_2_bn")(x)
    x = nn.Activation("relu", name=name + "_2_relu")(x)
    x = nn.Conv2D(expansion * filters, 1, name=name + "_3_conv")(x)
    x = nn.BatchNormalization(epsilon=BN_EPS, name=name + "_3_bn")(x)
    x = nn.Add(name=name + "_add")([shortcut, x])
    return nn.Activation("relu", name=name + "_out")(x)


def _stack1(x, filters, blocks, stride1=2, name=None, expansion=4):
    x = _block1(x, filters, stride=stride1, name=name + "_block1", expansion=expansion)
    for i in range(2, blocks + 1):
        x = _block1(x, filters, conv_shortcut=False, name=f"{name}_block{i}", expansion=expansion)
    return x


def ResNet(stack_blocks=(3, 4, 6, 3), input_shape=(224, 224, 3), classes: int = 1000, width: int = 64,
           include_top: bool = True, name: str = "resnet50", device=None, build: bool = True) -> nn.Model:
    """Keras ResNet v1 with bottleneck stacks ``stack_blocks`` (ResNet-50: 3,4,6,3) and base width
    ``width`` (64 for the real model; tests use narrow/short variants)."""
    L.reset_name_counters()
    inp = nn.Input(shape=input_shape, name="input_layer")
    x = nn.ZeroPadding2D(3, name="conv1_pad")(inp)
    x = nn.Conv2D(width, 7, strides=2, name="conv1_conv")(x)
    x = nn.BatchNormalization(epsilon=BN_EPS, name="conv1_bn")(x)
    x = nn.Activation("relu", name="conv1_relu")(x)
    x = nn.ZeroPadding2D(1, name="pool1_pad")(x)
    x = nn.MaxPooling2D(3, strides=2, name="pool1_pool")(x)
    f = width
    for s, nb in enumerate(stack_blocks):
        x = _stack1(x, f, nb, stride1=1 if s == 0 else 2, name=f"conv{s + 2}")
        f *= 2
    if include_top:
        x = nn.GlobalAveragePooling2D(name="avg_pool")(x)
        x = nn.Dense(classes, activation="softmax", name="predictions")(x)
    m = nn.Model(inp, x, name=name)
    if build:
        m.build(device=device)
    return m


def ResNet50(include_top: bool = True, weights=None, input_shape=(224, 224, 3), classes: int = 1000,
             device=None) -> nn.Model:
    if weights not in (None, "none"):
        raise ValueError("pretrained weights are not available offline; use weights=None (random init)")
    return ResNet((3, 4, 6, 3), input_shape, classes, include_top=include_top, name="resnet50", device=device)


def build_resnet50(input_shape=(224, 224, 3), classes: int = 1000, optimizer=None, device=None) -> nn.Model:
    m = ResNet50(input_shape=input_shape, classes=classes, device=device)
    m.compile(optimizer=optimizer or nn.optimizers.SGD(learning_rate=0.1, momentum=0.9),
              loss=nn.losses.SparseCategoricalCrossentropy(), metrics=["accuracy"])
    return m


RESNET50_PARAMS = 25_636_712
RESNET50_TRAINABLE = 25_583_592
