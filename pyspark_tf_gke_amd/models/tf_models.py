"""Model builders of the reference's TF workloads plus the BASELINE.json model families.

* :func:`build_deep_model` — CSV MLP ``3 -> 16 -> 32 -> 64 -> C(softmax)``, Adam(1e-3),
  SparseCategoricalCrossentropy, accuracy (train_tf_ps.py:328-343).
* :func:`build_cnn_model` — the laser-spot CNN regressor: 5 x [Conv2D(5x5, same) -> PReLU ->
  MaxPooling2D] with channels 8,16,32,64,64 (no pool after the 5th), then Flatten -> Dense(2048,
  relu) (``flat=True``, "CNN-B1", 43,368,850 params) or GAP -> Dense(128, relu), then Dense(2);
  Adam(1e-3), MSE, MAE/MSE metrics (train_tf_ps.py:346-378; the ``__main__`` path uses flat=True,
  :883).
* :func:`build_cnn_a1` — the 3-conv 32/64/128 + GAP + Dense(128) variant whose summary ships in the
  reference (tf-model/100-320-by-256-A1-model.txt; 4,862,914 params).
* :func:`build_mnist_cnn` — BASELINE.json's "MNIST CNN bf16" config (28x28x1, 10 classes).
"""
from __future__ import annotations

from .. import nn
from ..nn import layers as L


def build_deep_model(input_dim: int, num_classes: int, compile: bool = True, device=None) -> nn.Sequential:
    L.reset_name_counters()
    m = nn.Sequential([
        nn.Input(shape=(input_dim,)),
        nn.Dense(16, activation="relu"),
        nn.Dense(32, activation="relu"),
        nn.Dense(64, activation="relu"),
        nn.Dense(num_classes, activation="softmax"),
    ])
    m.build(device=device)
    if compile:
        m.compile(optimizer=nn.optimizers.Adam(learning_rate=1e-3),
                  loss=nn.losses.SparseCategoricalCrossentropy(), metrics=["accuracy"])
    return m


def build_cnn_model(input_shape=(256, 320, 3), num_outputs: int = 2, flat: bool = False, compile: bool = True,
                    summary: bool = True, print_fn=None, device=None) -> nn.Sequential:
    L.reset_name_counters()
    m = nn.Sequential([
        nn.Input(shape=input_shape),
        nn.Conv2D(8, 5, padding="same"), nn.PReLU(), nn.MaxPooling2D(),
        nn.Conv2D(16, 5, padding="same"), nn.PReLU(), nn.MaxPooling2D(),
        nn.Conv2D(32, 5, padding="same"), nn.PReLU(), nn.MaxPooling2D(),
        nn.Conv2D(64, 5, padding="same"), nn.PReLU(), nn.MaxPooling2D(),
        nn.Conv2D(64, 5, padding="same"), nn.PReLU(),
        nn.Flatten() if flat else nn.GlobalAveragePooling2D(),
        nn.Dense(2048, activation="relu") if flat else nn.Dense(128, activation="relu"),
        nn.Dense(num_outputs, activation="linear"),
    ])
    m.build(device=device)
    if summary:
        m.summary(print_fn=print_fn)
    if compile:
        m.compile(optimizer=nn.optimizers.Adam(learning_rate=1e-3), loss=nn.losses.MeanSquaredError(),
                  metrics=[nn.metrics.MeanAbsoluteError(name="mae"), nn.metrics.MeanSquaredError(name="mse")])
    return m


def build_cnn_a1(input_shape=(256, 320, 3), num_outputs: int = 2, compile: bool = True, device=None) -> nn.Sequential:
    L.reset_name_counters()
    m = nn.Sequential([
        nn.Input(shape=input_shape),
        nn.Conv2D(32, 5, padding="same"), nn.PReLU(), nn.MaxPooling2D(),
        nn.Conv2D(64, 5, padding="same"), nn.PReLU(), nn.MaxPooling2D(),
        nn.Conv2D(128, 5, padding="same"), nn.PReLU(),
        nn.GlobalAveragePooling2D(),
        nn.Dense(128, activation="relu"),
        nn.Dense(num_outputs, activation="linear"),
    ])
    m.build(device=device)
    if compile:
        m.compile(optimizer=nn.optimizers.Adam(learning_rate=1e-3), loss="mse", metrics=["mae", "mse"])
    return m


def build_mnist_cnn(num_classes: int = 10, compile: bool = True, device=None) -> nn.Sequential:
    """Keras-examples MNIST convnet shape (28x28x1 -> conv32/pool -> conv64/pool -> dense)."""
    L.reset_name_counters()
    m = nn.Sequential([
        nn.Input(shape=(28, 28, 1)),
        nn.Conv2D(32, 3, padding="same", activation="relu"), nn.MaxPooling2D(),
        nn.Conv2D(64, 3, padding="same", activation="relu"), nn.MaxPooling2D(),
        nn.Flatten(),
        nn.Dense(128, activation="relu"),
        nn.Dense(num_classes, activation="softmax"),
    ])
    m.build(device=device)
    if compile:
        m.compile(optimizer=nn.optimizers.Adam(1e-3), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    return m


CNN_B1_PARAMS = 43_368_850
CNN_A1_PARAMS = 4_862_914
