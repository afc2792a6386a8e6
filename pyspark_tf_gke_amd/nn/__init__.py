"""Keras-shaped training API on the MI355X kernels: layers, Sequential, losses, metrics, optimizers,
GradientTape-style loops.  Mirrors the ``tf.keras`` surface used by train_tf_ps.py."""
from . import layers, losses, metrics, optimizers, saved_model  # noqa: F401
from .layers import (Activation, Add, BatchNormalization, Conv2D, Dense, Flatten,  # noqa: F401
                     GlobalAveragePooling2D, Input, MaxPooling2D, PReLU, ReLU, ZeroPadding2D)
from .functional import Model  # noqa: F401
from .model import Sequential, load_model  # noqa: F401
from .tape import GradientTape, add_n  # noqa: F401
