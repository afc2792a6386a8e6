"""Keras-shaped layer objects (configuration + parameter declaration).

The layer list mirrors what the reference builds with ``tf.keras.Sequential``
(train_tf_ps.py:328-378): Input, Dense(relu/softmax/linear), Conv2D(k, 5, padding="same"),
PReLU (per-element alpha), MaxPooling2D(2x2), Flatten, GlobalAveragePooling2D.  Execution is not
here: :mod:`.engine` fuses consecutive layers into device ops (e.g. Conv2D+PReLU+MaxPooling2D
becomes one implicit-GEMM conv + one fused PReLU/pool kernel).

Weight layouts (device): Conv2D kernel [Cout][KH][KW][Cin_padded], Dense kernel [out][in].
``keras_weights`` / ``set_keras_weights`` convert to/from Keras layouts ([KH,KW,Cin,Cout],
[in,out]) for the saved model format.
"""
from __future__ import annotations

import re

import numpy as np

from .params import ParamStore, glorot_uniform, ones, zeros

_counters: dict = {}


def _auto_name(base: str) -> str:
    n = _counters.get(base, 0)
    _counters[base] = n + 1
    return base if n == 0 else f"{base}_{n}"


def reset_name_counters() -> None:
    _counters.clear()


class Layer:
    kind = "Layer"
    keras_class = "Layer"

    def __init__(self, name: str | None = None):
        self.name = name or _auto_name(self.default_base())
        self.in_shape = None
        self.out_shape = None
        self.params = []

    @classmethod
    def default_base(cls) -> str:
        # Keras' to_snake_case: Conv2D -> conv2d, PReLU -> p_re_lu, MaxPooling2D -> max_pooling2d
        s = re.sub("(.)([A-Z][a-z]+)", r"\1_\2", cls.keras_class)
        return re.sub("([a-z])([A-Z])", r"\1_\2", s).lower()

    def build(self, in_shape: tuple, store: ParamStore) -> tuple:
        self.in_shape = tuple(in_shape)
        self.out_shape = self.compute_output_shape(self.in_shape)
        return self.out_shape

    def __call__(self, inputs):
        """Functional API: ``y = layer(x)`` records a graph node (see :class:`.functional.Model`)."""
        from .functional import KerasTensor

        ins = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        ins = [t.output if isinstance(t, Input) else t for t in ins]
        for t in ins:
            if not isinstance(t, KerasTensor):
                raise TypeError(f"{self.name}: functional call expects KerasTensors, got {type(t).__name__}")
        if getattr(self, "_inbound", None) is not None:
            raise NotImplementedError(f"layer {self.name} is already connected (shared layers are not supported)")
        self._inbound = ins
        shape = self.compute_output_shape(ins[0].shape if len(ins) == 1 else tuple(t.shape for t in ins))
        return KerasTensor(tuple(shape), self, ins)

    def compute_output_shape(self, s):
        return s

    def get_config(self) -> dict:
        return {"name": self.name}

    def param_count(self) -> int:
        return sum(p.logical_numel if p.logical_numel is not None else p.numel for p in self.params)

    def keras_weights(self) -> list:
        return []

    def set_keras_weights(self, ws: list) -> None:
        pass


class Input(Layer):
    kind = "Input"
    keras_class = "InputLayer"

    def __init__(self, shape, name=None, dtype="float32"):
        super().__init__(name or _auto_name("input_layer"))
        self.shape = tuple(int(s) for s in shape)
        self.dtype = dtype
        from .functional import KerasTensor

        self.output = KerasTensor(self.shape, self, [])

    def get_config(self):
        return {"name": self.name, "batch_shape": [None, *self.shape], "dtype": self.dtype}


class Dense(Layer):
    kind = "Dense"
    keras_class = "Dense"

    def __init__(self, units: int, activation=None, use_bias=True, name=None):
        super().__init__(name)
        self.units = int(units)
        self.activation = activation or "linear"
        self.use_bias = use_bias

    def compute_output_shape(self, s):
        return (*s[:-1], self.units)

    def build(self, in_shape, store):
        super().build(in_shape, store)
        fin = int(in_shape[-1])
        self.fan_in = fin
        self.kernel = store.add(f"{self.name}/kernel", (self.units, fin), glorot_uniform(fin, self.units))
        self.params = [self.kernel]
        if self.use_bias:
            self.bias = store.add(f"{self.name}/bias", (self.units,), zeros)
            self.params.append(self.bias)
        else:
            self.bias = None
        return self.out_shape

    def get_config(self):
        return {"name": self.name, "units": self.units, "activation": self.activation, "use_bias": self.use_bias}

    def keras_weights(self):
        out = [self.kernel.data.detach().float().cpu().numpy().T.copy()]
        if self.bias is not None:
            out.append(self.bias.data.detach().float().cpu().numpy().copy())
        return out

    def set_keras_weights(self, ws):
        import torch

        self.kernel.data.copy_(torch.from_numpy(np.ascontiguousarray(ws[0].T)))
        if self.bias is not None:
            self.bias.data.copy_(torch.from_numpy(ws[1]))


class Conv2D(Layer):
    """NHWC conv; input channels are padded to a power of two >= 4 on device (the padded filter
    channels are zero and stay zero: their gradient is the zero padded input)."""

    kind = "Conv2D"
    keras_class = "Conv2D"

    def __init__(self, filters: int, kernel_size, strides=1, padding="valid", activation=None, use_bias=True,
                 name=None):
        super().__init__(name)
        self.filters = int(filters)
        ks = kernel_size if isinstance(kernel_size, (tuple, list)) else (kernel_size, kernel_size)
        self.kernel_size = (int(ks[0]), int(ks[1]))
        st = strides if isinstance(strides, (tuple, list)) else (strides, strides)
        self.strides = (int(st[0]), int(st[1]))
        self.padding = padding
        self.activation = activation or "linear"
        self.use_bias = use_bias

    @staticmethod
    def padded_channels(c: int) -> int:
        p = 4
        while p < c:
            p *= 2
        return p

    def pad_amount(self) -> int:
        if self.padding == "same":
            return (self.kernel_size[0] - 1) // 2
        return 0

    def compute_output_shape(self, s):
        H, W, _ = s
        KH, KW = self.kernel_size
        sh, sw = self.strides
        if self.padding == "same":
            OH, OW = -(-H // sh), -(-W // sw)
        else:
            OH, OW = (H - KH) // sh + 1, (W - KW) // sw + 1
        return (OH, OW, self.filters)

    def build(self, in_shape, store):
        super().build(in_shape, store)
        cin = int(in_shape[-1])
        self.cin = cin
        self.cin_p = self.padded_channels(cin)
        KH, KW = self.kernel_size
        fan_in, fan_out = KH * KW * cin, KH * KW * self.filters
        cp = self.cin_p

        def mask(v, cin=cin, cp=cp):
            if cp != cin:
                v[..., cin:] = 0.0
            return v

        self.kernel = store.add(f"{self.name}/kernel", (self.filters, KH, KW, cp), glorot_uniform(fan_in, fan_out),
                                logical_numel=self.filters * KH * KW * cin, mask_fn=mask)
        self.params = [self.kernel]
        if self.use_bias:
            self.bias = store.add(f"{self.name}/bias", (self.filters,), zeros)
            self.params.append(self.bias)
        else:
            self.bias = None
        return self.out_shape

    def get_config(self):
        return {"name": self.name, "filters": self.filters, "kernel_size": list(self.kernel_size),
                "strides": list(self.strides), "padding": self.padding, "activation": self.activation,
                "use_bias": self.use_bias}

    def keras_weights(self):
        k = self.kernel.data.detach().float().cpu().numpy()[..., : self.cin]  # [Cout,KH,KW,Cin]
        out = [np.ascontiguousarray(k.transpose(1, 2, 3, 0))]
        if self.bias is not None:
            out.append(self.bias.data.detach().float().cpu().numpy().copy())
        return out

    def set_keras_weights(self, ws):
        import torch

        k = np.zeros((self.filters, *self.kernel_size, self.cin_p), np.float32)
        k[..., : self.cin] = ws[0].transpose(3, 0, 1, 2)
        self.kernel.data.copy_(torch.from_numpy(k))
        if self.bias is not None:
            self.bias.data.copy_(torch.from_numpy(ws[1]))


class PReLU(Layer):
    """Keras PReLU with the default ``shared_axes=None``: one alpha per activation element."""

    kind = "PReLU"
    keras_class = "PReLU"

    def build(self, in_shape, store):
        super().build(in_shape, store)
        self.alpha = store.add(f"{self.name}/alpha", tuple(in_shape), zeros)
        self.params = [self.alpha]
        return self.out_shape

    def keras_weights(self):
        return [self.alpha.data.detach().float().cpu().numpy().copy()]

    def set_keras_weights(self, ws):
        import torch

        self.alpha.data.copy_(torch.from_numpy(ws[0]))


def _pair(v):
    return (int(v[0]), int(v[1])) if isinstance(v, (tuple, list)) else (int(v), int(v))


class MaxPooling2D(Layer):
    """Square windows, 'valid' padding (Keras pads explicitly with ZeroPadding2D, which the engine
    folds into the pooling kernel).  2x2/stride 2 is the reference CNN's configuration
    (train_tf_ps.py:353); 3x3/stride 2 is ResNet-50's stem."""

    kind = "MaxPooling2D"
    keras_class = "MaxPooling2D"

    def __init__(self, pool_size=2, strides=None, padding="valid", name=None):
        super().__init__(name)
        self.pool_size = _pair(pool_size)
        self.strides = _pair(strides) if strides is not None else self.pool_size
        if self.pool_size[0] != self.pool_size[1] or self.strides[0] != self.strides[1] or padding != "valid":
            raise NotImplementedError("MaxPooling2D: square windows/strides with padding='valid'")
        self.padding = padding

    def compute_output_shape(self, s):
        H, W, C = s
        k, st = self.pool_size[0], self.strides[0]
        return ((H - k) // st + 1, (W - k) // st + 1, C)

    def get_config(self):
        return {"name": self.name, "pool_size": list(self.pool_size), "strides": list(self.strides),
                "padding": "valid"}


class ZeroPadding2D(Layer):
    kind = "ZeroPadding2D"
    keras_class = "ZeroPadding2D"

    def __init__(self, padding=1, name=None):
        super().__init__(name)
        if isinstance(padding, (tuple, list)):
            a, b = padding
            if isinstance(a, (tuple, list)) or isinstance(b, (tuple, list)) or a != b:
                raise NotImplementedError("ZeroPadding2D: symmetric padding only")
            padding = a
        self.pad = int(padding)

    def compute_output_shape(self, s):
        H, W, C = s
        return (H + 2 * self.pad, W + 2 * self.pad, C)

    def get_config(self):
        return {"name": self.name, "padding": [[self.pad, self.pad], [self.pad, self.pad]]}


class BatchNormalization(Layer):
    """Keras BatchNormalization over the last (channel) axis.  gamma/beta are trainable parameters of
    the flat store; moving_mean/moving_variance are non-trainable device buffers (updated during
    training steps with ``momentum``)."""

    kind = "BatchNormalization"
    keras_class = "BatchNormalization"

    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, name=None):
        super().__init__(name)
        if axis not in (-1, 3):
            raise NotImplementedError("BatchNormalization over the channel (last) axis only")
        self.momentum, self.epsilon = float(momentum), float(epsilon)
        self.center, self.scale = center, scale
        self.moving_mean = self.moving_variance = None

    def build(self, in_shape, store):
        super().build(in_shape, store)
        C = int(in_shape[-1])
        self.channels = C
        self.params = []
        self.gamma = store.add(f"{self.name}/gamma", (C,), ones) if self.scale else None
        self.beta = store.add(f"{self.name}/beta", (C,), zeros) if self.center else None
        self.params = [p for p in (self.gamma, self.beta) if p is not None]
        return self.out_shape

    def init_state(self, device) -> None:
        import torch

        if self.moving_mean is None or self.moving_mean.device != torch.device(device):
            self.moving_mean = torch.zeros(self.channels, dtype=torch.float32, device=device)
            self.moving_variance = torch.ones(self.channels, dtype=torch.float32, device=device)

    def param_count(self) -> int:
        return super().param_count() + 2 * self.channels

    def non_trainable_count(self) -> int:
        return 2 * self.channels

    def get_config(self):
        return {"name": self.name, "axis": -1, "momentum": self.momentum, "epsilon": self.epsilon,
                "center": self.center, "scale": self.scale}

    def keras_weights(self):
        out = [p.data.detach().float().cpu().numpy().copy() for p in self.params]
        out += [self.moving_mean.detach().cpu().numpy().copy(), self.moving_variance.detach().cpu().numpy().copy()]
        return out

    def set_keras_weights(self, ws):
        import torch

        for p, w in zip(self.params, ws):
            p.data.copy_(torch.from_numpy(np.ascontiguousarray(w)))
        self.moving_mean.copy_(torch.from_numpy(np.ascontiguousarray(ws[-2])))
        self.moving_variance.copy_(torch.from_numpy(np.ascontiguousarray(ws[-1])))


class Activation(Layer):
    kind = "Activation"
    keras_class = "Activation"

    def __init__(self, activation, name=None):
        super().__init__(name)
        if activation not in ("relu", "linear", "softmax"):
            raise NotImplementedError(f"Activation({activation!r})")
        self.activation = activation

    def get_config(self):
        return {"name": self.name, "activation": self.activation}


class Add(Layer):
    kind = "Add"
    keras_class = "Add"

    def compute_output_shape(self, s):
        shapes = s if isinstance(s[0], tuple) else (s,)
        if any(tuple(x) != tuple(shapes[0]) for x in shapes):
            raise ValueError(f"Add: shape mismatch {shapes}")
        return tuple(shapes[0])


class Flatten(Layer):
    kind = "Flatten"
    keras_class = "Flatten"

    def compute_output_shape(self, s):
        return (int(np.prod(s)),)


class GlobalAveragePooling2D(Layer):
    kind = "GlobalAveragePooling2D"
    keras_class = "GlobalAveragePooling2D"

    def compute_output_shape(self, s):
        return (s[-1],)


class ReLU(Layer):
    kind = "ReLU"
    keras_class = "ReLU"


LAYER_CLASSES = {c.keras_class: c for c in (Input, Dense, Conv2D, PReLU, MaxPooling2D, Flatten,
                                              GlobalAveragePooling2D, ReLU, ZeroPadding2D, BatchNormalization,
                                              Activation, Add)}


def layer_from_config(cls_name: str, cfg: dict) -> Layer:
    cls = LAYER_CLASSES[cls_name]
    cfg = dict(cfg)
    if cls is Input:
        return Input(cfg["batch_shape"][1:], name=cfg.get("name"))
    if cls is Dense:
        return Dense(cfg["units"], cfg.get("activation"), cfg.get("use_bias", True), name=cfg.get("name"))
    if cls is Conv2D:
        return Conv2D(cfg["filters"], tuple(cfg["kernel_size"]), tuple(cfg.get("strides", (1, 1))),
                      cfg.get("padding", "valid"), cfg.get("activation"), cfg.get("use_bias", True),
                      name=cfg.get("name"))
    if cls is MaxPooling2D:
        return MaxPooling2D(tuple(cfg.get("pool_size", (2, 2))), tuple(cfg.get("strides", cfg.get("pool_size", (2, 2)))),
                            name=cfg.get("name"))
    if cls is ZeroPadding2D:
        pad = cfg.get("padding", 1)
        return ZeroPadding2D(pad[0][0] if isinstance(pad, (list, tuple)) else pad, name=cfg.get("name"))
    if cls is BatchNormalization:
        return BatchNormalization(momentum=cfg.get("momentum", 0.99), epsilon=cfg.get("epsilon", 1e-3),
                                  center=cfg.get("center", True), scale=cfg.get("scale", True), name=cfg.get("name"))
    if cls is Activation:
        return Activation(cfg["activation"], name=cfg.get("name"))
    return cls(name=cfg.get("name"))


__all__ = ["Layer", "Input", "Dense", "Conv2D", "PReLU", "MaxPooling2D", "Flatten", "GlobalAveragePooling2D",
           "ReLU", "ZeroPadding2D", "BatchNormalization", "Activation", "Add", "layer_from_config",
           "reset_name_counters"]

