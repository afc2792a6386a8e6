"""Model families: the reference's TF models (CSV-MLP, CNN-B1/A1) and the BASELINE configs
(MNIST CNN, ResNet-50)."""
from .tf_models import (CNN_A1_PARAMS, CNN_B1_PARAMS, build_cnn_a1, build_cnn_model, build_deep_model,  # noqa: F401
                        build_mnist_cnn)
