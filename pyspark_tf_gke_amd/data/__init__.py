"""Input pipelines: tf.data-shaped Dataset, CSV loader, image datasets."""
from .dataset import AUTOTUNE, Dataset  # noqa: F401
