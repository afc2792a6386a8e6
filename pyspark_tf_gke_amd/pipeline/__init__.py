"""End-to-end pipelines that chain the DataFrame engine and the training runtime."""
from .joint import run_joint  # noqa: F401
