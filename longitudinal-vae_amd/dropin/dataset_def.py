"""dataset_def.py surface for Health-MNIST (reference dataset_def.py:172-219): the dataset is
preloaded into device tensors (lvae_amd.data)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from lvae_amd.data import DeviceBatchLoader, HealthMNISTDatasetConv  # noqa: E402,F401

__all__ = ["HealthMNISTDatasetConv", "DeviceBatchLoader"]
