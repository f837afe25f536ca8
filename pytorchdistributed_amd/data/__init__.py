"""Data layer: distributed sampler, the reference's synthetic datasets, on-device synthetic
batch generators and a side-stream prefetcher."""
from .sampler import DistributedSampler  # noqa: F401
from .datasets import MyTrainDataset, SimpleDataset, SyntheticMNIST, SyntheticTokens, random_image_batch  # noqa: F401
from .device import DeviceSyntheticImages, DeviceSyntheticTokens, DevicePrefetcher  # noqa: F401
