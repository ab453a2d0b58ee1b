"""The MNIST networks of the reference example jobs (parameter counts in SURVEY.md §2.7 K1-K9).

linear       EX/mnist-pytorch/mnist_distributed.py:129-136      Linear(784, 10)
deepnn       EX/mnist-tensorflow/mnist_distributed.py:64-124    conv5x5(32) pool conv5x5(64) pool fc1024 fc10
                                                                  (3,274,634 params)
keras_cnn    EX/mnist-tensorflow/mnist_keras_distributed.py     Conv2D(32,3) Dense(128) Dense(10) (2,770,634)
hvd_cnn      EX/horovod-on-tony/tensorflow2_mnist.py            Conv(32,3) Conv(64,3) pool Dense(128) Dense(10)
                                                                  (1,199,882)
dnn          EX/mnist-tensorflow/mnist_estimator_distributed.py DNNClassifier([256, 128]) (235,146)
"""
from __future__ import annotations

import torch
from torch import nn


class _Flatten(nn.Module):
    def forward(self, x):
        return x.reshape(x.shape[0], -1)


def linear() -> nn.Module:
    return nn.Sequential(_Flatten(), nn.Linear(784, 10))


def deepnn() -> nn.Module:
    return nn.Sequential(
        nn.Conv2d(1, 32, 5, padding=2), nn.ReLU(), nn.MaxPool2d(2),
        nn.Conv2d(32, 64, 5, padding=2), nn.ReLU(), nn.MaxPool2d(2),
        _Flatten(), nn.Linear(7 * 7 * 64, 1024), nn.ReLU(), nn.Linear(1024, 10))


def keras_cnn() -> nn.Module:
    return nn.Sequential(nn.Conv2d(1, 32, 3), nn.ReLU(), _Flatten(), nn.Linear(26 * 26 * 32, 128), nn.ReLU(),
                         nn.Linear(128, 10))


def hvd_cnn() -> nn.Module:
    return nn.Sequential(nn.Conv2d(1, 32, 3), nn.ReLU(), nn.Conv2d(32, 64, 3), nn.ReLU(), nn.MaxPool2d(2),
                         _Flatten(), nn.Linear(12 * 12 * 64, 128), nn.ReLU(), nn.Linear(128, 10))


def dnn() -> nn.Module:
    return nn.Sequential(_Flatten(), nn.Linear(784, 256), nn.ReLU(), nn.Linear(256, 128), nn.ReLU(),
                         nn.Linear(128, 10))


MODELS = {"linear": linear, "deepnn": deepnn, "keras_cnn": keras_cnn, "hvd_cnn": hvd_cnn, "dnn": dnn}


def mnist_model(name: str = "deepnn", seed: int = 0) -> nn.Module:
    torch.manual_seed(seed)
    return MODELS[name]()


def synthetic_mnist(n: int, seed: int = 0, device="cpu"):
    """Deterministic MNIST-shaped batch (no dataset download): images in [0,1], labels from a fixed
    random linear teacher so the task is learnable (loss decreases)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, 1, 28, 28, generator=g)
    teacher = torch.randn(784, 10, generator=torch.Generator().manual_seed(1234))
    y = (x.reshape(n, -1) @ teacher).argmax(1)
    return x.to(device), y.to(device)
