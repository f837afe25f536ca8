"""Model zoo: tutorial MLPs, ResNet-50, GPT-2, Llama-3 (all on the framework's native layers)."""
from .mlp import TutorialMLP, MnistMLP, linear_20_1  # noqa: F401
from .resnet import ResNet, resnet50  # noqa: F401
