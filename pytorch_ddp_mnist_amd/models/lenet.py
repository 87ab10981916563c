"""LeNet-5 (BASELINE.json north star: Conv2d, ReLU, MaxPool2d, Linear, LogSoftmax/NLLLoss).

Conv2d(1,6,5,pad=2) -> ReLU -> MaxPool2d(2) -> Conv2d(6,16,5) -> ReLU -> MaxPool2d(2) -> Flatten
-> Linear(400,120) -> ReLU -> Linear(120,84) -> ReLU -> Linear(84,10) -> LogSoftmax(dim=1).
61,706 parameters; state_dict keys 0.*, 3.*, 7.*, 9.*, 11.* (survey §2.6).  The loss is
NLLLoss on the log-probabilities, i.e. the same value as CrossEntropyLoss on the logits; the
native kernels fuse log-softmax + NLL + their backward into one epilogue.
"""
from torch import nn


def create_lenet5() -> nn.Sequential:
    return nn.Sequential(
        nn.Conv2d(1, 6, kernel_size=5, padding=2),
        nn.ReLU(),
        nn.MaxPool2d(2),
        nn.Conv2d(6, 16, kernel_size=5),
        nn.ReLU(),
        nn.MaxPool2d(2),
        nn.Flatten(),
        nn.Linear(400, 120),
        nn.ReLU(),
        nn.Linear(120, 84),
        nn.ReLU(),
        nn.Linear(84, 10),
        nn.LogSoftmax(dim=1),
    )
