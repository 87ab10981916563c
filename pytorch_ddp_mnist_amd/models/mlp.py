"""The reference network (ddp_tutorial_cpu.py:43-53 and its four copies, survey C1).

Linear(784,128) -> ReLU -> Dropout(0.2) -> Linear(128,128) -> ReLU -> Linear(128,10,bias=False);
118,272 parameters, no buffers.  Trained with CrossEntropyLoss (mean) and SGD(lr=0.01).
"""
from torch import nn


def create_model(dropout: float = 0.2) -> nn.Sequential:
    return nn.Sequential(
        nn.Linear(28 * 28, 128),
        nn.ReLU(),
        nn.Dropout(dropout),
        nn.Linear(128, 128),
        nn.ReLU(),
        nn.Linear(128, 10, bias=False),
    )
