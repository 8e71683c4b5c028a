"""Drop-in for /root/reference/utils/loss.py (CrossEntropy2d) on the HIP CE kernel.

Reference semantics (utils/loss.py:14-36): pixels with target < 0 or target ==
ignore_label are dropped, the rest are averaged (``size_average=True``) or weighted by
``weight[target]``; shape asserts as in the reference.  The reference's ``:31-32`` zero
branch is unreachable (it tests ``target.data.dim()`` after masking, which is always 1), so
an all-ignored batch gives NaN there and here.  ``size_average=False`` returns the sum
(``F.cross_entropy(..., size_average=False)``, reference :35; 0 for an all-ignored batch).
"""
from __future__ import annotations

import torch.nn as nn

from ..functional import cross_entropy2d


class CrossEntropy2d(nn.Module):

    def __init__(self, size_average=True, ignore_label=255):
        super().__init__()
        self.size_average = size_average
        self.ignore_label = ignore_label

    def forward(self, predict, target, weight=None):
        assert not target.requires_grad
        assert predict.dim() == 4
        assert target.dim() == 3
        assert predict.size(0) == target.size(0), "{0} vs {1} ".format(predict.size(0), target.size(0))
        assert predict.size(2) == target.size(1), "{0} vs {1} ".format(predict.size(2), target.size(1))
        assert predict.size(3) == target.size(2), "{0} vs {1} ".format(predict.size(3), target.size(2))
        return cross_entropy2d(predict, target.long(), self.ignore_label, weight,
                               reduction="mean" if self.size_average else "sum")
