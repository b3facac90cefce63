"""Wide-ResNet of the reference's model zoo (BASELINE config c5: WRN-16-4).

The reference pulls its WRN from the git submodule ``wide_resnet_submodule`` =
meliketoy/wide-resnet.pytorch @ 292b3ede0651e349dd566f9c23408aa572f1bd92 (``.gitmodules:1-3``;
the commit is the one ``notebooks/Man_Colab.ipynb`` cell 5 checks out).  The submodule is not
vendored in /root/reference (empty directory), so this is a restatement of that repository's
published ``networks/wide_resnet.py``: pre-activation basic blocks (BN -> ReLU -> conv3x3 ->
dropout -> BN -> ReLU -> conv3x3, strided on the second conv, 1x1 conv shortcut when the shape
changes), stages [16, 16k, 32k, 64k], final BN(momentum=0.9) -> ReLU -> 8x8 average pool ->
linear.  Every conv carries a bias, as in that file.  Parity with the original is unpinned (the
source is absent here); the parameter registration order below -- which is the ``Mixer`` flatten
order (mixer.py:68-69) -- follows the module attribute order of the published file.
"""
import torch.nn as nn
import torch.nn.functional as F


def conv3x3(in_planes, out_planes, stride=1):
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=1, bias=True)


class wide_basic(nn.Module):  # noqa: N801 -- the published class name
    def __init__(self, in_planes, planes, dropout_rate, stride=1):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(in_planes)
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, bias=True)
        self.dropout = nn.Dropout(p=dropout_rate)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, stride=stride, padding=1, bias=True)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != planes:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride, bias=True))

    def forward(self, x):
        out = self.dropout(self.conv1(F.relu(self.bn1(x))))
        out = self.conv2(F.relu(self.bn2(out)))
        return out + self.shortcut(x)


class Wide_ResNet(nn.Module):  # noqa: N801 -- the published class name
    def __init__(self, depth, widen_factor, dropout_rate, num_classes):
        super().__init__()
        self.in_planes = 16
        if (depth - 4) % 6 != 0:
            raise ValueError("Wide-resnet depth should be 6n+4")
        n = (depth - 4) // 6
        k = widen_factor
        stages = [16, 16 * k, 32 * k, 64 * k]
        self.conv1 = conv3x3(3, stages[0])
        self.layer1 = self._wide_layer(wide_basic, stages[1], n, dropout_rate, stride=1)
        self.layer2 = self._wide_layer(wide_basic, stages[2], n, dropout_rate, stride=2)
        self.layer3 = self._wide_layer(wide_basic, stages[3], n, dropout_rate, stride=2)
        self.bn1 = nn.BatchNorm2d(stages[3], momentum=0.9)
        self.linear = nn.Linear(stages[3], num_classes)

    def _wide_layer(self, block, planes, num_blocks, dropout_rate, stride):
        layers = []
        for s in [stride] + [1] * (num_blocks - 1):
            layers.append(block(self.in_planes, planes, dropout_rate, s))
            self.in_planes = planes
        return nn.Sequential(*layers)

    def forward(self, x):
        out = self.conv1(x)
        out = self.layer1(out)
        out = self.layer2(out)
        out = self.layer3(out)
        out = F.relu(self.bn1(out))
        out = F.avg_pool2d(out, 8)
        out = out.view(out.size(0), -1)
        return self.linear(out)
