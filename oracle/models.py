"""PyTorch fp32 CPU restatements of the reference backbones (TEST INFRASTRUCTURE ONLY).

State-dict key names match the reference exactly so that a reference checkpoint (or the
synthetic one from facerecognition_amd.weights.synth_state_dict) loads with strict=True.

* ``ArcFaceModel``      models/arcface/arcface_model.py:135-202, trunk = torchvision resnet50
                        (v1.5: stride on the 3x3) as copied at :88-98, forward :118-132.
* ``IResNet100``        insightface iresnet100 (IBasicBlock: bn1→conv→bn2→PReLU→conv(stride)→bn3
                        (+downsample), no ReLU after the add); README.md:72,119,300 only.
* ``FaceNetModel``      models/facenet/facenet_model.py:7-36 around facenet-pytorch 2.5.x
                        InceptionResnetV1 (classify=False: last_linear → last_bn → F.normalize).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# ------------------------------------------------------------------ ResNet-50 (torchvision layout)
class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            idt = self.downsample(x)
        return self.relu(out + idt)


class ResNet50(nn.Module):
    """torchvision.models.resnet50 module layout (used as the trunk and as the golden shim)."""

    def __init__(self):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._make(64, 3, 1)
        self.layer2 = self._make(128, 4, 2)
        self.layer3 = self._make(256, 6, 2)
        self.layer4 = self._make(512, 3, 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, 1000)

    def _make(self, planes, blocks, stride):
        ds = None
        if stride != 1 or self.inplanes != planes * 4:
            ds = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                               nn.BatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, ds)]
        self.inplanes = planes * 4
        layers += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)


class ResNetBackbone(nn.Module):
    """arcface_model.py:65-132 with pretrained=False (no ImageNet download)."""

    def __init__(self):
        super().__init__()
        r = ResNet50()
        self.conv1, self.bn1, self.relu, self.maxpool = r.conv1, r.bn1, r.relu, r.maxpool
        self.layer1, self.layer2, self.layer3, self.layer4 = r.layer1, r.layer2, r.layer3, r.layer4
        self.avgpool = r.avgpool

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return torch.flatten(self.avgpool(x), 1)


class ArcFaceModel(nn.Module):
    """arcface_model.py:135-202; forward(x, labels=None) returns the un-normalized embedding."""

    def __init__(self, num_classes=100, embedding_size=512, dropout=0.5):
        super().__init__()
        self.backbone = ResNetBackbone()
        self.bn1 = nn.BatchNorm1d(2048)
        self.dropout = nn.Dropout(p=dropout)
        self.fc = nn.Linear(2048, embedding_size)
        self.bn2 = nn.BatchNorm1d(embedding_size)
        self.arcface = nn.Module()
        self.arcface.weight = nn.Parameter(torch.zeros(num_classes, embedding_size))

    def forward(self, x, labels=None):
        if labels is not None:
            raise NotImplementedError("training head (ArcMarginProduct) is out of scope")
        x = self.dropout(self.bn1(self.backbone(x)))
        return self.bn2(self.fc(x))


# ------------------------------------------------------------------ IResNet100 (insightface)
class IBasicBlock(nn.Module):
    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.bn1 = nn.BatchNorm2d(inplanes, eps=1e-05)
        self.conv1 = nn.Conv2d(inplanes, planes, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes, eps=1e-05)
        self.prelu = nn.PReLU(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes, eps=1e-05)
        self.downsample = downsample

    def forward(self, x):
        idt = x
        out = self.conv1(self.bn1(x))
        out = self.prelu(self.bn2(out))
        out = self.bn3(self.conv2(out))
        if self.downsample is not None:
            idt = self.downsample(x)
        return out + idt


class IResNet100(nn.Module):
    def __init__(self, num_features=512):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 3, stride=1, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(64, eps=1e-05)
        self.prelu = nn.PReLU(64)
        self.layer1 = self._make(64, 3, 2)
        self.layer2 = self._make(128, 13, 2)
        self.layer3 = self._make(256, 30, 2)
        self.layer4 = self._make(512, 3, 2)
        self.bn2 = nn.BatchNorm2d(512, eps=1e-05)
        self.dropout = nn.Dropout(p=0.0)
        self.fc = nn.Linear(512 * 49, num_features)
        self.features = nn.BatchNorm1d(num_features, eps=1e-05)

    def _make(self, planes, blocks, stride):
        ds = None
        if stride != 1 or self.inplanes != planes:
            ds = nn.Sequential(nn.Conv2d(self.inplanes, planes, 1, stride=stride, bias=False),
                               nn.BatchNorm2d(planes, eps=1e-05))
        layers = [IBasicBlock(self.inplanes, planes, stride, ds)]
        self.inplanes = planes
        layers += [IBasicBlock(planes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x, labels=None):
        x = self.prelu(self.bn1(self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.bn2(x), 1)
        return self.features(self.fc(self.dropout(x)))


# ------------------------------------------------------------------ InceptionResnetV1 (facenet-pytorch 2.5.x)
class BasicConv2d(nn.Module):
    def __init__(self, cin, cout, k, stride, padding=0):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, stride=stride, padding=padding, bias=False)
        self.bn = nn.BatchNorm2d(cout, eps=0.001, momentum=0.1, affine=True)
        self.relu = nn.ReLU(inplace=False)

    def forward(self, x):
        return self.relu(self.bn(self.conv(x)))


class Block35(nn.Module):
    def __init__(self, scale=1.0):
        super().__init__()
        self.scale = scale
        self.branch0 = BasicConv2d(256, 32, 1, 1)
        self.branch1 = nn.Sequential(BasicConv2d(256, 32, 1, 1), BasicConv2d(32, 32, 3, 1, 1))
        self.branch2 = nn.Sequential(BasicConv2d(256, 32, 1, 1), BasicConv2d(32, 32, 3, 1, 1),
                                     BasicConv2d(32, 32, 3, 1, 1))
        self.conv2d = nn.Conv2d(96, 256, 1, stride=1)
        self.relu = nn.ReLU(inplace=False)

    def forward(self, x):
        out = torch.cat((self.branch0(x), self.branch1(x), self.branch2(x)), 1)
        return self.relu(self.conv2d(out) * self.scale + x)


class Block17(nn.Module):
    def __init__(self, scale=1.0):
        super().__init__()
        self.scale = scale
        self.branch0 = BasicConv2d(896, 128, 1, 1)
        self.branch1 = nn.Sequential(BasicConv2d(896, 128, 1, 1), BasicConv2d(128, 128, (1, 7), 1, (0, 3)),
                                     BasicConv2d(128, 128, (7, 1), 1, (3, 0)))
        self.conv2d = nn.Conv2d(256, 896, 1, stride=1)
        self.relu = nn.ReLU(inplace=False)

    def forward(self, x):
        out = torch.cat((self.branch0(x), self.branch1(x)), 1)
        return self.relu(self.conv2d(out) * self.scale + x)


class Block8(nn.Module):
    def __init__(self, scale=1.0, noReLU=False):
        super().__init__()
        self.scale = scale
        self.noReLU = noReLU
        self.branch0 = BasicConv2d(1792, 192, 1, 1)
        self.branch1 = nn.Sequential(BasicConv2d(1792, 192, 1, 1), BasicConv2d(192, 192, (1, 3), 1, (0, 1)),
                                     BasicConv2d(192, 192, (3, 1), 1, (1, 0)))
        self.conv2d = nn.Conv2d(384, 1792, 1, stride=1)
        if not noReLU:
            self.relu = nn.ReLU(inplace=False)

    def forward(self, x):
        out = torch.cat((self.branch0(x), self.branch1(x)), 1)
        out = self.conv2d(out) * self.scale + x
        return out if self.noReLU else self.relu(out)


class Mixed_6a(nn.Module):
    def __init__(self):
        super().__init__()
        self.branch0 = BasicConv2d(256, 384, 3, 2)
        self.branch1 = nn.Sequential(BasicConv2d(256, 192, 1, 1), BasicConv2d(192, 192, 3, 1, 1),
                                     BasicConv2d(192, 256, 3, 2))
        self.branch2 = nn.MaxPool2d(3, stride=2)

    def forward(self, x):
        return torch.cat((self.branch0(x), self.branch1(x), self.branch2(x)), 1)


class Mixed_7a(nn.Module):
    def __init__(self):
        super().__init__()
        self.branch0 = nn.Sequential(BasicConv2d(896, 256, 1, 1), BasicConv2d(256, 384, 3, 2))
        self.branch1 = nn.Sequential(BasicConv2d(896, 256, 1, 1), BasicConv2d(256, 256, 3, 2))
        self.branch2 = nn.Sequential(BasicConv2d(896, 256, 1, 1), BasicConv2d(256, 256, 3, 1, 1),
                                     BasicConv2d(256, 256, 3, 2))
        self.branch3 = nn.MaxPool2d(3, stride=2)

    def forward(self, x):
        return torch.cat((self.branch0(x), self.branch1(x), self.branch2(x), self.branch3(x)), 1)


class InceptionResnetV1(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv2d_1a = BasicConv2d(3, 32, 3, 2)
        self.conv2d_2a = BasicConv2d(32, 32, 3, 1)
        self.conv2d_2b = BasicConv2d(32, 64, 3, 1, 1)
        self.maxpool_3a = nn.MaxPool2d(3, stride=2)
        self.conv2d_3b = BasicConv2d(64, 80, 1, 1)
        self.conv2d_4a = BasicConv2d(80, 192, 3, 1)
        self.conv2d_4b = BasicConv2d(192, 256, 3, 2)
        self.repeat_1 = nn.Sequential(*[Block35(scale=0.17) for _ in range(5)])
        self.mixed_6a = Mixed_6a()
        self.repeat_2 = nn.Sequential(*[Block17(scale=0.10) for _ in range(10)])
        self.mixed_7a = Mixed_7a()
        self.repeat_3 = nn.Sequential(*[Block8(scale=0.20) for _ in range(5)])
        self.block8 = Block8(noReLU=True)
        self.avgpool_1a = nn.AdaptiveAvgPool2d(1)
        self.dropout = nn.Dropout(0.6)
        self.last_linear = nn.Linear(1792, 512, bias=False)
        self.last_bn = nn.BatchNorm1d(512, eps=0.001, momentum=0.1, affine=True)

    def forward(self, x):
        x = self.conv2d_4b(self.conv2d_4a(self.conv2d_3b(self.maxpool_3a(self.conv2d_2b(self.conv2d_2a(
            self.conv2d_1a(x)))))))
        x = self.mixed_7a(self.repeat_2(self.mixed_6a(self.repeat_1(x))))
        x = self.block8(self.repeat_3(x))
        x = self.dropout(self.avgpool_1a(x))
        x = self.last_bn(self.last_linear(x.view(x.shape[0], -1)))
        return F.normalize(x, p=2, dim=1)


class FaceNetModel(nn.Module):
    """facenet_model.py:7-36 (pretrained weights replaced by a state_dict load)."""

    def __init__(self, embedding_size=512):
        super().__init__()
        self.model = InceptionResnetV1()
        self.projection = nn.Linear(512, embedding_size) if embedding_size != 512 else None

    def forward(self, x):
        e = self.model(x)
        if self.projection is not None:
            e = self.projection(e)
        return F.normalize(e, p=2, dim=1)


# ------------------------------------------------------------------ helpers
def build_model(arch: str, state_dict=None, num_classes: int = 100) -> nn.Module:
    if arch == "resnet50_arcface":
        m = ArcFaceModel(num_classes=num_classes)
    elif arch == "iresnet100":
        m = IResNet100()
    elif arch == "irv1_facenet":
        emb = 512
        if state_dict is not None and "projection.weight" in state_dict:
            emb = int(np.asarray(state_dict["projection.weight"]).shape[0])
        m = FaceNetModel(embedding_size=emb)
    else:
        raise ValueError(arch)
    if state_dict is not None:
        sd = {k: torch.as_tensor(np.asarray(v)) for k, v in state_dict.items()}
        m.load_state_dict(sd, strict=True)
    return m.eval()


def preprocess_u8_nhwc(u8: np.ndarray) -> torch.Tensor:
    """get_transform() on an already-sized crop (extract_embeddings.py:170-176):
    Resize is the identity, ToTensor = u8/255 (HWC→CHW), Normalize(0.5, 0.5)."""
    x = torch.from_numpy(np.ascontiguousarray(u8)).float().div(255)
    x = x.permute(0, 3, 1, 2).contiguous()
    return (x - 0.5) / 0.5


@torch.no_grad()
def embed(model: nn.Module, arch: str, u8: np.ndarray, normalize: bool = True, batch: int = 64) -> np.ndarray:
    """model(x, labels=None) → F.normalize (extract_embeddings.py:377-382, :430-435)."""
    outs = []
    for i in range(0, len(u8), batch):
        x = preprocess_u8_nhwc(u8[i:i + batch])
        e = model(x) if arch == "irv1_facenet" else model(x, labels=None)
        if normalize:
            e = F.normalize(e, p=2, dim=1)
        outs.append(e.numpy())
    return np.concatenate(outs, 0).astype(np.float32)


@torch.no_grad()
def calibrate_bn(model: nn.Module, x: torch.Tensor) -> dict:
    """One train-mode pass with cumulative BN averaging (momentum=None) → running stats."""
    bns = [m for m in model.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
    for m in bns:
        m.reset_running_stats()
        m.momentum = None
    model.train()
    for m in model.modules():  # calibrate the eval-mode graph: dropout stays the identity
        if isinstance(m, nn.Dropout):
            m.eval()
    model(x) if isinstance(model, FaceNetModel) else model(x, labels=None)
    model.eval()
    out = {}
    for name, m in model.named_modules():
        if isinstance(m, nn.modules.batchnorm._BatchNorm):
            out[name + ".running_mean"] = m.running_mean.numpy().astype(np.float32).copy()
            out[name + ".running_var"] = m.running_var.numpy().astype(np.float32).copy()
    return out
