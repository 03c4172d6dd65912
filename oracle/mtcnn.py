"""CPU restatement of the reference's face detector (TEST INFRASTRUCTURE ONLY: imported by tests/ and
tools/, never by the product path in facerecognition_amd/).

The reference detects with facenet-pytorch's MTCNN (`preprocessing/face_detector.py:78-97`:
``MTCNN(image_size=160, margin=0, min_face_size=20, thresholds=[0.6, 0.7, 0.7], factor=0.709,
post_process=False, keep_all=True)``, select_largest left at its default True) and then keeps the most
confident-enough, large-enough face (`_detect_mtcnn`, `:144-210`).  facenet-pytorch (requirements.txt:20,
``facenet-pytorch>=2.5.2``) is absent from /root/reference and from this image; this module restates its
published 2.5.x algorithm (``models/mtcnn.py`` PNet/RNet/ONet, ``models/utils/detect_face.py``
detect_face / generateBoundingBox / bbreg / rerec / pad / imresample / nms) with torchvision's
``batched_nms`` (also absent) restated as the greedy IoU suppression it is.  No reference test or fixture
pins MTCNN outputs, and its pretrained P/R/O-net weights are not in the reference: parity of the device
detector against this restatement is **parity unpinned** (DESIGN.md §2), on synthetic weights.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

THRESHOLDS = (0.6, 0.7, 0.7)
FACTOR = 0.709
MIN_FACE = 20


class PNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1, self.prelu1 = nn.Conv2d(3, 10, 3), nn.PReLU(10)
        self.pool1 = nn.MaxPool2d(2, 2, ceil_mode=True)
        self.conv2, self.prelu2 = nn.Conv2d(10, 16, 3), nn.PReLU(16)
        self.conv3, self.prelu3 = nn.Conv2d(16, 32, 3), nn.PReLU(32)
        self.conv4_1, self.conv4_2 = nn.Conv2d(32, 2, 1), nn.Conv2d(32, 4, 1)

    def forward(self, x):
        x = self.pool1(self.prelu1(self.conv1(x)))
        x = self.prelu3(self.conv3(self.prelu2(self.conv2(x))))
        return self.conv4_2(x), F.softmax(self.conv4_1(x), dim=1)


class RNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1, self.prelu1 = nn.Conv2d(3, 28, 3), nn.PReLU(28)
        self.pool1 = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.conv2, self.prelu2 = nn.Conv2d(28, 48, 3), nn.PReLU(48)
        self.pool2 = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.conv3, self.prelu3 = nn.Conv2d(48, 64, 2), nn.PReLU(64)
        self.dense4, self.prelu4 = nn.Linear(576, 128), nn.PReLU(128)
        self.dense5_1, self.dense5_2 = nn.Linear(128, 2), nn.Linear(128, 4)

    def forward(self, x):
        x = self.pool1(self.prelu1(self.conv1(x)))
        x = self.pool2(self.prelu2(self.conv2(x)))
        x = self.prelu3(self.conv3(x)).permute(0, 3, 2, 1).contiguous()
        x = self.prelu4(self.dense4(x.view(x.shape[0], -1)))
        return self.dense5_2(x), F.softmax(self.dense5_1(x), dim=1)


class ONet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1, self.prelu1 = nn.Conv2d(3, 32, 3), nn.PReLU(32)
        self.pool1 = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.conv2, self.prelu2 = nn.Conv2d(32, 64, 3), nn.PReLU(64)
        self.pool2 = nn.MaxPool2d(3, 2, ceil_mode=True)
        self.conv3, self.prelu3 = nn.Conv2d(64, 64, 3), nn.PReLU(64)
        self.pool3 = nn.MaxPool2d(2, 2, ceil_mode=True)
        self.conv4, self.prelu4 = nn.Conv2d(64, 128, 2), nn.PReLU(128)
        self.dense5, self.prelu5 = nn.Linear(1152, 256), nn.PReLU(256)
        self.dense6_1, self.dense6_2, self.dense6_3 = nn.Linear(256, 2), nn.Linear(256, 4), nn.Linear(256, 10)

    def forward(self, x):
        x = self.pool1(self.prelu1(self.conv1(x)))
        x = self.pool2(self.prelu2(self.conv2(x)))
        x = self.pool3(self.prelu3(self.conv3(x)))
        x = self.prelu4(self.conv4(x)).permute(0, 3, 2, 1).contiguous()
        x = self.prelu5(self.dense5(x.view(x.shape[0], -1)))
        return self.dense6_2(x), self.dense6_3(x), F.softmax(self.dense6_1(x), dim=1)


def build_nets(state: dict):
    """P/R/O-nets (eval, fp32) from a {"pnet.<param>": array, "rnet.…", "onet.…"} dict."""
    nets = {"pnet": PNet(), "rnet": RNet(), "onet": ONet()}
    for name, net in nets.items():
        sd = {k[len(name) + 1:]: torch.as_tensor(np.asarray(v, np.float32)) for k, v in state.items()
              if k.startswith(name + ".")}
        net.load_state_dict(sd, strict=True)
        net.eval()
    return nets["pnet"], nets["rnet"], nets["onet"]


def imresample(img, sz):
    """detect_face.imresample: F.interpolate(mode='area')."""
    return F.interpolate(img, size=sz, mode="area")


def generate_bounding_box(reg, probs, scale, thresh):
    """detect_face.generateBoundingBox (stride 2, cell 12)."""
    stride, cellsize = 2, 12
    reg = reg.permute(1, 0, 2, 3)
    mask = probs >= thresh
    mask_inds = mask.nonzero()
    image_inds = mask_inds[:, 0]
    score = probs[mask]
    reg = reg[:, mask].permute(1, 0)
    bb = mask_inds[:, 1:].type(reg.dtype).flip(1)
    q1 = ((stride * bb + 1) / scale).floor()
    q2 = ((stride * bb + cellsize - 1 + 1) / scale).floor()
    return torch.cat([q1, q2, score.unsqueeze(1), reg], dim=1), image_inds


def nms_iou(boxes: np.ndarray, scores: np.ndarray, thresh: float) -> np.ndarray:
    """torchvision.ops.nms: greedy, by score descending (stable: lower index first among equal scores),
    suppress IoU > thresh, IoU with areas (x2 - x1) * (y2 - y1)."""
    order = np.argsort(-scores, kind="stable")
    x1, y1, x2, y2 = boxes.T
    area = (x2 - x1) * (y2 - y1)
    keep = []
    alive = np.ones(len(order), bool)
    for a, i in enumerate(order):
        if not alive[a]:
            continue
        keep.append(i)
        rest = order[a + 1:]
        xx1, yy1 = np.maximum(x1[i], x1[rest]), np.maximum(y1[i], y1[rest])
        xx2, yy2 = np.minimum(x2[i], x2[rest]), np.minimum(y2[i], y2[rest])
        inter = np.clip(xx2 - xx1, 0, None) * np.clip(yy2 - yy1, 0, None)
        iou = inter / (area[i] + area[rest] - inter)
        alive[a + 1:] &= ~(iou > thresh)
    return np.asarray(keep, np.int64)


def batched_nms(boxes, scores, idxs, thresh):
    """torchvision.ops.batched_nms (the coordinate-offset trick: per-image NMS)."""
    if boxes.numel() == 0:
        return torch.empty((0,), dtype=torch.int64)
    off = idxs.to(boxes) * (boxes.max() + 1)
    b = (boxes + off[:, None]).numpy().astype(np.float32)
    return torch.as_tensor(nms_iou(b, scores.numpy().astype(np.float32), thresh))


def nms_numpy(boxes, scores, threshold, method):
    """detect_face.nms_numpy (the ONet stage's 'Min' NMS; +1 pixel areas; np.argsort ascending)."""
    if boxes.size == 0:
        return np.empty((0,), np.int64)
    x1, y1, x2, y2 = (boxes[:, i].copy() for i in range(4))
    area = (x2 - x1 + 1) * (y2 - y1 + 1)
    I = np.argsort(scores)
    pick = []
    while I.size > 0:
        i = I[-1]
        pick.append(i)
        idx = I[0:-1]
        xx1, yy1 = np.maximum(x1[i], x1[idx]), np.maximum(y1[i], y1[idx])
        xx2, yy2 = np.minimum(x2[i], x2[idx]), np.minimum(y2[i], y2[idx])
        w, h = np.maximum(0.0, xx2 - xx1 + 1), np.maximum(0.0, yy2 - yy1 + 1)
        inter = w * h
        o = inter / np.minimum(area[i], area[idx]) if method == "Min" else inter / (area[i] + area[idx] - inter)
        I = I[np.where(o <= threshold)]
    return np.asarray(pick, np.int64)


def batched_nms_numpy(boxes, scores, idxs, threshold, method):
    if boxes.numel() == 0:
        return torch.empty((0,), dtype=torch.int64)
    off = idxs.to(boxes) * (boxes.max() + 1)
    b = (boxes + off[:, None]).numpy()
    return torch.as_tensor(nms_numpy(b, scores.numpy(), threshold, method), dtype=torch.long)


def bbreg(boundingbox, reg):
    w = boundingbox[:, 2] - boundingbox[:, 0] + 1
    h = boundingbox[:, 3] - boundingbox[:, 1] + 1
    b1 = boundingbox[:, 0] + reg[:, 0] * w
    b2 = boundingbox[:, 1] + reg[:, 1] * h
    b3 = boundingbox[:, 2] + reg[:, 2] * w
    b4 = boundingbox[:, 3] + reg[:, 3] * h
    boundingbox[:, :4] = torch.stack([b1, b2, b3, b4]).permute(1, 0)
    return boundingbox


def rerec(b):
    h = b[:, 3] - b[:, 1]
    w = b[:, 2] - b[:, 0]
    l = torch.max(w, h)
    b[:, 0] = b[:, 0] + w * 0.5 - l * 0.5
    b[:, 1] = b[:, 1] + h * 0.5 - l * 0.5
    b[:, 2:4] = b[:, :2] + l.repeat(2, 1).permute(1, 0)
    return b


def pad(boxes, w, h):
    boxes = boxes.trunc().int().numpy()
    x, y, ex, ey = boxes[:, 0], boxes[:, 1], boxes[:, 2], boxes[:, 3]
    x[x < 1] = 1
    y[y < 1] = 1
    ex[ex > w] = w
    ey[ey > h] = h
    return y, ey, x, ex


def pyramid_scales(h: int, w: int, minsize: int = MIN_FACE, factor: float = FACTOR):
    m = 12.0 / minsize
    minl = min(h, w) * m
    scales, s = [], m
    while minl >= 12:
        scales.append(s)
        s *= factor
        minl *= factor
    return scales


def _crops(imgs, boxes, image_inds, w, h, size):
    y, ey, x, ex = pad(boxes, w, h)
    out = []
    for k in range(len(y)):
        if ey[k] > (y[k] - 1) and ex[k] > (x[k] - 1):
            img_k = imgs[image_inds[k], :, (y[k] - 1):ey[k], (x[k] - 1):ex[k]].unsqueeze(0)
            out.append(imresample(img_k, (size, size)))
    return (torch.cat(out, 0) - 127.5) * 0.0078125


def detect_face(imgs_u8: np.ndarray, pnet, rnet, onet, minsize=MIN_FACE, threshold=THRESHOLDS, factor=FACTOR):
    """detect_face on a batch of equal-size RGB u8 images [B, H, W, 3] -> (boxes [B] of [n, 5] = x1, y1, x2,
    y2, prob; points [B] of [n, 5, 2])."""
    with torch.no_grad():
        imgs = torch.as_tensor(np.ascontiguousarray(imgs_u8)).permute(0, 3, 1, 2).float()
        B = len(imgs)
        h, w = imgs.shape[2:4]
        boxes, image_inds, scale_picks, offset = [], [], [], 0
        for scale in pyramid_scales(h, w, minsize, factor):
            im = (imresample(imgs, (int(h * scale + 1), int(w * scale + 1))) - 127.5) * 0.0078125
            reg, probs = pnet(im)
            bs, ii = generate_bounding_box(reg, probs[:, 1], scale, threshold[0])
            boxes.append(bs)
            image_inds.append(ii)
            scale_picks.append(batched_nms(bs[:, :4], bs[:, 4], ii, 0.5) + offset)
            offset += bs.shape[0]
        boxes, image_inds = torch.cat(boxes, 0), torch.cat(image_inds, 0)
        scale_picks = torch.cat(scale_picks, 0)
        boxes, image_inds = boxes[scale_picks], image_inds[scale_picks]
        pick = batched_nms(boxes[:, :4], boxes[:, 4], image_inds, 0.7)
        boxes, image_inds = boxes[pick], image_inds[pick]
        regw, regh = boxes[:, 2] - boxes[:, 0], boxes[:, 3] - boxes[:, 1]
        boxes = torch.stack([boxes[:, 0] + boxes[:, 5] * regw, boxes[:, 1] + boxes[:, 6] * regh,
                             boxes[:, 2] + boxes[:, 7] * regw, boxes[:, 3] + boxes[:, 8] * regh,
                             boxes[:, 4]]).permute(1, 0)
        boxes = rerec(boxes)
        if len(boxes) > 0:
            out = rnet(_crops(imgs, boxes, image_inds, w, h, 24))
            score = out[1][:, 1]
            ipass = score > threshold[1]
            boxes = torch.cat((boxes[ipass, :4], score[ipass].unsqueeze(1)), dim=1)
            image_inds, mv = image_inds[ipass], out[0][ipass]
            pick = batched_nms(boxes[:, :4], boxes[:, 4], image_inds, 0.7)
            boxes, image_inds, mv = boxes[pick], image_inds[pick], mv[pick]
            boxes = rerec(bbreg(boxes, mv))
        points = torch.zeros(0, 5, 2)
        if len(boxes) > 0:
            out = onet(_crops(imgs, boxes, image_inds, w, h, 48))
            score = out[2][:, 1]
            ipass = score > threshold[2]
            pts = out[1][ipass].permute(1, 0)
            boxes = torch.cat((boxes[ipass, :4], score[ipass].unsqueeze(1)), dim=1)
            image_inds, mv = image_inds[ipass], out[0][ipass]
            w_i = boxes[:, 2] - boxes[:, 0] + 1
            h_i = boxes[:, 3] - boxes[:, 1] + 1
            px = w_i.repeat(5, 1) * pts[:5, :] + boxes[:, 0].repeat(5, 1) - 1
            py = h_i.repeat(5, 1) * pts[5:10, :] + boxes[:, 1].repeat(5, 1) - 1
            points = torch.stack((px, py)).permute(2, 1, 0)
            boxes = bbreg(boxes, mv)
            pick = batched_nms_numpy(boxes[:, :4], boxes[:, 4], image_inds, 0.7, "Min")
            boxes, image_inds, points = boxes[pick], image_inds[pick], points[pick]
        boxes, points, image_inds = boxes.numpy(), points.numpy(), image_inds.numpy()
        return ([boxes[image_inds == b].copy() for b in range(B)], [points[image_inds == b].copy() for b in range(B)])


def mtcnn_detect(img_rgb_u8: np.ndarray, nets, select_largest: bool = True):
    """MTCNN.detect(img, landmarks=True) for one image: (boxes [n, 4] or None, probs, points [n, 5, 2]),
    largest box first when select_largest (facenet-pytorch's default)."""
    boxes, points = detect_face(img_rgb_u8[None], *nets)
    box, point = boxes[0], points[0]
    if len(box) == 0:
        return None, [None], None
    if select_largest:
        order = np.argsort((box[:, 2] - box[:, 0]) * (box[:, 3] - box[:, 1]))[::-1]
        box, point = box[order], point[order]
    return box[:, :4], box[:, 4], point


def face_detector_detect(img_bgr_u8: np.ndarray, nets, confidence_threshold=0.9, min_face_size=MIN_FACE,
                         select_largest=True):
    """The reference's FaceDetector._detect_mtcnn (preprocessing/face_detector.py:144-210) on top of
    mtcnn_detect: BGR -> RGB, confidence >= threshold, min(w, h) >= min_face_size, the largest (or the
    first) survivor; bbox ints, landmarks as named points."""
    rgb = np.ascontiguousarray(img_bgr_u8[..., ::-1])
    boxes, probs, lms = mtcnn_detect(rgb, nets)
    if boxes is None or len(boxes) == 0:
        return None
    valid = np.asarray(probs) >= confidence_threshold
    if not np.any(valid):
        return None
    boxes, probs, lms = boxes[valid], np.asarray(probs)[valid], lms[valid]
    faces = [i for i, b in enumerate(boxes) if min(b[2] - b[0], b[3] - b[1]) >= min_face_size]
    if not faces:
        return None
    if select_largest and len(faces) > 1:
        best = faces[int(np.argmax([(boxes[i][2] - boxes[i][0]) * (boxes[i][3] - boxes[i][1]) for i in faces]))]
    else:
        best = faces[0]
    b, lm = boxes[best], lms[best]
    names = ("left_eye", "right_eye", "nose", "left_mouth", "right_mouth")
    return {"bbox": [int(b[0]), int(b[1]), int(b[2]), int(b[3])], "confidence": float(probs[best]),
            "landmarks": {n: (float(lm[k][0]), float(lm[k][1])) for k, n in enumerate(names)}}
