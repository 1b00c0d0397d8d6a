"""Deterministic synthetic weights and episodes for the CWT episode path.

There are no datasets or checkpoints offline, so parity and
benchmarks run on PRNG-filled weights and PASCAL/COCO-shaped synthetic episodes.
Everything here is a pure function of (seed, name, index) through a counter-based
splitmix64 generator, so the GPU box regenerates exactly what the golden fixtures
were produced from in the survey container, without shipping any weight blob.

State-dict keys and shapes follow the reference modules exactly:
  * ``PSPNet.state_dict()``          — reference src/model/pspnet.py:70-141 with the
    ResNet Bottleneck/stem of src/model/resnet.py:57-147 (``gamma`` first, pspnet.py:141)
  * ``MultiHeadAttentionOne``        — reference src/model/transformer.py:38-52
so either side can ``load_state_dict`` the same dictionary.
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Dict, List, Tuple

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

# ResNet depth -> blocks per stage (reference src/model/resnet.py:198,210)
RESNET_BLOCKS = {50: (3, 4, 6, 3), 101: (3, 4, 23, 3)}
PPM_BINS = (1, 2, 3, 6)                 # config_files/pascal.yaml:48
BN_EPS = 1e-5                           # nn.BatchNorm2d default
IMG_MEAN = (0.485, 0.456, 0.406)        # config_files/pascal.yaml:15
IMG_STD = (0.229, 0.224, 0.225)         # config_files/pascal.yaml:16
# FG ratios of PASCAL split-0 val classes 1..5 (reference src/dataset/classes.py:89-93 comments)
PASCAL_FG_RATIO = (0.14, 0.07, 0.13, 0.12, 0.15)


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def uniform01(seed: int, stream: str, n: int) -> np.ndarray:
    """n float64 values in [0, 1): splitmix64(key + (i+1)*golden)."""
    key = np.uint64((_fnv1a64(stream) ^ (seed * 0x2545F4914F6CDD1D)) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        idx = np.arange(1, n + 1, dtype=np.uint64)
        z = _mix(key + idx * _GOLD)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def uniform(seed: int, stream: str, shape, lo: float, hi: float) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    return (lo + (hi - lo) * uniform01(seed, stream, n)).reshape(shape).astype(np.float32)


def normal(seed: int, stream: str, shape, std: float = 1.0, mean: float = 0.0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform01(seed, stream, 2 * n)
    u1, u2 = u[0::2], u[1::2]
    z = np.sqrt(-2.0 * np.log1p(-u1)) * np.cos(2.0 * math.pi * u2)
    return (mean + std * z).reshape(shape).astype(np.float32)


# --------------------------------------------------------------------------------------
# PSPNet / ResNet parameter layout (names + shapes in reference state_dict order)
# --------------------------------------------------------------------------------------

def _bn_keys(prefix: str, c: int) -> List[Tuple[str, tuple, str]]:
    return [(f"{prefix}.weight", (c,), "bn_w"), (f"{prefix}.bias", (c,), "bn_b"),
            (f"{prefix}.running_mean", (c,), "bn_rm"), (f"{prefix}.running_var", (c,), "bn_rv"),
            (f"{prefix}.num_batches_tracked", (), "bn_nbt")]


def pspnet_param_specs(layers: int = 50, bottleneck_dim: int = 512,
                       num_classes_tr: int = 2) -> List[Tuple[str, tuple, str]]:
    """(name, shape, kind) for every entry of reference ``PSPNet.state_dict()``."""
    specs: List[Tuple[str, tuple, str]] = [("gamma", (), "gamma")]
    # layer0: deep-base stem (resnet.py:110-118, pspnet.py:93-95)
    specs += [("layer0.0.weight", (64, 3, 3, 3), "conv")] + _bn_keys("layer0.1", 64)
    specs += [("layer0.3.weight", (64, 64, 3, 3), "conv")] + _bn_keys("layer0.4", 64)
    specs += [("layer0.6.weight", (128, 64, 3, 3), "conv")] + _bn_keys("layer0.7", 128)
    inplanes = 128
    for li, (planes, nblk) in enumerate(zip((64, 128, 256, 512), RESNET_BLOCKS[layers]), start=1):
        for b in range(nblk):
            p = f"layer{li}.{b}"
            specs += [(f"{p}.conv1.weight", (planes, inplanes, 1, 1), "conv")] + _bn_keys(f"{p}.bn1", planes)
            specs += [(f"{p}.conv2.weight", (planes, planes, 3, 3), "conv")] + _bn_keys(f"{p}.bn2", planes)
            specs += [(f"{p}.conv3.weight", (planes * 4, planes, 1, 1), "conv")] + _bn_keys(f"{p}.bn3", planes * 4)
            if b == 0:
                specs += [(f"{p}.downsample.0.weight", (planes * 4, inplanes, 1, 1), "conv")]
                specs += _bn_keys(f"{p}.downsample.1", planes * 4)
            inplanes = planes * 4
    red = 2048 // len(PPM_BINS)
    for i in range(len(PPM_BINS)):
        specs += [(f"ppm.features.{i}.1.weight", (red, 2048, 1, 1), "conv")]
        specs += _bn_keys(f"ppm.features.{i}.2", red)
    specs += [("bottleneck.0.weight", (bottleneck_dim, 4096, 3, 3), "conv")]
    specs += _bn_keys("bottleneck.1", bottleneck_dim)
    specs += [("classifier.weight", (num_classes_tr, bottleneck_dim, 1, 1), "cls")]
    return specs


def _damped_bn(name: str) -> bool:
    # last BN of a residual branch and the shortcut BN: keep the residual stream tame
    return name.endswith(".bn3.weight") or name.endswith("downsample.1.weight")


def make_pspnet_state(layers: int = 50, seed: int = 2021, bottleneck_dim: int = 512,
                      num_classes_tr: int = 2) -> "OrderedDict[str, np.ndarray]":
    """Synthetic frozen backbone: Kaiming(fan_in) convs, non-trivial eval-mode BN."""
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    for name, shape, kind in pspnet_param_specs(layers, bottleneck_dim, num_classes_tr):
        if kind == "gamma":
            sd[name] = np.array(0.2, dtype=np.float32)
        elif kind == "conv":
            fan_in = shape[1] * shape[2] * shape[3]
            sd[name] = normal(seed, name, shape, std=math.sqrt(2.0 / fan_in))
        elif kind == "cls":
            sd[name] = normal(seed, name, shape, std=math.sqrt(1.0 / shape[1]))
        elif kind == "bn_w":
            lo, hi = (0.2, 0.4) if _damped_bn(name) else (0.6, 1.0)
            sd[name] = uniform(seed, name, shape, lo, hi)
        elif kind == "bn_b":
            sd[name] = normal(seed, name, shape, std=0.05)
        elif kind == "bn_rm":
            sd[name] = normal(seed, name, shape, std=0.1)
        elif kind == "bn_rv":
            sd[name] = uniform(seed, name, shape, 0.5, 1.5)
        elif kind == "bn_nbt":
            sd[name] = np.array(0, dtype=np.int64)
        else:
            raise ValueError(kind)
    return sd


def transformer_param_specs(heads: int = 4, d_model: int = 512) -> List[Tuple[str, tuple]]:
    """Reference MultiHeadAttentionOne state_dict (transformer.py:44-52), d_k = d_v = d_model."""
    return [("w_qkvs.weight", (heads * d_model, d_model)),
            ("layer_norm.weight", (d_model,)), ("layer_norm.bias", (d_model,)),
            ("fc.weight", (d_model, heads * d_model)), ("fc.bias", (d_model,))]


def make_transformer_state(heads: int = 4, d_model: int = 512,
                           seed: int = 2021) -> "OrderedDict[str, np.ndarray]":
    """Init as transformer.py:45,51 (normal std sqrt(2/(d_model+d_k)), xavier fc) with a
    perturbed LayerNorm so the affine path is exercised."""
    s = seed + 7919
    sd: "OrderedDict[str, np.ndarray]" = OrderedDict()
    sd["w_qkvs.weight"] = normal(s, "w_qkvs", (heads * d_model, d_model), std=math.sqrt(2.0 / (2 * d_model)))
    sd["layer_norm.weight"] = uniform(s, "ln_w", (d_model,), 0.8, 1.2)
    sd["layer_norm.bias"] = normal(s, "ln_b", (d_model,), std=0.05)
    fan_in, fan_out = heads * d_model, d_model
    sd["fc.weight"] = normal(s, "fc_w", (d_model, heads * d_model), std=math.sqrt(2.0 / (fan_in + fan_out)))
    b = 1.0 / math.sqrt(fan_in)
    sd["fc.bias"] = uniform(s, "fc_b", (d_model,), -b, b)
    return sd


# --------------------------------------------------------------------------------------
# Episodes
# --------------------------------------------------------------------------------------

def feature_side(image_size: int) -> int:
    """h = (S-1)/8 + 1 (pspnet.py:150 assert; test.py:116-119)."""
    assert (image_size - 1) % 8 == 0, image_size
    return (image_size - 1) // 8 + 1


def _content_side(S: int) -> int:
    # reference Resize (transform.py:128-135): longest side -> S, then floor to a multiple of 8
    return S if S % 8 == 0 else (S // 8) * 8


def make_image_and_mask(seed: int, stream: str, S: int, fg_ratio: float) -> Tuple[np.ndarray, np.ndarray]:
    """One normalised image [3,S,S] f32 and label [S,S] int64 (0 BG, 1 FG, 255 pad).

    Mimics the reference pipeline (dataset.py:205-327): content occupies the top-left
    c x c block (c = S floored to /8), the rest is zero-padded image / 255 label; the image
    is ToTensor (/255) + Normalize (transform.py:70-72,102-103)."""
    c = _content_side(S)
    r = uniform01(seed, stream + "/ell", 8)
    area = fg_ratio * c * c
    aspect = 0.6 + 0.8 * r[0]
    ry = math.sqrt(area / math.pi * aspect)
    rx = math.sqrt(area / math.pi / aspect)
    cy = ry + (c - 2 * ry) * r[1]
    cx = rx + (c - 2 * rx) * r[2]
    yy, xx = np.mgrid[0:c, 0:c].astype(np.float64)
    fg = ((yy - cy) / ry) ** 2 + ((xx - cx) / rx) ** 2 <= 1.0
    label = np.full((S, S), 255, dtype=np.int64)
    label[:c, :c] = fg.astype(np.int64)
    # smooth background texture + per-image FG colour + pixel noise, quantised to uint8
    fy, fx, ph = 2 + 6 * r[3], 2 + 6 * r[4], 2 * math.pi * r[5]
    base = 0.5 + 0.2 * np.sin(2 * math.pi * fy * yy / c + ph) * np.cos(2 * math.pi * fx * xx / c)
    noise = uniform(seed, stream + "/px", (3, c, c), -0.15, 0.15)
    fg_col = uniform(seed, stream + "/fgc", (3,), -0.3, 0.3)
    img_u8 = np.zeros((3, S, S), dtype=np.float32)
    for ch in range(3):
        v = base + noise[ch] + fg * fg_col[ch]
        img_u8[ch, :c, :c] = np.floor(np.clip(v, 0.0, 1.0) * 255.0)
    img = img_u8 / np.float32(255.0)
    for ch in range(3):
        img[ch] = (img[ch] - np.float32(IMG_MEAN[ch])) / np.float32(IMG_STD[ch])
    return img.astype(np.float32), label


def pascal_val_classes(split: int = 0) -> List[int]:
    return list(range(5 * split + 1, 5 * split + 6))


def coco_val_classes(split: int = 0) -> List[int]:
    # use_split_coco split-0 val classes: range(1, 78, 4) (classes.py:135-137)
    return list(range(split + 1, 81, 4))


def make_episode(seed: int, index: int, S: int = 473, shot: int = 1,
                 classes: List[int] = None) -> dict:
    """Synthetic episode in the reference loader's 7-tuple shapes (dataset.py:326-327),
    as numpy arrays: qry_img [1,3,S,S], q_label [1,S,S], spprt_imgs [1,shot,3,S,S],
    s_label [1,shot,S,S], subcls [int]."""
    classes = classes or pascal_val_classes(0)
    cls = classes[index % len(classes)]
    ratio = PASCAL_FG_RATIO[(cls - 1) % len(PASCAL_FG_RATIO)]
    stream = f"ep{index}"
    qi, ql = make_image_and_mask(seed, stream + "/q", S, ratio)
    simgs, slabs = [], []
    for k in range(shot):
        si, sl = make_image_and_mask(seed, stream + f"/s{k}", S, ratio)
        simgs.append(si)
        slabs.append(sl)
    return dict(qry_img=qi[None], q_label=ql[None], spprt_imgs=np.stack(simgs)[None],
                s_label=np.stack(slabs)[None], subcls=[cls])


def cfg_defaults(**over) -> Dict:
    """The CWT configuration the reference is measured with: config_files/pascal.yaml
    merged with the scripts/test.sh / train.sh overrides (heads 4, cls_lr 0.1, ...)."""
    cfg = dict(image_size=473, layers=50, shot=1, heads=4, cls_lr=0.1, trans_lr=0.001,
               scale_lr=1.0, adapt_iter=200, bottleneck_dim=512, num_classes_tr=2,
               bins=list(PPM_BINS), dropout=0.1, m_scale=False, arch="resnet",
               batch_size=1, batch_size_val=1, manual_seed=2021, momentum=0.9,
               weight_decay=0.0001, nesterov=True, main_optim="SGD", test_num=1000,
               n_runs=1, train_name="pascal", train_split=0, cls_type="oooo",
               distributed=False)
    cfg.update(over)
    return cfg
