"""Episode data path: the reference's episodic loader with its
transforms on the device.

Host side, restated from src/dataset/: the PASCAL-5i / COCO-20i class splits
(classes.py:119-199), ``make_dataset`` / ``process_image`` (utils.py:27-118: keep an image for a
class only with >= 2*32*32 pixels of it), and ``EpisodicData.__getitem__``
(dataset.py:205-327) with the SAME random calls in the same order -- ``np.random.choice`` for
the query class, ``random.randint`` for the supports (distinct, never the query), and one
``random.random()`` per flip augmentation per image (transform.py:403-422) -- so a seeded run
draws the same episodes as the reference's loader.

Device side: each decoded image / label is uploaded once and Resize + ToTensor + Normalize
(+ flips) and the label remap / nearest resize / padding run as the HIP kernels of
csrc/preprocess.hip (cwt_preprocess_image / cwt_preprocess_label), writing the episode
tensors the extractor reads.  There is no JPEG/PNG decoder in this image (cv2 and PIL are
absent): images and labels are read through ``read_image`` / ``read_label`` callables (the
default reads ``.npy`` arrays: HxWx3 RGB uint8 and HxW uint8).
"""
from __future__ import annotations

import os
import random
from collections import defaultdict
from typing import Callable, Dict, List, Tuple

import numpy as np
import torch

from . import _lib


def _g(args, k, default=None):
    if isinstance(args, dict):
        return args.get(k, default)
    return getattr(args, k, default) if hasattr(args, k) else default


# -------------------------------------------------------------------------------- splits
def get_split_classes(args) -> Dict:
    """classes.py:119-165: split_classes[name][split]['train' | 'val']."""
    split_classes = {"coco": defaultdict(dict), "pascal": defaultdict(dict)}
    class_list = list(range(1, 81))
    split_classes["coco"][-1]["val"] = class_list
    if _g(args, "use_split_coco", False):
        vals = [list(range(1, 78, 4)), list(range(2, 79, 4)), list(range(3, 80, 4)), list(range(4, 81, 4))]
    else:
        vals = [list(range(1, 21)), list(range(21, 41)), list(range(41, 61)), list(range(61, 81))]
    for i, v in enumerate(vals):
        split_classes["coco"][i]["val"] = v
        split_classes["coco"][i]["train"] = list(set(class_list) - set(v))
    class_list = list(range(1, 21))
    split_classes["pascal"][-1]["val"] = class_list
    for i, v in enumerate([list(range(1, 6)), list(range(6, 11)), list(range(11, 16)), list(range(16, 21))]):
        split_classes["pascal"][i]["val"] = v
        split_classes["pascal"][i]["train"] = list(set(class_list) - set(v))
    return split_classes


def filter_classes(train_name: str, train_split: int, test_name: str, test_split: int, split_classes: Dict) -> List[int]:
    """classes.py:168-199 for the in-domain case (test_name == train_name, the CWT scripts):
    the test split's val classes minus those seen in training.  Cross-domain runs compare class
    NAMES between datasets (the name tables are not restated): NotImplementedError."""
    if test_name != train_name:
        raise NotImplementedError("cross-domain class filtering (pascal <-> coco) is not on the CWT path")
    seen = set(split_classes[train_name][train_split]["train"])
    return [c for c in split_classes[test_name][test_split]["val"] if c not in seen]


# -------------------------------------------------------------------------------- readers
def read_npy(path: str) -> np.ndarray:
    """Default reader: a .npy array (no pickles)."""
    if not path.endswith(".npy"):
        raise RuntimeError(f"{path}: no image decoder in this environment (cv2 / PIL absent); pass read_image / "
                           "read_label callables or use .npy arrays")
    return np.load(path, allow_pickle=False)


def process_image(line: str, data_root: str, class_list: List[int], read_label: Callable = read_npy):
    """utils.py:64-118: (image, label) kept for every class of class_list with >= 2*32*32 pixels."""
    parts = line.strip().split(" ")
    item = (os.path.join(data_root, parts[0]), os.path.join(data_root, parts[1]))
    label = read_label(item[1])
    label_class = np.unique(label).tolist()
    if 0 in label_class:
        label_class.remove(0)
    if 255 in label_class:
        label_class.remove(255)
    for c in label_class:
        assert c in range(1, 81), c
    kept = [c for c in label_class if c in class_list and int((label == c).sum()) >= 2 * 32 * 32]
    image_label_list, class_file_dict = [], defaultdict(list)
    if kept:
        image_label_list.append(item)
        for c in kept:
            class_file_dict[c].append(item)
    return image_label_list, class_file_dict


def make_dataset(data_root: str, data_list: str, class_list: List[int], read_label: Callable = read_npy):
    """utils.py:27-61 (list order preserved, as Pool.map preserves it)."""
    if not os.path.isfile(data_list):
        raise RuntimeError("Image list file do not exist: " + data_list + "\n")
    image_label_list: List[Tuple[str, str]] = []
    class_file_dict: Dict[int, List[Tuple[str, str]]] = defaultdict(list)
    for line in open(data_list).readlines():
        sub, subdict = process_image(line, data_root, class_list, read_label)
        image_label_list += sub
        for k, v in subdict.items():
            class_file_dict[k] += v
    return image_label_list, class_file_dict


# -------------------------------------------------------------------------------- device transforms
def preprocess_image(image: torch.Tensor, S: int, mean, std, padding=None, flip_h=False, flip_v=False,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """Resize(S) + ToTensor + Normalize of one device HWC RGB image (uint8 or fp32) into fp32
    [3, S, S] (cwt_preprocess_image)."""
    if image.dtype not in (torch.uint8, torch.float32) or image.dim() != 3 or image.shape[2] != 3:
        raise TypeError("image must be a HxWx3 uint8 or float32 tensor")
    _lib.require(image, "image", image.dtype)
    image = image.contiguous()
    if out is None:
        out = torch.empty((3, S, S), device=image.device, dtype=torch.float32)
    f3 = _lib.C.c_float * 3
    pad = f3(*[float(p) for p in padding]) if padding else None
    _lib.check(_lib.lib().cwt_preprocess_image(
        _lib.ctx(image.device.index), _lib.ptr(image), 1 if image.dtype == torch.float32 else 0,
        image.shape[0], image.shape[1], S, f3(*[float(m) for m in mean]), f3(*[float(s) for s in std]), pad,
        int(flip_h), int(flip_v), _lib.ptr(out), _lib.stream_ptr(image.device)), "cwt_preprocess_image")
    return out


def preprocess_label(label: torch.Tensor, S: int, class_chosen: int = -1, flip_h=False, flip_v=False,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """Remap (class_chosen -> 1, 255 kept, else 0; < 0 keeps the values) + nearest Resize(S) +
    255 padding of one device HxW uint8 label into int64 [S, S] (cwt_preprocess_label)."""
    _lib.require(label, "label", torch.uint8)
    label = label.contiguous()
    if out is None:
        out = torch.empty((S, S), device=label.device, dtype=torch.int64)
    _lib.check(_lib.lib().cwt_preprocess_label(
        _lib.ctx(label.device.index), _lib.ptr(label), label.shape[0], label.shape[1], S, int(class_chosen),
        int(flip_h), int(flip_v), _lib.ptr(out), _lib.stream_ptr(label.device)), "cwt_preprocess_label")
    return out


def standard_label(label: np.ndarray, class_list: List[int]) -> np.ndarray:
    """StandardData's label remap (dataset.py:144-168): every class of class_list present becomes
    class_list.index(c) + 1, other classes 255, everything else -- including the source's own 255
    void pixels -- background 0 (new_label starts as zeros and the void value is never copied)."""
    label_class = np.unique(label).tolist()
    for v in (0, 255):
        if v in label_class:
            label_class.remove(v)
    wanted = [c for c in label_class if c in class_list]
    unwanted = [c for c in label_class if c not in class_list]
    assert len(wanted) > 0
    new_label = np.zeros_like(label)
    for c in wanted:
        new_label[label == c] = class_list.index(c) + 1
    for c in unwanted:
        new_label[label == c] = 255
    return new_label


class StandardData:
    """dataset.py:120-177 (the non-episodic loader stage-1 pretraining reads, pretrain.py:83) with
    the transforms on the device: ``__getitem__`` returns (image fp32 [3,S,S], label int64 [S,S])
    on ``device`` (+ the paths with ``return_paths``).  The pretraining configs' augmentations are
    hor_flip, vert_flip, resize (pascal_pretrain.yaml / coco_pretrain.yaml); one
    ``random.random()`` per flip as transform.py:403-422 draws it."""

    SUPPORTED_AUG = ("hor_flip", "vert_flip", "resize")

    def __init__(self, args, data_list_path: str, class_list: List[int], return_paths: bool = False,
                 augmentations=None, read_image: Callable = read_npy, read_label: Callable = read_npy, device=None):
        self.S = int(_g(args, "image_size", 473))
        self.mean, self.std = list(_g(args, "mean")), list(_g(args, "std"))
        self.padding = [v * 255 for v in self.mean] if _g(args, "padding") == "avg" else None
        augs = list(augmentations if augmentations is not None else ["resize"])
        bad = [a for a in augs if a not in self.SUPPORTED_AUG]
        if bad or "resize" not in augs:
            raise NotImplementedError(f"augmentations {bad or augs}: the pretraining configs use hor_flip, "
                                      "vert_flip, resize")
        self.flips = [a for a in augs if a != "resize"]
        self.class_list = class_list
        self.return_paths = return_paths
        self.read_image, self.read_label = read_image, read_label
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.data_list, _ = make_dataset(_g(args, "data_root"), data_list_path, class_list, read_label)

    def __len__(self):
        return len(self.data_list)

    def host_item(self, index: int):
        """The decoded image and the remapped label before the transform (host arrays)."""
        image_path, label_path = self.data_list[index]
        image = self.read_image(image_path)
        label = self.read_label(label_path)
        if image.shape[0] != label.shape[0] or image.shape[1] != label.shape[1]:
            raise RuntimeError("Query Image & label shape mismatch: " + image_path + " " + label_path + "\n")
        return image, standard_label(label, self.class_list), image_path, label_path

    def __getitem__(self, index: int):
        image, label, image_path, label_path = self.host_item(index)
        fl = {"hor_flip": False, "vert_flip": False}
        for a in self.flips:
            fl[a] = random.random() < 0.5
        img = torch.from_numpy(np.ascontiguousarray(image)).to(self.device)
        lab = torch.from_numpy(np.ascontiguousarray(label.astype(np.uint8))).to(self.device)
        t = preprocess_image(img, self.S, self.mean, self.std, self.padding, fl["hor_flip"], fl["vert_flip"])
        lt = preprocess_label(lab, self.S, -1, fl["hor_flip"], fl["vert_flip"])
        if self.return_paths:
            return t, lt, image_path, label_path
        return t, lt


def _draw_base_seed() -> None:
    """iter(DataLoader) draws the iterator's base seed from the global torch RNG before the
    sampler draws anything (torch/utils/data/dataloader.py, _BaseDataLoaderIter.__init__; the
    reference's pretrain.py:105 and train.py:188 iterators): consume the same draw, so every later
    torch RNG draw (the shuffle order, W0, dropout seeds) lines up with the reference's."""
    torch.empty((), dtype=torch.int64).random_()


class StandardLoader:
    """``torch.utils.data.DataLoader(StandardData, batch_size, shuffle, sampler, drop_last)``
    (dataset.py:61-68) in the calling process: batches stacked on the device, order from torch's
    RNG as RandomSampler draws it (or the sampler's shard).  The iterator has ``.next()`` like the
    torch-1.6 iterators pretrain.py:105,110 use."""

    def __init__(self, dataset: StandardData, batch_size: int, shuffle: bool, drop_last: bool,
                 sampler: "EpisodeSampler | None" = None):
        self.dataset, self.batch_size, self.drop_last, self.sampler = dataset, int(batch_size), drop_last, sampler
        self.shuffle = shuffle and sampler is None

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.dataset)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self):
        n = len(self.dataset)
        _draw_base_seed()
        if self.sampler is not None:
            order = list(self.sampler)
        elif self.shuffle:
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            order = torch.randperm(n, generator=torch.Generator().manual_seed(seed)).tolist()
        else:
            order = list(range(n))
        nb, bs, ds = len(self), self.batch_size, self.dataset

        class _It:
            def __init__(self):
                self.i = 0

            def next(self):
                if self.i >= nb:
                    raise StopIteration
                items = [ds[j] for j in order[self.i * bs:(self.i + 1) * bs]]
                self.i += 1
                out = [torch.stack([it[0] for it in items]), torch.stack([it[1] for it in items])]
                if ds.return_paths:
                    out += [[it[2] for it in items], [it[3] for it in items]]
                return tuple(out)

            __next__ = next

            def __iter__(self):
                return self
        return _It()


class EpisodicData:
    """dataset.py:180-327 with the transforms on the device.  ``__getitem__`` returns the
    reference's 7-tuple: (qry_img [3,S,S], target [S,S], spprt_imgs [shot,3,S,S],
    spprt_labels [shot,S,S], subcls_list, [support paths, support labels], [image_path, label]),
    the tensors on ``device``."""

    SUPPORTED_AUG = ("hor_flip", "vert_flip", "resize")

    def __init__(self, mode_train: bool, class_list: List[int], args, read_image: Callable = read_npy,
                 read_label: Callable = read_npy, device=None):
        self.shot = int(_g(args, "shot", 1))
        self.random_shot = bool(_g(args, "random_shot", False))
        self.S = int(_g(args, "image_size", 473))
        self.mean, self.std = list(_g(args, "mean")), list(_g(args, "std"))
        self.padding = [v * 255 for v in self.mean] if _g(args, "padding") == "avg" else None
        if int(_g(args, "meta_aug", 0) or 0) > 1:
            raise NotImplementedError("meta_aug support augmentation is not on the CWT path")
        augs = list(_g(args, "augmentations", ["resize"])) if mode_train else ["resize"]
        bad = [a for a in augs if a not in self.SUPPORTED_AUG]
        if bad or "resize" not in augs:
            raise NotImplementedError(f"augmentations {bad or augs}: the CWT configs use hor_flip, vert_flip, resize")
        self.flips = [a for a in augs if a != "resize"]      # in Compose order, before the resize
        self.class_list = class_list
        self.read_image, self.read_label = read_image, read_label
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        lst = _g(args, "train_list") if mode_train else _g(args, "val_list")
        self.data_list, self.sub_class_file_list = make_dataset(_g(args, "data_root"), lst, class_list, read_label)

    def __len__(self):
        return len(self.data_list)

    def _transform(self, image: np.ndarray, label: np.ndarray):
        fl = {"hor_flip": False, "vert_flip": False}
        for a in self.flips:                              # transform.py:407-422: one draw per flip
            fl[a] = random.random() < 0.5
        img = torch.from_numpy(np.ascontiguousarray(image)).to(self.device)
        lab = torch.from_numpy(np.ascontiguousarray(label.astype(np.uint8))).to(self.device)
        t = preprocess_image(img, self.S, self.mean, self.std, self.padding, fl["hor_flip"], fl["vert_flip"])
        lt = preprocess_label(lab, self.S, -1, fl["hor_flip"], fl["vert_flip"])
        return t, lt

    def __getitem__(self, index: int):
        image_path, label_path = self.data_list[index]
        image = self.read_image(image_path)
        label = self.read_label(label_path)
        if image.shape[0] != label.shape[0] or image.shape[1] != label.shape[1]:
            raise RuntimeError("Query Image & label shape mismatch: " + image_path + " " + label_path + "\n")
        label_class = np.unique(label).tolist()
        if 0 in label_class:
            label_class.remove(0)
        if 255 in label_class:
            label_class.remove(255)
        label_class = [c for c in label_class if c in self.class_list]
        assert len(label_class) > 0
        class_chosen = np.random.choice(label_class)               # dataset.py:220
        new_label = np.zeros_like(label)
        new_label[label == 255] = 255
        new_label[label == class_chosen] = 1
        label = new_label
        file_class_chosen = self.sub_class_file_list[class_chosen]
        num_file = len(file_class_chosen)
        shot = random.randint(1, self.shot) if self.random_shot else self.shot
        s_img_paths, s_lbl_paths, s_idx = [], [], []
        for _ in range(shot):                                      # dataset.py:245-256
            support_idx = random.randint(1, num_file) - 1
            sip, slp = image_path, label_path
            while (sip == image_path and slp == label_path) or support_idx in s_idx:
                support_idx = random.randint(1, num_file) - 1
                sip, slp = file_class_chosen[support_idx]
            s_idx.append(support_idx)
            s_img_paths.append(sip)
            s_lbl_paths.append(slp)
        s_imgs, s_lbls = [], []
        for k in range(shot):
            si = self.read_image(s_img_paths[k])
            raw = self.read_label(s_lbl_paths[k])
            sl = np.zeros_like(raw)
            sl[raw == class_chosen] = 1
            sl[raw == 255] = 255
            if si.shape[0] != sl.shape[0] or si.shape[1] != sl.shape[1]:
                raise RuntimeError("Support Image & label shape mismatch: " + s_img_paths[k] + " " + s_lbl_paths[k])
            s_imgs.append(si)
            s_lbls.append(sl)
        subcls_list = [self.class_list.index(class_chosen) + 1]
        support_labels_orig = [x.copy() for x in s_lbls]
        qry_img, target = self._transform(image, label)
        st = [self._transform(s_imgs[k], s_lbls[k]) for k in range(shot)]
        spprt_imgs = torch.stack([t for t, _ in st])
        spprt_labels = torch.stack([l for _, l in st])
        return qry_img, target, spprt_imgs, spprt_labels, subcls_list, [s_img_paths, support_labels_orig], \
            [image_path, label]


class EpisodeSampler:
    """``torch.utils.data.DistributedSampler(train_data)`` (dataset.py:57-59): rank ``rank`` of
    ``world`` gets every ``world``-th position of one permutation seeded ``seed + epoch`` (the
    same on every rank), padded by wrapping, so ranks train on disjoint episodes.  Call
    ``set_epoch`` before each epoch as with the torch sampler."""

    def __init__(self, n: int, rank: int, world: int, shuffle: bool = True, seed: int = 0):
        from .dist import shard_indices
        self._shard = shard_indices
        self.n, self.rank, self.world, self.shuffle, self.seed, self.epoch = n, rank, world, shuffle, seed, 0

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def __iter__(self):
        return iter(self._shard(self.n, self.rank, self.world, self.shuffle, self.seed, self.epoch))

    def __len__(self):
        return -(-self.n // self.world) if self.n else 0


class EpisodeLoader:
    """``torch.utils.data.DataLoader(dataset, batch_size=1, shuffle=..., sampler=...)`` over
    :class:`EpisodicData` in the calling process (dataset.py:51-63, 95-101): the batch
    dimension is added and ``subcls_list`` collated to ``[tensor([c])]``.  Without a sampler the
    order comes from torch's RNG as RandomSampler draws it (one int64 seed, then randperm); with
    one (multi-rank training) it is the sampler's shard.  The reference's worker processes
    (``workers: 2``) reseed their own RNGs, which is not reproduced."""

    def __init__(self, dataset: EpisodicData, shuffle: bool, sampler: EpisodeSampler | None = None):
        self.dataset, self.shuffle, self.sampler = dataset, shuffle and sampler is None, sampler

    def __len__(self):
        return len(self.sampler) if self.sampler is not None else len(self.dataset)

    def __iter__(self):
        n = len(self.dataset)
        _draw_base_seed()
        if self.sampler is not None:
            order = list(self.sampler)
        elif self.shuffle:
            seed = int(torch.empty((), dtype=torch.int64).random_().item())
            order = torch.randperm(n, generator=torch.Generator().manual_seed(seed)).tolist()
        else:
            order = list(range(n))
        ds = self.dataset

        class _It:
            def __init__(self):
                self.i = 0

            def next(self):
                if self.i >= len(order):
                    raise StopIteration
                q, t, si, sl, sub, sp, qp = ds[order[self.i]]
                self.i += 1
                return q[None], t[None], si[None], sl[None], [torch.tensor([c]) for c in sub], sp, qp

            __next__ = next

            def __iter__(self):
                return self
        return _It()


def get_train_loader(args, read_image: Callable = read_npy, read_label: Callable = read_npy, device=None,
                     episodic: bool = True, return_path: bool = False):
    """dataset.py:17-63: (loader, sampler).  ``episodic=False`` (pretrain.py:83): StandardData over
    ``args.train_list`` with ``args.augmentations``, batches of ``batch_size`` (per rank
    ``batch_size / world`` when distributed, as dataset.py:59), shuffled, drop_last.  Episodic:
    distributed when ``args.distributed`` is
    set or torch.distributed runs more than one rank: the loader iterates this rank's
    :class:`EpisodeSampler` shard (``DistributedSampler`` in the reference) and the sampler is
    returned for ``set_epoch``; otherwise (loader, None).  Each rank runs ONE episode per
    iteration: the reference's per-rank ``int(batch_size / world_size)`` (dataset.py:59) would be
    0 for the scripts' ``batch_size 1``, so the global batch is ``world`` episodes, all-reduced
    (DESIGN.md §6)."""
    from .dist import rank_world
    assert _g(args, "train_split") in [0, 1, 2, 3]
    split_classes = get_split_classes(args)
    class_list = split_classes[_g(args, "train_name")][_g(args, "train_split")]["train"]
    rank, world = rank_world()
    distributed = bool(_g(args, "distributed", False)) or world > 1
    if not episodic:
        ds = StandardData(args, _g(args, "train_list"), class_list, return_path, _g(args, "augmentations", ["resize"]),
                          read_image, read_label, device)
        sampler = EpisodeSampler(len(ds), rank, world, shuffle=True) if distributed else None
        bs = int(_g(args, "batch_size", 1)) // (world if distributed else 1)
        return StandardLoader(ds, max(bs, 1), shuffle=sampler is None, drop_last=True, sampler=sampler), sampler
    ds = EpisodicData(True, class_list, args, read_image, read_label, device)
    if _g(args, "distributed", False) or world > 1:
        sampler = EpisodeSampler(len(ds), rank, world, shuffle=True)
        return EpisodeLoader(ds, shuffle=False, sampler=sampler), sampler
    return EpisodeLoader(ds, shuffle=True), None


def get_val_loader(args, read_image: Callable = read_npy, read_label: Callable = read_npy, device=None):
    """dataset.py:66-117 (episodic): (loader, None).  test_name 'default' = the train dataset
    and split."""
    test_name = _g(args, "test_name", "default")
    if test_name == "default":
        test_name, test_split = _g(args, "train_name"), _g(args, "train_split")
    else:
        test_split = _g(args, "test_split")
    class_list = filter_classes(_g(args, "train_name"), _g(args, "train_split"), test_name, test_split,
                                get_split_classes(args))
    ds = EpisodicData(False, class_list, args, read_image, read_label, device)
    return EpisodeLoader(ds, shuffle=False), None
