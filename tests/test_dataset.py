"""Episode data path (few_shot_seg_cwt_amd/dataset.py, csrc/preprocess.hip; SURVEY.md §8(f)
rank 1).  CPU: class splits, the list filter, Resize geometry.  GPU: the preprocessing kernels
bit-exact against oracle/data_oracle.py (the restated transform.py / cv2.resize arithmetic --
parity against cv2 itself is unpinned: cv2 is not installed), and EpisodicData end to end on a
small on-disk .npy dataset (sampling invariants of dataset.py:205-266)."""
import os
import random

import numpy as np
import pytest
import torch

from few_shot_seg_cwt_amd import dataset as D
from oracle import data_oracle as DO

MEAN, STD = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]


def test_split_classes():
    sc = D.get_split_classes({"use_split_coco": True})
    assert sc["pascal"][0]["val"] == [1, 2, 3, 4, 5]
    assert sorted(sc["pascal"][0]["train"]) == list(range(6, 21))
    assert sc["coco"][0]["val"] == list(range(1, 78, 4))
    assert len(sc["coco"][2]["train"]) == 60
    assert D.filter_classes("pascal", 0, "pascal", 0, sc) == [1, 2, 3, 4, 5]
    assert D.filter_classes("pascal", 0, "pascal", -1, sc) == [1, 2, 3, 4, 5]   # -1 = all, minus seen
    sc2 = D.get_split_classes({"use_split_coco": False})
    assert sc2["coco"][1]["val"] == list(range(21, 41))


def test_find_new_hw_matches_oracle_and_quirk():
    # 473 -> 472 (the %8 quirk of transform.py:128-135)
    assert DO.find_new_hw(500, 375, 473) == (472, 352)
    assert DO.find_new_hw(375, 500, 473) == (352, 472)
    assert DO.find_new_hw(641, 641, 641) == (640, 640)


def _write_dataset(root, n=8, H=(50, 70), classes=(1, 2, 3), seed=0):
    rng = np.random.default_rng(seed)
    lines = []
    for i in range(n):
        h, w = int(rng.integers(*H)), int(rng.integers(*H))
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        lab = np.zeros((h, w), np.uint8)
        c = classes[i % len(classes)]
        lab[: h // 2 + 20, : w // 2 + 20] = c       # >= 2*32*32 pixels only for the large ones
        lab[-3:, :] = 255
        if i % 2:
            lab[h // 2:, w // 2:] = classes[(i + 1) % len(classes)]
        np.save(os.path.join(root, f"img{i}.npy"), img)
        np.save(os.path.join(root, f"lab{i}.npy"), lab)
        lines.append(f"img{i}.npy lab{i}.npy")
    lst = os.path.join(root, "list.txt")
    open(lst, "w").write("\n".join(lines) + "\n")
    return lst


def test_make_dataset_filter(tmp_path):
    lst = _write_dataset(str(tmp_path), n=6, H=(90, 110))
    items, by_cls = D.make_dataset(str(tmp_path), lst, [1, 2, 3])
    for c, files in by_cls.items():
        for _, lp in files:
            assert int((np.load(lp) == c).sum()) >= 2048
    assert len(items) == len({i for f in by_cls.values() for i in f})


# ------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,S", [(500, 375, 473), (375, 500, 473), (333, 500, 473), (480, 640, 641),
                                   (40, 33, 473), (473, 473, 473), (100, 60, 57)])
@pytest.mark.parametrize("src_f32", [False, True])
def test_preprocess_image_bitexact(dev, H, W, S, src_f32):
    rng = np.random.default_rng(H * 7 + W)
    img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    src = img.astype(np.float32) if src_f32 else img
    for fh, fv, pad in [(False, False, None), (True, False, None), (True, True, [v * 255 for v in MEAN])]:
        out = D.preprocess_image(torch.from_numpy(src).to(dev), S, MEAN, STD, pad, fh, fv)
        ref, _ = DO.val_transform(img, None, S, MEAN, STD, pad, fh, fv)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("H,W,S", [(500, 375, 473), (375, 500, 473), (77, 91, 473), (480, 640, 641)])
def test_preprocess_label_bitexact(dev, H, W, S):
    rng = np.random.default_rng(H + W)
    lab = rng.integers(0, 6, (H, W)).astype(np.uint8)
    lab[rng.random((H, W)) < 0.05] = 255
    for cls, fh, fv in [(3, False, False), (2, True, True), (-1, False, True)]:
        out = D.preprocess_label(torch.from_numpy(lab).to(dev), S, cls, fh, fv)
        rl = DO.remap_label(lab, cls) if cls >= 0 else lab
        _, ref = DO.val_transform(np.zeros((H, W, 3), np.uint8), rl, S, MEAN, STD, None, fh, fv)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize("mode_train", [False, True])
def test_episodic_data_end_to_end(dev, tmp_path, mode_train):
    lst = _write_dataset(str(tmp_path), n=12, H=(90, 130))
    args = dict(shot=2, random_shot=False, image_size=97, mean=MEAN, std=STD, padding=None,
                augmentations=["hor_flip", "vert_flip", "resize"], data_root=str(tmp_path),
                train_list=lst, val_list=lst)
    ds = D.EpisodicData(mode_train, [1, 2, 3], args, device=dev)
    random.seed(5)
    np.random.seed(5)
    for i in range(len(ds)):
        qry, tgt, simgs, slbls, subcls, (s_paths, s_raw), (qpath, qlab) = ds[i]
        assert qry.shape == (3, 97, 97) and tgt.shape == (97, 97) and tgt.dtype == torch.int64
        assert simgs.shape == (2, 3, 97, 97) and slbls.shape == (2, 97, 97)
        assert qpath not in s_paths and len(set(s_paths)) == 2            # distinct supports, never the query
        assert set(np.unique(tgt.cpu().numpy())) <= {0, 1, 255}
        c = [1, 2, 3][subcls[0] - 1]
        for p in s_paths:
            lp = os.path.join(os.path.dirname(p), os.path.basename(p).replace("img", "lab"))
            assert int((np.load(lp) == c).sum()) >= 2048
        if not mode_train:   # no flips: the transform is the oracle's exactly
            ref, reft = DO.val_transform(np.load(qpath), qlab, 97, MEAN, STD)
            np.testing.assert_array_equal(qry.cpu().numpy(), ref)
            np.testing.assert_array_equal(tgt.cpu().numpy(), reft)


@pytest.mark.gpu
def test_validate_transformer_over_episodic_loader(dev, tmp_path):
    """The reference's validation loop fed by the device data path (get_val_loader): it runs
    and its per-episode W matches EpisodeEngine on the same preprocessed tensors."""
    from few_shot_seg_cwt_amd import MultiHeadAttentionOne, get_model
    from few_shot_seg_cwt_amd import synthetic as syn
    from few_shot_seg_cwt_amd.episode import validate_transformer
    lst = _write_dataset(str(tmp_path), n=12, H=(90, 130))
    args = syn.cfg_defaults(image_size=97, test_num=3, n_runs=1, shot=1)
    args.update(mean=MEAN, std=STD, padding=None, augmentations=["hor_flip", "vert_flip", "resize"],
                data_root=str(tmp_path), train_list=lst, val_list=lst, train_name="pascal", train_split=0,
                test_name="default", use_split_coco=False, random_shot=False)
    loader, _ = D.get_val_loader(args, device=dev)
    assert len(loader) > 0
    model = get_model(args).load_state_dict(syn.make_pspnet_state(50, 2021))
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    t.load_state_dict(syn.make_transformer_state(4, 512, 2021))
    random.seed(1)
    np.random.seed(1)
    torch.manual_seed(1)
    eps = []
    miou, loss = validate_transformer(args, loader, model, t, episodes_out=eps)
    assert np.isfinite(miou) and np.isfinite(loss) and len(eps) == 3


def test_standard_label_remap():
    """dataset.py:144-168: classes of class_list -> index + 1, other classes 255, the source's
    own void (255) and background -> 0."""
    lab = np.array([[0, 3, 3, 255], [5, 5, 7, 0]], np.uint8)
    out = D.standard_label(lab, [3, 7, 9])
    np.testing.assert_array_equal(out, np.array([[0, 1, 1, 0], [255, 255, 2, 0]], np.uint8))
    with pytest.raises(AssertionError):
        D.standard_label(np.array([[0, 5]], np.uint8), [3])


def test_standard_data_host_items(tmp_path):
    """StandardData over make_dataset's list (utils.py filter), remapped labels (host part)."""
    lst = _write_dataset(str(tmp_path), n=6, H=(90, 110))
    args = dict(image_size=65, mean=MEAN, std=STD, data_root=str(tmp_path))
    ds = D.StandardData.__new__(D.StandardData)
    ds.class_list, ds.read_image, ds.read_label = [1, 2, 3], D.read_npy, D.read_npy
    ds.data_list, _ = D.make_dataset(args["data_root"], lst, [1, 2, 3])
    for i in range(len(ds.data_list)):
        img, lab, ip, lp = D.StandardData.host_item(ds, i)
        raw = np.load(lp)
        assert img.shape[:2] == lab.shape
        np.testing.assert_array_equal(lab[raw == 255], 0)
        for c in (1, 2, 3):
            np.testing.assert_array_equal(lab[raw == c], c)   # index + 1 with class_list [1, 2, 3]


@pytest.mark.gpu
def test_standard_loader_end_to_end(dev, tmp_path):
    """get_train_loader(args, episodic=False) (pretrain.py:83): batches of batch_size, drop_last,
    every item the oracle's transform of the remapped pair (no flips here: bit-exact)."""
    lst = _write_dataset(str(tmp_path), n=9, H=(90, 130))
    args = dict(image_size=65, mean=MEAN, std=STD, padding=None, augmentations=["resize"], data_root=str(tmp_path),
                train_list=lst, train_name="pascal", train_split=0, batch_size=2, use_split_coco=False)
    # the synthetic classes 1..3 are PASCAL split-0 val classes: a split-1 train list holds them
    args["train_split"] = 1
    loader, sampler = D.get_train_loader(args, device=dev, episodic=False, return_path=True)
    assert sampler is None and len(loader) == len(loader.dataset) // 2
    cl = D.get_split_classes(args)["pascal"][1]["train"]
    n = 0
    for images, gt, ipaths, lpaths in loader:
        assert images.shape == (2, 3, 65, 65) and gt.shape == (2, 65, 65) and gt.dtype == torch.int64
        for k in range(2):
            lab = D.standard_label(np.load(lpaths[k]), cl)
            ref, reft = DO.val_transform(np.load(ipaths[k]), lab, 65, MEAN, STD)
            np.testing.assert_array_equal(images[k].cpu().numpy(), ref)
            np.testing.assert_array_equal(gt[k].cpu().numpy(), reft)
        n += 1
    assert n == len(loader)


class _Items:
    """A stand-in dataset of n (tensor, tensor) items for the loaders' order logic."""
    return_paths = False

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return torch.tensor([float(i)]), torch.tensor([i])


@pytest.mark.parametrize("shuffle", [True, False])
def test_standard_loader_rng_matches_torch_dataloader(shuffle):
    """The loader's batch order and the global torch RNG stream after it equal
    torch.utils.data.DataLoader's (the iterator's base-seed draw, then RandomSampler's seed):
    pretrain.py:105 iterates a DataLoader, so every later draw lines up with the reference's."""
    n, bs = 11, 3
    torch.manual_seed(123)
    ref = [b[1].view(-1).tolist() for b in torch.utils.data.DataLoader(_Items(n), batch_size=bs, shuffle=shuffle,
                                                                       drop_last=True)]
    after_ref = torch.rand(4)
    torch.manual_seed(123)
    got = [b[1].view(-1).tolist() for b in D.StandardLoader(_Items(n), bs, shuffle, drop_last=True)]
    after = torch.rand(4)
    assert got == ref
    assert torch.equal(after, after_ref)


def test_episode_loader_rng_matches_torch_dataloader():
    """The episodic loader (batch 1, shuffled) consumes the global RNG like DataLoader too."""
    n = 7
    torch.manual_seed(5)
    ref = [int(b[1]) for b in torch.utils.data.DataLoader(_Items(n), batch_size=1, shuffle=True)]
    after_ref = torch.rand(3)
    torch.manual_seed(5)

    class _Ep(_Items):
        def __getitem__(self, i):
            t = torch.tensor([i])
            return t, t, t, t, [i], "", ""
    got = [int(b[1]) for b in D.EpisodeLoader(_Ep(n), shuffle=True)]
    after = torch.rand(3)
    assert got == ref
    assert torch.equal(after, after_ref)
