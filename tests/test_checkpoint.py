"""Checkpoint compatibility (few_shot_seg_cwt_amd/checkpoint.py):
CWT checkpoints in the reference's {'epoch','state_dict','optimizer'} layout with
torch.optim.SGD's per-parameter momentum buffers (train.py:147-152; test.py:83-89), and the
two backbone loaders (by name with 'module.', train.py:57-75; by position, test.py:61-81).
CPU only: no kernel runs."""
from collections import OrderedDict

import numpy as np
import pytest
import torch

from few_shot_seg_cwt_amd import checkpoint as ck
from few_shot_seg_cwt_amd import synthetic as syn
from few_shot_seg_cwt_amd.optimizer import HipSGD
from few_shot_seg_cwt_amd.transformer import MultiHeadAttentionOne

REF_PARAMS = [("w_qkvs.weight", (2048, 512)), ("layer_norm.weight", (512,)), ("layer_norm.bias", (512,)),
              ("fc.weight", (512, 2048)), ("fc.bias", (512,))]


def _cwt_cpu():
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5, device=None)
    t.load_state_dict(syn.make_transformer_state(4, 512, 2021))
    return t.cpu() if t.flat.is_cuda else t


def test_model_dirs():
    a = dict(model_dir="model_ckpt", train_name="pascal", train_split=0, shot=1, arch="resnet", layers=50)
    assert ck.get_model_dir_trans(a) == "model_ckpt/pascal/split=0/model/shot_1/transformer_resnet50"
    assert ck.get_model_dir(a) == "model_ckpt/pascal/split=0/model/shot_1/pspnet_resnet50"


def test_optimizer_state_matches_torch_sgd_layout():
    t = _cwt_cpu()
    opt = HipSGD([t.flat], lr=0.001, momentum=0.9, weight_decay=1e-4, nesterov=True)
    opt.bufs = [torch.randn(t.flat.numel())]
    ours = ck.optimizer_state_dict(opt, t)
    params = [torch.nn.Parameter(torch.zeros(s)) for _, s in REF_PARAMS]
    ref = torch.optim.SGD(params, lr=0.001, momentum=0.9, weight_decay=1e-4, nesterov=True)
    for p in params:
        p.grad = torch.ones_like(p)
    ref.step()
    rsd = ref.state_dict()
    assert set(ours["param_groups"][0]) == set(rsd["param_groups"][0])
    assert ours["param_groups"][0]["params"] == rsd["param_groups"][0]["params"]
    assert sorted(ours["state"]) == sorted(rsd["state"])
    for i in rsd["state"]:
        assert ours["state"][i]["momentum_buffer"].shape == rsd["state"][i]["momentum_buffer"].shape
    # concatenation in parameter order is the flat buffer
    cat = torch.cat([ours["state"][i]["momentum_buffer"].reshape(-1) for i in range(5)])
    assert torch.equal(cat, opt.bufs[0])
    # a torch.optim.SGD state loads into HipSGD (per-parameter -> flat)
    opt2 = HipSGD([t.flat], lr=0.5)
    ck.load_optimizer_state_dict(opt2, t, rsd)
    assert opt2.lr == 0.001 and opt2.momentum == 0.9 and opt2.nesterov
    ref_cat = torch.cat([rsd["state"][i]["momentum_buffer"].reshape(-1) for i in range(5)])
    assert torch.equal(opt2.bufs[0].cpu(), ref_cat)


def test_transformer_checkpoint_roundtrip(tmp_path):
    t = _cwt_cpu()
    opt = HipSGD([t.flat], lr=0.001, momentum=0.9)
    opt.bufs = [torch.randn(t.flat.numel())]
    path = str(tmp_path / "split=0" / "best.pth")
    ck.save_transformer_checkpoint(path, 7, t, opt)
    raw = torch.load(path, weights_only=True)
    assert set(raw) == {"epoch", "state_dict", "optimizer"} and raw["epoch"] == 7
    assert list(raw["state_dict"]) == [n for n, _ in REF_PARAMS]
    t2 = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.5)
    opt2 = HipSGD([t2.flat], lr=0.1)
    ck.load_transformer_checkpoint(path, t2, opt2)
    assert torch.equal(t2.flat.detach().cpu(), t.flat.detach().cpu())
    assert torch.equal(opt2.bufs[0].cpu(), opt.bufs[0])


def _sd(layers=50):
    return OrderedDict((k, torch.as_tensor(np.asarray(v))) for k, v in syn.make_pspnet_state(layers, 2021).items())


def test_backbone_by_name_module_prefix():
    sd = _sd()
    base = OrderedDict((k, torch.zeros_like(v)) for k, v in sd.items())
    pre = OrderedDict(("module." + k, v) for k, v in sd.items())
    bad = "layer1.0.conv1.weight"
    pre["module." + bad] = torch.zeros(3)
    msgs = []
    out = ck.map_backbone_by_name(base, pre, log=msgs.append)
    assert len(msgs) == 1 and bad in msgs[0]
    for k in sd:
        if "classifier" in k or "gamma" in k or k == bad:
            assert torch.equal(out[k], base[k]), k
        else:
            assert torch.equal(out[k], sd[k]), k


def test_backbone_by_position():
    sd = _sd()
    base = OrderedDict((k, torch.zeros_like(v)) for k, v in sd.items())
    pre = OrderedDict((f"anything.{i}", v) for i, v in enumerate(sd.values()))   # names ignored, order used
    out = ck.map_backbone_by_position(base, pre, log=lambda m: None)
    for k in sd:
        assert torch.equal(out[k], base[k] if "classifier" in k else sd[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("by", ["name", "position"])
def test_load_backbone_checkpoint_gpu(tmp_path, by):
    """A reference-style backbone checkpoint ({'state_dict': ...}, 'module.' keys for the
    by-name loader) loads through checkpoint.load_backbone and extracts the same features."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from few_shot_seg_cwt_amd import get_model
    sd = _sd()
    keys = ("module." + k for k in sd) if by == "name" else (f"p{i}" for i in range(len(sd)))
    path = str(tmp_path / "best.pth")
    torch.save({"state_dict": OrderedDict(zip(keys, sd.values()))}, path)
    m1 = ck.load_backbone(get_model(syn.cfg_defaults()), path, by=by, log=lambda m: None)
    m2 = get_model(syn.cfg_defaults()).load_state_dict(syn.make_pspnet_state(50, 2021))
    x = torch.from_numpy(syn.make_episode(2021, 3, 33, 1)["qry_img"]).cuda()
    f1, _ = m1.extract_features(x)
    f2, _ = m2.extract_features(x)
    torch.cuda.synchronize()
    assert torch.equal(f1, f2)
