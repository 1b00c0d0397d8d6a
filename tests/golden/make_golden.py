"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself.

Runs only in the survey container (needs /root/reference, read-only).  The reference's
own modules and drivers are imported with the shims of SURVEY.md §8(c) — stub modules for
cv2/torchvision (imported only by data code), ``.cuda()`` patched to identity, the two
missing config keys (``cls_type``, ``distributed``) set by attribute — and fed the
deterministic synthetic weights/episodes of few_shot_seg_cwt_amd/synthetic.py.  Only
inputs' seeds and outputs are committed (small .npz/.json); no reference source travels.

    python tests/golden/make_golden.py            # everything (≈2-3 min on 8 cores)

Captured:
  keys_r{50,101}.json          reference PSPNet state_dict keys + shapes
  modules_small.npz            PSPNet.extract_features at S=33 (R50, R101), MultiHeadAttentionOne
                               (H=1,4), the validate_transformer inner loop at small size,
                               intersectionAndUnionGPU
  episode_*.npz                validate_transformer (test.py:103) full-size episodes
  train_pascal_r50_1shot.npz   do_epoch (train.py:166) training episodes, dropout off, BN eval
  train_pascal_r50_1shot_bnq.npz  the same with the reference's first-episode train-mode BN
                               (model.train() at train.py:184), Dropout2d p = 0
  bn_train_small.npz           PSPNet.extract_features in train mode at S=33 (batch statistics,
                               running-statistic update, Dropout2d p = 0), then eval on the query
  variants_small.npz           CosCls (every cls_type flag, n = 2 / 16: output, parameter gradients,
                               parameters after the forward) and get_corr (small + 60x60 samples)
  episode_coco_r101_5shot.npz  validate_transformer 5-shot R101@641 (BASELINE config #5's shapes)
  train_coco_r101_1shot.npz    do_epoch COCO R101@641 (BASELINE config #4), dropout off, BN eval
"""
from __future__ import annotations

import json
import os
import sys
import types

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402

SEED = 2021


def import_reference():
    for name in ["cv2", "torchvision", "torchvision.transforms", "torchvision.transforms.functional",
                 "torchvision.models", "torchvision.ops"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    tv = sys.modules["torchvision"]
    tv.transforms = sys.modules["torchvision.transforms"]
    tv.models = sys.modules["torchvision.models"]
    sys.modules["torchvision.transforms"].functional = sys.modules["torchvision.transforms.functional"]
    torch.nn.Module.cuda = lambda self, *a, **k: self
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.path.insert(0, REF)
    import src.test as rtest
    import src.train as rtrain
    import src.util as rutil
    import src.model.pspnet as rpsp
    import src.model.transformer as rtr
    return rtest, rtrain, rutil, rpsp, rtr


def ref_args(rutil, yaml_name: str, overrides: list):
    cfg = rutil.load_cfg_from_cfg_file(os.path.join(REF, "config_files", yaml_name))
    cfg = rutil.merge_cfg_from_list(cfg, overrides)
    cfg.cls_type = "oooo"        # missing from the yaml, read at pspnet.py:133
    cfg.distributed = False      # missing, read at dataset.py:57
    return cfg


def build_model(rpsp, args, layers):
    model = rpsp.get_model(args)
    sd = syn.make_pspnet_state(layers, SEED)
    ref_sd = model.state_dict()
    assert list(ref_sd.keys()) == list(sd.keys()), "synthetic key order differs from reference"
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}, strict=True)
    model.eval()
    return model


def build_transformer(rtr, heads):
    t = rtr.MultiHeadAttentionOne(heads, 512, 512, 512, dropout=0.5)
    tsd = syn.make_transformer_state(heads, 512, SEED)
    assert list(t.state_dict().keys()) == list(tsd.keys())
    t.load_state_dict({k: torch.from_numpy(v) for k, v in tsd.items()}, strict=True)
    return t


class Loader:
    """Iterable whose iterator has .next() (test.py:150,153; train.py:188)."""

    def __init__(self, S, shot, n, classes=None, start=0):
        self.S, self.shot, self.n, self.classes, self.start = S, shot, n, classes, start

    def __iter__(self):
        return _It(self)

    def __len__(self):
        return self.n


class _It:
    def __init__(self, ld):
        self.ld, self.i = ld, 0

    def next(self):
        ep = syn.make_episode(SEED, self.ld.start + self.i % self.ld.n, self.ld.S, self.ld.shot, self.ld.classes)
        self.i += 1
        t = torch.from_numpy
        return (t(ep["qry_img"]), t(ep["q_label"]), t(ep["spprt_imgs"]), t(ep["s_label"]),
                [torch.tensor([c]) for c in ep["subcls"]], "", "")

    __next__ = next


class Capture:
    """Wraps reference call sites in place to record per-episode tensors."""

    def __init__(self, model, transformer):
        self.rec = []
        self.cur = None
        orig_ef = model.extract_features

        def ef(x):
            out = orig_ef(x)
            self.cur.setdefault("feats", []).append(out[0].detach().clone())
            return out
        model.extract_features = ef
        orig_tf = transformer.forward

        def tf(q, k, v, *a, **kw):
            out = orig_tf(q, k, v, *a, **kw)
            self.cur["W"] = q.detach().clone()
            self.cur["W2"] = out.detach().clone()
            return out
        transformer.forward = tf
        self.orig_conv_fwd = torch.nn.Conv2d.forward
        cap = self

        def conv_fwd(mod, x):
            y = cap.orig_conv_fwd(mod, x)
            if mod.weight.shape[:2] == (2, 512) and not torch.is_grad_enabled():
                cap.cur.setdefault("cls_out", []).append(y.detach().clone())
            return y
        torch.nn.Conv2d.forward = conv_fwd
        self.orig_sgd = torch.optim.SGD.__init__

        def sgd_init(opt, params, *a, **kw):
            params = list(params)
            if len(params) == 1 and isinstance(params[0], torch.Tensor) and params[0].shape == (2, 512, 1, 1):
                cap.cur = {"W0": params[0].detach().clone()}
                cap.rec.append(cap.cur)
            return cap.orig_sgd(opt, params, *a, **kw)
        torch.optim.SGD.__init__ = sgd_init

    def restore(self):
        torch.nn.Conv2d.forward = self.orig_conv_fwd
        torch.optim.SGD.__init__ = self.orig_sgd


def stat(x: torch.Tensor) -> np.ndarray:
    x = x.double()
    return np.array([x.sum().item(), x.abs().sum().item(), (x * x).sum().item()])


def run_validate(rtest, rutil, rpsp, rtr, name, yaml_name, layers, S, shot, n_episodes, classes=None):
    over = ["batch_size_val", "1", "shot", str(shot), "layers", str(layers), "cls_lr", "0.1", "heads", "4",
            "test_num", str(n_episodes), "n_runs", "1", "image_size", str(S)]
    args = ref_args(rutil, yaml_name, over)
    torch.manual_seed(SEED)
    model = build_model(rpsp, args, layers)
    if S != 473:
        model.feature_res = (syn.feature_side(S),) * 2     # test.py:116-119 reads it
    transformer = build_transformer(rtr, 4)
    cap = Capture(model, transformer)
    iu = []
    orig_biu = rtest.batch_intersectionAndUnionGPU

    def biu(logits, target, nc, *a, **k):
        r = orig_biu(logits, target, nc, *a, **k)
        iu.append(np.stack([r[0].numpy().reshape(-1), r[1].numpy().reshape(-1), r[2].numpy().reshape(-1)]))
        return r
    rtest.batch_intersectionAndUnionGPU = biu
    torch.manual_seed(SEED)
    miou, loss = rtest.validate_transformer(args=args, val_loader=Loader(S, shot, n_episodes, classes),
                                            model=model, transformer=transformer)
    rtest.batch_intersectionAndUnionGPU = orig_biu
    cap.restore()
    out = {"mIoU": np.float64(miou), "loss": np.float64(loss), "S": S, "shot": shot, "layers": layers,
           "n_episodes": n_episodes, "seed": SEED}
    for e, r in enumerate(cap.rec):
        f_s, f_q = r["feats"]
        pred_q0, pred_q = r["cls_out"]
        out[f"e{e}_W0"] = r["W0"].numpy().reshape(2, 512)
        out[f"e{e}_W"] = r["W"].numpy().reshape(2, 512)
        out[f"e{e}_W2"] = r["W2"].numpy().reshape(2, 512)
        out[f"e{e}_pred_q"] = pred_q.numpy()[0]
        out[f"e{e}_pred_q0"] = pred_q0.numpy()[0]
        out[f"e{e}_fs_stat"] = stat(f_s)
        out[f"e{e}_fq_stat"] = stat(f_q)
        out[f"e{e}_fq_sample"] = f_q.numpy().reshape(-1)[::997].copy()
        out[f"e{e}_iu"] = iu[2 * e]        # logits (CWT)
        out[f"e{e}_iu0"] = iu[2 * e + 1]   # logits0 (support classifier only)
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(name, "mIoU", miou, "loss", loss)


BN_PROBES = ["layer0.1", "layer1.0.downsample.1", "layer4.2.bn3", "ppm.features.0.2", "ppm.features.3.2",
             "bottleneck.1"]


def run_train(rtrain, rutil, rpsp, rtr, name, n_iter, bn_quirk=False, yaml_name="pascal.yaml", layers=50, S=473,
              classes=None):
    from src.optimizer import get_optimizer
    over = ["shot", "1", "layers", str(layers), "trans_lr", "0.001", "heads", "4", "cls_lr", "0.1", "batch_size", "1",
            "batch_size_val", "1", "image_size", str(S)]
    if bn_quirk:
        over += ["dropout", "0.0"]                   # Dropout2d identity (its RNG is torch's)
    args = ref_args(rutil, yaml_name, over)
    torch.manual_seed(SEED)
    model = build_model(rpsp, args, layers)
    if not bn_quirk:
        model.train = lambda mode=True: model        # exclude the first-episode BN quirk
    transformer = build_transformer(rtr, 4)
    transformer.attention.dropout.p = 0.0            # dropout off for parity (SURVEY §7 hard part 3)
    transformer.dropout.p = 0.0
    opt = get_optimizer(args, [dict(params=transformer.parameters(), lr=args.trans_lr * args.scale_lr)])
    cap = Capture(model, transformer)
    losses, grads = [], []
    orig_step = opt.step

    def step(*a, **k):
        grads.append({n: p.grad.detach().clone() for n, p in transformer.named_parameters()})
        return orig_step(*a, **k)
    opt.step = step
    orig_backward = torch.Tensor.backward

    def backward(t, *a, **k):
        if t.dim() == 0 and t.requires_grad and cap.cur is not None and "W2" in cap.cur and "loss_q" not in cap.cur:
            cap.cur["loss_q"] = t.detach().clone()
        return orig_backward(t, *a, **k)
    torch.Tensor.backward = backward
    torch.manual_seed(SEED)
    ious, tl = rtrain.do_epoch(args=args, train_loader=Loader(S, 1, n_iter, classes, start=1000), model=model,
                               transformer=transformer, optimizer_trans=opt, epoch=1, iter_per_epoch=n_iter,
                               log_iter=n_iter)
    torch.Tensor.backward = orig_backward
    cap.restore()
    out = {"n_iter": n_iter, "train_ious": ious.numpy(), "train_losses": tl.numpy(), "seed": SEED, "start": 1000,
           "S": S, "layers": layers}
    for e, r in enumerate(cap.rec):
        out[f"e{e}_W0"] = r["W0"].numpy().reshape(2, 512)
        out[f"e{e}_W"] = r["W"].numpy().reshape(2, 512)
        out[f"e{e}_W2"] = r["W2"].numpy().reshape(2, 512)
        out[f"e{e}_loss_q"] = r["loss_q"].numpy()
        out[f"e{e}_fs_stat"] = stat(r["feats"][0])
        pred_q0 = r["cls_out"][0]                      # binary_cls(f_q) under no_grad (train.py:249)
        out[f"e{e}_pred_q0"] = pred_q0.numpy()[0]
        if bn_quirk:
            out[f"e{e}_fs_sample"] = r["feats"][0].numpy().reshape(-1)[::997].copy()
            out[f"e{e}_fq_sample"] = r["feats"][1].numpy().reshape(-1)[::997].copy()
        for n, g in grads[e].items():
            out[f"e{e}_grad_{n}_stat"] = stat(g)
            out[f"e{e}_grad_{n}_sample"] = g.numpy().reshape(-1)[::101].copy()
    if bn_quirk:
        sd = model.state_dict()
        for p in BN_PROBES:
            out[f"rm_{p}"] = sd[p + ".running_mean"].numpy().copy()
            out[f"rv_{p}"] = sd[p + ".running_var"].numpy().copy()
    for n, p in transformer.named_parameters():
        out[f"final_{n}_stat"] = stat(p.detach())
        out[f"final_{n}_sample"] = p.detach().numpy().reshape(-1)[::101].copy()
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(name, "losses", tl.numpy())


def run_modules(rutil, rpsp, rtr):
    out = {}
    S = 33
    for layers in (50, 101):
        args = ref_args(rutil, "pascal.yaml", ["layers", str(layers)])
        model = build_model(rpsp, args, layers)
        keys = [(k, list(v.shape)) for k, v in model.state_dict().items()]
        with open(os.path.join(HERE, f"keys_r{layers}.json"), "w") as f:
            json.dump(keys, f)
        ep = syn.make_episode(SEED, 7, S, 2)
        x = torch.from_numpy(ep["spprt_imgs"][0])
        with torch.no_grad():
            fe, lst = model.extract_features(x)
        assert lst == []
        out[f"feat_r{layers}_S{S}"] = fe.numpy()
    # MultiHeadAttentionOne (transformer.py:38-83), eval
    for heads in (1, 4):
        t = build_transformer(rtr, heads).eval()
        q = torch.from_numpy(syn.normal(SEED, f"mq{heads}", (1, 2, 512), 0.05))
        k = torch.from_numpy(out["feat_r50_S33"][:1]).clone()
        k = torch.nn.functional.normalize(k, dim=1)
        with torch.no_grad():
            out[f"mha_h{heads}_out"] = t(q, k, k).numpy()
        out[f"mha_h{heads}_q"] = q.numpy()
    # validate_transformer inner loop (test.py:164-187), at S=33 with the support features above
    f_s = torch.from_numpy(out["feat_r50_S33"])          # 2 shots
    ep = syn.make_episode(SEED, 7, S, 2)
    s_label = torch.from_numpy(ep["s_label"])             # [1,2,S,S]
    torch.manual_seed(SEED)
    clf = torch.nn.Conv2d(512, 2, kernel_size=1, bias=False)
    out["inner_W0"] = clf.weight.detach().numpy().copy()
    opt = torch.optim.SGD(clf.parameters(), lr=0.1)
    arr = s_label.numpy()
    crit = torch.nn.CrossEntropyLoss(weight=torch.tensor([1.0, len(np.where(arr == 0)[0]) / len(np.where(arr == 1)[0])]),
                                     ignore_index=255)
    for _ in range(200):
        o = torch.nn.functional.interpolate(clf(f_s), size=s_label.size()[2:], mode="bilinear", align_corners=True)
        loss = crit(o, s_label.squeeze(0))
        opt.zero_grad()
        loss.backward()
        opt.step()
    out["inner_W200"] = clf.weight.detach().numpy().copy()
    out["inner_loss_last"] = np.float32(loss.item())
    # intersectionAndUnionGPU (util.py:280-308) on random small maps with ignore pixels
    rng = np.random.default_rng(SEED)
    preds = rng.integers(0, 2, (37, 41)).astype(np.int64)
    target = rng.integers(0, 2, (37, 41)).astype(np.int64)
    target[rng.random((37, 41)) < 0.1] = 255
    out["iou_preds"], out["iou_target"] = preds, target
    i, u, tt = rutil.intersectionAndUnionGPU(torch.from_numpy(preds.copy()), torch.from_numpy(target), 2, 255)
    out["iou_out"] = np.stack([i.numpy(), u.numpy(), tt.numpy()])
    np.savez_compressed(os.path.join(HERE, "modules_small.npz"), **out)
    print("modules_small.npz written")


def run_bn_train(rutil, rpsp):
    """PSPNet.extract_features with the module in train mode (every BN on batch statistics,
    running statistics moved by momentum 0.1), then eval mode over the updated statistics."""
    out = {}
    S = 33
    for layers in (50, 101):
        args = ref_args(rutil, "pascal.yaml", ["layers", str(layers), "dropout", "0.0"])
        model = build_model(rpsp, args, layers)
        ep = syn.make_episode(SEED, 7, S, 2)
        model.train()
        with torch.no_grad():
            f_tr, _ = model.extract_features(torch.from_numpy(ep["spprt_imgs"][0]))
        model.eval()
        with torch.no_grad():
            f_ev, _ = model.extract_features(torch.from_numpy(ep["qry_img"]))
        out[f"feat_train_r{layers}"] = f_tr.numpy()
        out[f"feat_eval_after_r{layers}"] = f_ev.numpy()
        sd = model.state_dict()
        for p in BN_PROBES:
            out[f"r{layers}_rm_{p}"] = sd[p + ".running_mean"].numpy().copy()
            out[f"r{layers}_rv_{p}"] = sd[p + ".running_var"].numpy().copy()
    np.savez_compressed(os.path.join(HERE, "bn_train_small.npz"), **out)
    print("bn_train_small.npz written")


COS_TYPES = ["0000", "0n00", "00b0", "000t", "r000", "rnbt", "0nbt", "r0b0"]


def run_variants(rpsp):
    """CosCls (pspnet.py:290-313) for every cls_type flag combination at n = 2 and 16: output,
    the gradients of sum(G * out) w.r.t. its parameters, and the parameters after the forward
    (weight_norm rewrites the stored weight); get_corr (model_util.py:101-109) at a small size
    and at 60 x 60 (samples + checksums)."""
    import src.model.model_util as rmu
    out = {}
    x = torch.from_numpy(syn.normal(SEED, "cosx", (2, 512, 5, 7), 1.0))
    for ct in COS_TYPES:
        for n in (2, 16):
            m = rpsp.CosCls(512, n, ct)
            tag = f"cos_{ct}_{n}"
            with torch.no_grad():
                for name, prm in m.named_parameters():
                    if name == "cls.weight_g":
                        prm.copy_(torch.from_numpy(syn.uniform(SEED, tag + name, tuple(prm.shape), 0.5, 1.5)))
                    elif name == "scale_factor":
                        prm.fill_(1.7)
                    else:
                        prm.copy_(torch.from_numpy(syn.normal(SEED, tag + name, tuple(prm.shape), 0.05)))
            y = m(x)
            G = torch.from_numpy(syn.normal(SEED, tag + "G", tuple(y.shape), 1.0))
            (y * G).sum().backward()
            out[f"{tag}_out"] = y.detach().numpy()
            for name, prm in m.named_parameters():   # inputs are regenerated from the same streams
                out[f"{tag}_grad_{name}"] = prm.grad.detach().numpy().copy()
                if ct[1] == "n" and name == "cls.weight":   # rewritten in place by the forward
                    out[f"{tag}_after_{name}"] = prm.detach().numpy().copy()
    q = torch.from_numpy(syn.normal(SEED, "corrq", (2, 512, 5, 7), 1.0))
    k = torch.from_numpy(syn.normal(SEED, "corrk", (2, 512, 5, 7), 1.0))
    out["corr_small"] = rmu.get_corr(q, k).numpy()
    q = torch.from_numpy(syn.normal(SEED, "corrQ", (1, 512, 60, 60), 1.0)).abs()
    k = torch.from_numpy(syn.normal(SEED, "corrK", (1, 512, 60, 60), 1.0)).abs()
    sim = rmu.get_corr(q, k)
    out["corr60_stat"] = stat(sim)
    out["corr60_sample"] = sim.numpy().reshape(-1)[::9973].copy()
    np.savez_compressed(os.path.join(HERE, "variants_small.npz"), **out)
    print("variants_small.npz written")


def main():
    torch.set_num_threads(8)
    rtest, rtrain, rutil, rpsp, rtr = import_reference()
    which = sys.argv[1:] or ["modules", "pascal1", "pascal5", "coco1", "coco5", "train", "train_coco", "bn_train",
                             "train_bnq", "variants"]
    if "modules" in which:
        run_modules(rutil, rpsp, rtr)
    if "pascal1" in which:
        run_validate(rtest, rutil, rpsp, rtr, "episode_pascal_r50_1shot.npz", "pascal.yaml", 50, 473, 1, 3)
    if "pascal5" in which:
        run_validate(rtest, rutil, rpsp, rtr, "episode_pascal_r50_5shot.npz", "pascal.yaml", 50, 473, 5, 1)
    if "coco1" in which:
        run_validate(rtest, rutil, rpsp, rtr, "episode_coco_r101_1shot.npz", "coco.yaml", 101, 641, 1, 1,
                     classes=syn.coco_val_classes(0))
    if "coco5" in which:       # BASELINE config #5's shapes (fp32 reference; the bf16 stack is scored by mIoU)
        run_validate(rtest, rutil, rpsp, rtr, "episode_coco_r101_5shot.npz", "coco.yaml", 101, 641, 5, 1,
                     classes=syn.coco_val_classes(0))
    if "train" in which:
        run_train(rtrain, rutil, rpsp, rtr, "train_pascal_r50_1shot.npz", 2)
    if "train_coco" in which:  # BASELINE config #4: COCO 1-shot R101 641 training (do_epoch), dropout off, BN eval
        run_train(rtrain, rutil, rpsp, rtr, "train_coco_r101_1shot.npz", 2, yaml_name="coco.yaml", layers=101, S=641,
                  classes=syn.coco_val_classes(0))
    if "bn_train" in which:
        run_bn_train(rutil, rpsp)
    if "train_bnq" in which:
        run_train(rtrain, rutil, rpsp, rtr, "train_pascal_r50_1shot_bnq.npz", 2, bn_quirk=True)
    if "variants" in which:
        run_variants(rpsp)


if __name__ == "__main__":
    main()
