"""Staged GPU diagnostic: run each kernel family once at small size with a device sync and a
timestamp after each, so a hang or fault is localised to one stage."""
import faulthandler
import os
import sys
import time

faulthandler.enable()
faulthandler.dump_traceback_later(int(os.environ.get("DIAG_DUMP_S", "90")), repeat=True)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
T0 = time.time()


def say(*a):
    print(f"[{time.time() - T0:7.2f}s]", *a, flush=True)


import numpy as np  # noqa: E402
import torch  # noqa: E402

say("torch imported", torch.__version__, torch.cuda.is_available())
from few_shot_seg_cwt_amd import MultiHeadAttentionOne, _lib, get_model  # noqa: E402
from few_shot_seg_cwt_amd import synthetic as syn  # noqa: E402
from few_shot_seg_cwt_amd.episode import classify, inner_adapt, normalize  # noqa: E402
from few_shot_seg_cwt_amd.util import seg_metrics  # noqa: E402

dev = torch.device("cuda", 0)
x = torch.zeros(1, device=dev)
torch.cuda.synchronize()
say("torch cuda init ok")
_lib.ctx(0)
say("cwt ctx ok", _lib.lib().cwt_version())
S = int(os.environ.get("DIAG_S", "33"))
cfg = syn.cfg_defaults(image_size=S)
sd = syn.make_pspnet_state(50, 2021)
say("weights generated")
m = get_model(cfg)
m.load_state_dict(sd)
torch.cuda.synchronize()
say("backbone loaded")
ep = syn.make_episode(2021, 0, S, 1)
imgs = torch.from_numpy(np.concatenate([ep["spprt_imgs"][0], ep["qry_img"]])).to(dev)
torch.cuda.synchronize()
say("inputs on device")
_lib.profile_enable(2)
f, _ = m.extract_features(imgs)
say("extract launched")
torch.cuda.synchronize()
say("extract done", tuple(f.shape), float(f.abs().sum()))
for name, fl, by, ms in _lib.profile_records():
    say(f"   {name:60s} {ms:8.3f} ms  {fl / max(ms, 1e-9) / 1e9:8.1f} TFLOP/s")
_lib.profile_enable(0)
W = torch.from_numpy(syn.normal(2021, "w", (2, 512), 0.04)).to(dev)
inner_adapt(f[:1], torch.from_numpy(ep["s_label"][0]).to(dev), W, 0.1, 1)
torch.cuda.synchronize()
say("inner_adapt x1 done", float(W.abs().sum()))
inner_adapt(f[:1], torch.from_numpy(ep["s_label"][0]).to(dev), W, 0.1, 200)
torch.cuda.synchronize()
say("inner_adapt x200 done", float(W.abs().sum()))
fqn, l0 = normalize(f[1:], W.view(1, 2, -1))
torch.cuda.synchronize()
say("normalize done")
t = MultiHeadAttentionOne(4, 512, 512, 512)
t.load_state_dict(syn.make_transformer_state(4, 512, 2021))
with torch.no_grad():
    W2 = t(W.view(1, 2, -1), fqn, fqn)
torch.cuda.synchronize()
say("attention fwd done", float(W2.abs().sum()))
lg = classify(W2, fqn)
torch.cuda.synchronize()
say("classify done")
iut, ce = seg_metrics(lg, torch.from_numpy(ep["q_label"]).to(dev))
torch.cuda.synchronize()
say("metrics done", iut.cpu().numpy().tolist(), ce.cpu().numpy().tolist())
faulthandler.cancel_dump_traceback_later()
say("ALL OK")
