import os, sys, numpy as np, torch
sys.path.insert(0, os.getcwd())
from few_shot_seg_cwt_amd import synthetic as syn, get_model
from oracle import cwt_oracle as O
g = dict(np.load("tests/golden/bn_train_small.npz"))
def rel(a, b):
    a = a.detach().double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    return float(np.max(np.abs(a - b)) / np.max(np.abs(b)))
dev = torch.device("cuda", 0)
ep = syn.make_episode(2021, 7, 33, 2)
for layers in (50,):
    m = get_model(syn.cfg_defaults(layers=layers, dropout=0.0)); m.load_state_dict(syn.make_pspnet_state(layers, 2021))
    fe0, _ = m.extract_features(torch.from_numpy(ep["spprt_imgs"][0]).to(dev))
    sd = O.to_torch_state(syn.make_pspnet_state(layers, 2021))
    ref0 = O.extract_features(torch.from_numpy(ep["spprt_imgs"][0]), sd, layers)
    print(os.environ.get("CWT_CONV"), "eval rel", rel(fe0, ref0.numpy()))
    m.train()
    f, _ = m.extract_features(torch.from_numpy(ep["spprt_imgs"][0]).to(dev))
    print(" train rel", rel(f, g[f"feat_train_r{layers}"]))
    st = m.state_dict()
    for k in ["layer0.1", "layer1.0.downsample.1", "layer4.2.bn3", "ppm.features.0.2", "ppm.features.3.2", "bottleneck.1"]:
        print("  ", k, "rm", rel(st[k + ".running_mean"], g[f"r{layers}_rm_{k}"]), "rv", rel(st[k + ".running_var"], g[f"r{layers}_rv_{k}"]))
for layers in (101,):
    m = get_model(syn.cfg_defaults(layers=layers, dropout=0.0)); m.load_state_dict(syn.make_pspnet_state(layers, 2021))
    m.train()
    f, _ = m.extract_features(torch.from_numpy(ep["spprt_imgs"][0]).to(dev))
    print("R101 train rel", rel(f, g[f"feat_train_r{layers}"]))
