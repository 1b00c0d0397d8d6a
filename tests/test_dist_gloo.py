"""Multi-process (world_size 2, gloo, CPU) tests of the two exchange points of the CWT path
(DESIGN.md §6): the mean all-reduce of the flat CWT gradient bucket before the identical SGD
step, the sum all-reduce of the per-class intersection/union table of sharded inference, and
the once-per-epoch broadcast of rank 0's BN running statistics."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat_grads(seed_ep: int):
    """Oracle CWT gradients of one small training episode, flattened in the layout of
    few_shot_seg_cwt_amd.transformer (w_qkvs, layer_norm.w/b, fc.w/b)."""
    from few_shot_seg_cwt_amd import synthetic as syn
    from few_shot_seg_cwt_amd.transformer import _layout
    from oracle import cwt_oracle as O
    heads = 2
    tsd = O.to_torch_state(syn.make_transformer_state(heads, 512, 2021))
    f_q = torch.from_numpy(syn.normal(seed_ep, "fq", (1, 512, 5, 5), 0.1))
    W = torch.from_numpy(syn.normal(seed_ep, "W", (2, 512), 0.05))
    ep = syn.make_episode(seed_ep, 0, 33, 1)
    _, grads, _ = O.cwt_train_step_grads(W, f_q, torch.from_numpy(ep["q_label"]), tsd, heads)
    lay, total = _layout(heads, 512)
    flat = torch.zeros(total)
    for n, shp, off, k in lay:
        flat[off:off + k] = grads[n].reshape(-1)
    return flat, tsd, lay


def _worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from few_shot_seg_cwt_amd import dist as cdist
    from oracle import cwt_oracle as O
    r, _, w = cdist.init_from_env(backend="gloo")
    assert (r, w) == (rank, WORLD)
    # --- training: rank r runs episode base + r (train_ddp.py:62-66 seeding idiom) ---
    mine, tsd, lay = _flat_grads(100 + rank)
    bucket = mine.clone()
    cdist.all_reduce_mean_(bucket)
    g0, _, _ = _flat_grads(100)
    g1, _, _ = _flat_grads(101)
    expect = (g0 + g1) / 2
    assert torch.allclose(bucket, expect, rtol=1e-6, atol=1e-9)
    # identical SGD step everywhere -> identical parameters on every rank
    params = {n: tsd[n].clone() for n, _, _, _ in lay}
    grads = {n: bucket[off:off + k].view(shp) for n, shp, off, k in lay}
    newp, _ = O.sgd_nesterov(params, grads, {}, lr=1e-3, momentum=0.9, wd=1e-4)
    flatp = torch.cat([newp[n].reshape(-1) for n, _, _, _ in lay])
    allp = [torch.zeros_like(flatp) for _ in range(WORLD)]
    torch.distributed.all_gather(allp, flatp)
    assert torch.equal(allp[0], allp[1])
    # --- inference: episodes sharded round-robin, per-class table summed once ---
    n_ep, classes = 10, [1, 2, 3, 4, 5]
    mine_eps = [e for e in range(n_ep) if e % WORLD == rank]
    table = {}
    for e in mine_eps:
        c = classes[e % len(classes)]
        t = table.setdefault(c, np.zeros(2))
        t += (e + 1, 2 * e + 3)      # stand-in (intersection, union) per episode
    keys = cdist.union_keys(sorted(table))
    assert keys == classes
    tab = np.array([table.get(c, np.zeros(2)) for c in keys])
    tab = cdist.all_reduce_sum_np(tab)
    ref = {c: np.zeros(2) for c in classes}
    for e in range(n_ep):
        ref[classes[e % len(classes)]] += (e + 1, 2 * e + 3)
    np.testing.assert_array_equal(tab, np.array([ref[c] for c in classes]))
    assert cdist.all_reduce_max_scalar(float(rank)) == WORLD - 1
    torch.distributed.destroy_process_group()
    open(os.path.join(out_dir, f"ok{rank}"), "w").write("ok")


def test_gloo_world2_exchange_points(tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    assert all((tmp_path / f"ok{r}").exists() for r in range(WORLD))


class _FakeExtractor:
    """state_dict / load_state_dict surface of PSPNet (pspnet.py) without the GPU library."""

    def __init__(self, rank):
        g = np.random.default_rng(rank)
        self.sd = {"layer0.1.weight": np.full(4, float(rank), np.float32),
                   "layer0.1.running_mean": g.standard_normal(4).astype(np.float32),
                   "layer0.1.running_var": g.random(4).astype(np.float32) + 0.5,
                   "layer0.1.num_batches_tracked": np.array(rank + 1),
                   "ppm.features.0.2.running_mean": g.standard_normal(512).astype(np.float32),
                   "ppm.features.0.2.running_var": g.random(512).astype(np.float32) + 0.5}
        self.loads = 0

    def state_dict(self):
        return {k: torch.from_numpy(np.array(v)) for k, v in self.sd.items()}

    def load_state_dict(self, sd):
        self.sd = {k: np.asarray(v) for k, v in sd.items()}
        self.loads += 1


def _bn_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from few_shot_seg_cwt_amd import dist as cdist
    cdist.init_from_env(backend="gloo")
    m = _FakeExtractor(rank)
    cdist.broadcast_backbone_bn_(m)
    ref = _FakeExtractor(0).sd
    for k, v in m.sd.items():
        if k.endswith((".running_mean", ".running_var")):
            np.testing.assert_array_equal(v, ref[k])        # rank 0's statistics, bit for bit
        else:
            np.testing.assert_array_equal(v, _FakeExtractor(rank).sd[k])   # weights untouched
    assert m.loads == (0 if rank == 0 else 1)
    torch.distributed.destroy_process_group()
    open(os.path.join(out_dir, f"bn{rank}"), "w").write("ok")


def test_gloo_world2_bn_broadcast(tmp_path):
    port = _free_port()
    mp.spawn(_bn_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    assert all((tmp_path / f"bn{r}").exists() for r in range(WORLD))


# ------------------------------------------------------------------ multi-rank do_epoch
def _stand_in_train_episode(model, transformer, args, batch, W0, dev):
    """CPU stand-in for episode.train_episode (whose kernels need the GPU): the oracle's CWT
    gradients of a tiny episode derived from the batch's query image and this rank's W0,
    ACCUMULATED into transformer.flat.grad like the HIP path does."""
    from few_shot_seg_cwt_amd.transformer import _layout
    from oracle import cwt_oracle as O
    qry_img, q_label = batch[0], batch[1]
    heads = transformer.n_head
    tsd = {n: transformer.view(n).detach().clone() for n, _, _, _ in _layout(heads, 512)[0]}
    f_q = torch.nn.functional.adaptive_avg_pool2d(qry_img.float(), 5).repeat(1, 171, 1, 1)[:, :512]
    W = W0.reshape(2, 512).float()
    loss, grads, _ = O.cwt_train_step_grads(W, f_q, q_label, tsd, heads)
    lay, _ = _layout(heads, 512)
    for n, shp, off, k in lay:
        transformer.flat.grad[off:off + k] += grads[n].reshape(-1)
    z = torch.zeros(1, 3, 2)
    _stand_in_train_episode.seen.append((float(qry_img.double().sum()), W0.clone(),
                                         transformer.flat.grad.clone()))
    return dict(loss=torch.tensor([float(loss)]), W=W, W2=W.view(1, 2, 512), pred_q=None, pred_q0=None,
                iut=z + 1, iut0=z + 1)


class _StubExtractor:
    training = False

    def train(self, mode=True):
        self.training = mode
        return self

    def eval(self):
        return self.train(False)


def _train_worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from few_shot_seg_cwt_amd import dist as cdist
    from few_shot_seg_cwt_amd import episode
    from few_shot_seg_cwt_amd import synthetic as syn
    from few_shot_seg_cwt_amd.transformer import MultiHeadAttentionOne
    cdist.init_from_env(backend="gloo")
    assert cdist.seed_everything(2021) == 2021 + rank          # train_ddp.py:62-66
    t = MultiHeadAttentionOne(2, 512, 512, 512, dropout=0.0)    # per-rank init: differs before the broadcast
    p0 = [torch.zeros_like(t.flat.data) for _ in range(WORLD)]
    torch.distributed.all_gather(p0, t.flat.data.clone())
    assert not torch.equal(p0[0], p0[1])
    opt = torch.optim.SGD([t.flat], lr=1e-3, momentum=0.9, weight_decay=1e-4, nesterov=True)
    n_iter = 3
    loader = episode.SyntheticEpisodes(n_iter * WORLD, S=33, seed=2021).shard(rank, WORLD)
    _stand_in_train_episode.seen = []
    episode.train_episode = _stand_in_train_episode
    cfg = syn.cfg_defaults(image_size=33)
    episode.do_epoch(cfg, loader, _StubExtractor(), t, opt, epoch=0, iter_per_epoch=n_iter, log_iter=n_iter)
    seen = _stand_in_train_episode.seen
    assert len(seen) == n_iter
    # every rank started from rank 0's parameters, ran its own episodes with its own W0, and the
    # identical SGD steps on the mean gradient kept the replicas bit-identical
    pf = [torch.zeros_like(t.flat.data) for _ in range(WORLD)]
    torch.distributed.all_gather(pf, t.flat.data.clone())
    assert torch.equal(pf[0], pf[1])
    ids = torch.tensor([s[0] for s in seen], dtype=torch.float64)
    w0 = torch.stack([s[1] for s in seen])
    all_ids = [torch.zeros_like(ids) for _ in range(WORLD)]
    all_w0 = [torch.zeros_like(w0) for _ in range(WORLD)]
    torch.distributed.all_gather(all_ids, ids)
    torch.distributed.all_gather(all_w0, w0)
    assert not set(all_ids[0].tolist()) & set(all_ids[1].tolist()), "ranks trained on the same episode"
    assert not torch.equal(all_w0[0], all_w0[1]), "ranks drew the same classifier init"
    # replay: rank 0's initial parameters, then per step the SGD update on the mean of the two
    # ranks' local gradients (recorded inside train_episode, before the all-reduce)
    local = torch.stack([s[2] for s in seen])
    all_local = [torch.zeros_like(local) for _ in range(WORLD)]
    torch.distributed.all_gather(all_local, local)
    ref = torch.nn.Parameter(p0[0].clone())
    ref_opt = torch.optim.SGD([ref], lr=1e-3, momentum=0.9, weight_decay=1e-4, nesterov=True)
    for k in range(n_iter):
        ref.grad = (all_local[0][k] + all_local[1][k]) / 2
        ref_opt.step()
    assert torch.allclose(ref.data, t.flat.data, rtol=0, atol=1e-7)
    torch.distributed.destroy_process_group()
    open(os.path.join(out_dir, f"tr{rank}"), "w").write("ok")


def test_gloo_world2_do_epoch_shards_episodes_and_seeds(tmp_path):
    """do_epoch over 2 ranks: disjoint episodes (SyntheticEpisodes.shard), per-rank W0
    (seed_everything), rank 0's starting parameters on both ranks (broadcast_params_), mean
    gradient all-reduce, identical parameters after every step."""
    port = _free_port()
    mp.spawn(_train_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    assert all((tmp_path / f"tr{r}").exists() for r in range(WORLD))


def test_episode_sampler_matches_distributed_sampler():
    """EpisodeSampler (get_train_loader's shard) hands out exactly DistributedSampler's indices
    (dataset.py:57-59): disjoint per rank, covering the permutation, per-epoch reshuffle."""
    from torch.utils.data import DistributedSampler
    from few_shot_seg_cwt_amd.dataset import EpisodeSampler
    for n in (1, 7, 8, 13, 5953):
        for world in (1, 2, 3, 8):
            shards = []
            for r in range(world):
                ours = EpisodeSampler(n, r, world, shuffle=True)
                ref = DistributedSampler(list(range(n)), num_replicas=world, rank=r, shuffle=True)
                for ep in (0, 1):
                    ours.set_epoch(ep)
                    ref.set_epoch(ep)
                    assert list(ours) == list(ref)
                shards.append(list(ours))
                assert len(ours) == len(ref)
            flat = sum(shards, [])
            assert set(flat) == set(range(n))
            if n % world == 0:
                assert len(flat) == len(set(flat)) == n
