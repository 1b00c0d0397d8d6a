"""The multi-rank training path on real kernels: do_epoch over two ranks that
share the one GPU of the box, gloo for the exchange (RCCL refuses two ranks on one device; the
exchange points are the same calls).  Each rank runs the HIP train_episode on its
DistributedSampler-style shard with its own seed; the test checks rank 0's parameters reach
rank 1 (broadcast), disjoint episodes, distinct W0, bit-identical replicas after every step, and
that the final parameters equal a replay of torch.optim.SGD on the mean of the two ranks' local
(pre-all-reduce) gradients."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK="0")
    torch.set_num_threads(2)
    torch.cuda.set_device(0)
    from few_shot_seg_cwt_amd import dist as cdist
    from few_shot_seg_cwt_amd import episode, get_model
    from few_shot_seg_cwt_amd import synthetic as syn
    from few_shot_seg_cwt_amd.transformer import MultiHeadAttentionOne
    cdist.init_from_env(backend="gloo")
    assert cdist.seed_everything(2021) == 2021 + rank
    dev = torch.device("cuda", 0)
    S, n_iter = 65, 2
    cfg = syn.cfg_defaults(image_size=S, pipeline=0)
    model = get_model(cfg)
    model.load_state_dict(syn.make_pspnet_state(50, 2021))
    t = MultiHeadAttentionOne(4, 512, 512, 512, dropout=0.0).to(dev)
    p0 = [torch.zeros_like(t.flat.data.cpu()) for _ in range(WORLD)]
    torch.distributed.all_gather(p0, t.flat.data.cpu().clone())
    assert not torch.equal(p0[0], p0[1])
    opt = torch.optim.SGD([t.flat], lr=1e-3, momentum=0.9, weight_decay=1e-4, nesterov=True)
    loader = episode.SyntheticEpisodes(n_iter * WORLD, S=S, seed=2021).shard(rank, WORLD)
    seen = []
    real = episode.train_episode

    def recording(model_, transformer, args, batch, W0, dev_):
        out = real(model_, transformer, args, batch, W0, dev_)
        torch.cuda.synchronize()
        seen.append((float(batch[0].double().sum()), W0.detach().cpu().clone(),
                     transformer.flat.grad.detach().cpu().clone()))
        return out

    episode.train_episode = recording
    episode.do_epoch(cfg, loader, model, t, opt, epoch=0, iter_per_epoch=n_iter, log_iter=n_iter)
    torch.cuda.synchronize()
    assert len(seen) == n_iter
    flat = t.flat.data.cpu().clone()
    pf = [torch.zeros_like(flat) for _ in range(WORLD)]
    torch.distributed.all_gather(pf, flat)
    assert torch.equal(pf[0], pf[1]), "replicas diverged"
    ids = torch.tensor([s[0] for s in seen], dtype=torch.float64)
    w0 = torch.stack([s[1] for s in seen])
    all_ids = [torch.zeros_like(ids) for _ in range(WORLD)]
    all_w0 = [torch.zeros_like(w0) for _ in range(WORLD)]
    torch.distributed.all_gather(all_ids, ids)
    torch.distributed.all_gather(all_w0, w0)
    assert not set(all_ids[0].tolist()) & set(all_ids[1].tolist()), "ranks trained on the same episode"
    assert not torch.equal(all_w0[0], all_w0[1]), "ranks drew the same classifier init"
    local = torch.stack([s[2] for s in seen])
    all_local = [torch.zeros_like(local) for _ in range(WORLD)]
    torch.distributed.all_gather(all_local, local)
    ref = torch.nn.Parameter(p0[0].clone())
    ref_opt = torch.optim.SGD([ref], lr=1e-3, momentum=0.9, weight_decay=1e-4, nesterov=True)
    for k in range(n_iter):
        ref.grad = (all_local[0][k] + all_local[1][k]) / 2
        ref_opt.step()
    err = float((ref.data - flat).abs().max() / ref.data.abs().max())
    assert err < 1e-6, err
    torch.distributed.destroy_process_group()
    open(os.path.join(out_dir, f"gpu_tr{rank}"), "w").write(f"{err}")


def test_do_epoch_two_ranks_on_device(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    port = _free_port()
    mp.spawn(_worker, args=(port, str(tmp_path)), nprocs=WORLD, join=True)
    errs = [float((tmp_path / f"gpu_tr{r}").read_text()) for r in range(WORLD)]
    print(f"two-rank do_epoch on the device: replay error {max(errs):.2e}")
