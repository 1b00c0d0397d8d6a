"""Multi-GPU plumbing: one process per GPU, torch.distributed over RCCL ("nccl" backend on
ROCm) on the GPU box, gloo in the CPU tests.

The CWT path has exactly two data-path exchange points:
  * training: the mean of the CWT gradients, ONE all-reduce of the flat 2,098,688-float
    (H=4) bucket per step, before the identical SGD step on every rank;
  * inference: one sum all-reduce of the per-class intersection/union table at the end of
    a run (episodes are sharded round-robin, no data-path collective).
Off the data path, training also broadcasts the extractor's BN running statistics from rank 0
once per epoch, after the train-mode-BN episode (broadcast_backbone_bn_).
The reference's own DDP code (src/train_ddp.py:106-119) wraps a different model (MMN) and
is not runnable; this is the CWT's equivalent, not a translation of it.
"""
from __future__ import annotations

import os
import random
from typing import List, Tuple

import numpy as np
import torch
import torch.distributed as dist


def rank_world() -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend: str | None = None) -> Tuple[int, int, int]:
    """Initialise from torchrun's env (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*).  Returns
    (rank, local_rank, world)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, local, world


def seed_everything(manual_seed: int) -> int:
    """Per-rank seeding of every host RNG the episode path draws from, as the reference's
    multi-process trainer does it (src/train_ddp.py:62-66: ``manual_seed + rank`` for
    ``random``, ``np.random``, ``torch`` and the CUDA generators).  Each rank then draws its own
    episodes' support/query choice and its own classifier init W0 (train.py:206).  Returns the
    seed used."""
    rank, _ = rank_world()
    s = int(manual_seed) + rank
    random.seed(s)
    np.random.seed(s)
    torch.manual_seed(s)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(s)
    return s


def broadcast_params_(flat: torch.Tensor, src: int = 0) -> torch.Tensor:
    """Make every rank start from rank ``src``'s parameters: one broadcast of the flat CWT
    parameter buffer (transformer.flat).  This is what ``DDP(module)`` does at construction
    (src/train_ddp.py:119); with per-rank seeds the modules' random inits differ otherwise.
    No-op at world size 1."""
    _, world = rank_world()
    if world > 1:
        if flat.device.type == _reduce_device().type:
            dist.broadcast(flat.data, src)
        else:
            t = flat.detach().to(_reduce_device())
            dist.broadcast(t, src)
            flat.data.copy_(t)
        # writes through .data do not bump the version counter that keys the transformer's
        # folded inference weights (MultiHeadAttentionOne.params_version): bump it here
        torch.autograd.graph.increment_version(flat)
    return flat


def shard_indices(n: int, rank: int, world: int, shuffle: bool, seed: int = 0, epoch: int = 0) -> List[int]:
    """The indices ``torch.utils.data.DistributedSampler(dataset)`` hands rank ``rank`` in
    epoch ``epoch`` (the reference's train sampler, src/dataset/dataset.py:57-59): a
    permutation drawn from a generator seeded ``seed + epoch`` (identical on every rank), padded
    by wrapping to a multiple of ``world``, then every ``world``-th entry from ``rank``.  Ranks get
    disjoint positions of one permutation; with world 1 and shuffle off it is range(n)."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(int(seed) + int(epoch))
        idx = torch.randperm(n, generator=g).tolist()
    else:
        idx = list(range(n))
    per = -(-n // world) if n else 0
    total = per * world
    if total > len(idx) and idx:
        pad = total - len(idx)
        idx += (idx * (-(-pad // len(idx))))[:pad]
    return idx[rank:total:world]


def all_reduce_mean_(t: torch.Tensor) -> torch.Tensor:
    """In-place mean over ranks of one flat bucket (the CWT gradient); staged through the host
    when the backend's device is not the tensor's (gloo with device tensors)."""
    _, world = rank_world()
    if world > 1:
        if t.device.type == _reduce_device().type:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)
            t.div_(world)
        else:
            h = t.detach().to(_reduce_device())
            dist.all_reduce(h, op=dist.ReduceOp.SUM)
            t.copy_(h.div_(world))
    return t


def _reduce_device() -> torch.device:
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_sum_np(a: np.ndarray) -> np.ndarray:
    _, world = rank_world()
    if world == 1:
        return a
    t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(_reduce_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy()


def all_reduce_mean_scalar(x: float) -> float:
    _, world = rank_world()
    if world == 1:
        return x
    return float(all_reduce_sum_np(np.array([x]))[0] / world)


def all_reduce_max_scalar(x: float) -> float:
    _, world = rank_world()
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_reduce_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def union_keys(keys: List[int], max_keys: int = 128) -> List[int]:
    """Union of integer class ids over ranks (fixed-size all-reduce of a presence mask)."""
    _, world = rank_world()
    if world == 1:
        return sorted(keys)
    mask = np.zeros(max_keys)
    for k in keys:
        mask[int(k)] = 1
    mask = all_reduce_sum_np(mask)
    return [i for i in range(max_keys) if mask[i] > 0]


def barrier():
    if rank_world()[1] > 1:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def broadcast_running_stats_(state: dict, src: int = 0) -> dict:
    """Replace every ``*.running_mean`` / ``*.running_var`` entry of ``state`` (a state dict of
    torch tensors or numpy arrays) by rank ``src``'s, in ONE broadcast of the flat fp32 bucket.
    Other entries are left alone.  No-op at world size 1."""
    _, world = rank_world()
    keys = sorted(k for k in state if k.endswith((".running_mean", ".running_var")))
    if world == 1 or not keys:
        return state
    vals = [torch.as_tensor(np.asarray(state[k]), dtype=torch.float32) for k in keys]
    flat = torch.cat([v.reshape(-1) for v in vals]).to(_reduce_device())
    dist.broadcast(flat, src)
    flat = flat.cpu()
    off = 0
    for k, v in zip(keys, vals):
        state[k] = flat[off:off + v.numel()].reshape(v.shape).clone()
        off += v.numel()
    return state


def broadcast_backbone_bn_(model, src: int = 0):
    """After the first episode of an epoch has moved each rank's BN running statistics with its
    own batch statistics (train.py:184,245), every rank takes rank ``src``'s,
    so the replicas extract identical features from that episode's query pass on.

    Declared deviation: the reference's multi-process idiom wraps the extractor in
    ``SyncBatchNorm`` (src/train_ddp.py:106), whose batch statistics span all ranks' batches; here
    each rank's train-mode support pass normalises over its own batch (the CWT trainer the
    north star names, src/train.py, is single-process, where the two agree), and the broadcast
    keeps the replicas identical afterwards, as DDP's ``broadcast_buffers`` would."""
    rank, world = rank_world()
    if world == 1:
        return model
    sd = broadcast_running_stats_(model.state_dict(), src)
    if rank != src:
        model.load_state_dict(sd)
    return model
