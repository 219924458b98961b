"""Data-parallel path on CPU with the gloo backend, world_size 2.

Checks, with the CPU oracle computing per-rank gradients:
* the flat-gradient all-reduce used by the fused step (parallel.make_allreduce)
  averages exactly;
* sharding a length-sorted global batch round-robin gives each rank a
  length-sorted shard of (nearly) equal frame count;
* averaged per-rank gradients (loss_r = (em_r + off_r + kl_r) / B_r, kl_r with
  the per-rank B_r and the global N) equal the gradient of the reference loss
  on the concatenated global batch -- the invariant that makes one all-reduce
  per step exact."""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "seq2seq_abcd-vae_amd"), HERE]


def _global_batch(F, lengths, seed=3):
    g = torch.Generator().manual_seed(seed)
    seqs = [torch.randn(T, F, generator=g) for T in lengths]
    return seqs


def _pack(seqs):
    order = sorted(range(len(seqs)), key=lambda i: -len(seqs[i]))
    seqs = [seqs[i] for i in order]
    p = torch.nn.utils.rnn.pack_sequence(seqs)
    off = torch.nn.utils.rnn.pack_sequence([torch.tensor([0.0] * (len(s) - 1) + [1.0]) for s in seqs]).data
    return dict(data=p.data, batch_sizes=p.batch_sizes, is_offset=off), order


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from modules import parallel
    from oracle import abcd_oracle as O
    F = 17
    cfg = O.default_cfg(F=F, H=16, Hdec=16, Hm=16, D=16, K=16)
    P = O.init_params(cfg, 1111)
    lengths = [9, 8, 8, 7, 5, 5, 3, 2]
    seqs = _global_batch(F, lengths)
    mine = parallel.shard_global_batch([len(s) for s in seqs], rank, world)
    batch, order = _pack([seqs[i] for i in mine])
    L = batch["data"].shape[0]
    g = torch.Generator().manual_seed(100 + rank)
    eps = torch.randn(L, F, generator=g)
    _, grads, _, _, _ = O.train_step(P, batch, cfg, dict(feat=None, eps=eps), 40, pretrain=True)
    flat = torch.cat([v.reshape(-1) for v in grads.values()])
    allreduce = parallel.make_allreduce()
    allreduce(flat)
    q.put((rank, mine, L, eps, flat))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_two_ranks_equals_global_batch():
    from oracle import abcd_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (r0, mine0, L0, eps0, flat0), (r1, mine1, L1, eps1, flat1) = res
    assert torch.equal(flat0, flat1)  # every rank holds the same averaged gradient
    assert sorted(mine0 + mine1) == list(range(8)) and abs(L0 - L1) <= 3
    # global-batch gradient with the same per-row noise (eps rows follow their segment)
    F = 17
    cfg = O.default_cfg(F=F, H=16, Hdec=16, Hm=16, D=16, K=16)
    P = O.init_params(cfg, 1111)
    seqs = _global_batch(F, [9, 8, 8, 7, 5, 5, 3, 2])
    # each rank's eps is per packed row; unpack per segment to rebuild the global packed eps
    per_seg = {}
    for mine, eps in ((mine0, eps0), (mine1, eps1)):
        b, order = _pack([seqs[i] for i in mine])
        segs = torch.nn.utils.rnn.unpack_sequence(torch.nn.utils.rnn.PackedSequence(eps, b["batch_sizes"]))
        for k, i in enumerate(order):
            per_seg[mine[i]] = segs[k]
    gb, gorder = _pack(seqs)
    geps = torch.nn.utils.rnn.pack_sequence([per_seg[i] for i in gorder]).data
    # loss on the global batch with B = 8: mean of the two rank losses when B_r = 4 each
    _, grads, _, _, _ = O.train_step(P, gb, cfg, dict(feat=None, eps=geps), 40, pretrain=True)
    gflat = torch.cat([v.reshape(-1) for v in grads.values()])
    err = (gflat - flat0).abs().max().item() / gflat.abs().max().item()
    assert err < 1e-5, err
