"""Data-parallel path on CPU with the gloo backend.

Checks, with the CPU oracle computing per-rank gradients:
* the flat-gradient all-reduce used by the fused step (parallel.make_allreduce)
  sums exactly;
* sharding a length-sorted global batch round-robin gives each rank a
  length-sorted shard of (nearly) equal frame count;
* summed per-rank gradients (loss_r = (em_r + off_r + kl_r) / B_global, kl_r
  with the per-rank B_r and the global N) equal the gradient of the reference
  loss on the concatenated global batch -- for 2 equal shards and for 3
  unequal ones (8 = 3 + 3 + 2 segments): the invariant that makes one
  all-reduce per step exact.
* learning.py's host side of the same: the shard of a global batch with fewer
  segments than ranks is empty (the rank joins the all-reduce with zero
  gradients), and the per-rank Philox keys differ while rank 0 keeps the
  single-device stream."""
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
    _, grads, _, _, _ = O.train_step(P, batch, cfg, dict(feat=None, eps=eps), 40, pretrain=True,
                                     loss_batch=len(lengths))
    flat = torch.cat([v.reshape(-1) for v in grads.values()])
    allreduce = parallel.make_allreduce()
    allreduce(flat)
    q.put((rank, mine, L, eps, flat))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_dp_ranks_equal_global_batch(world):
    from oracle import abcd_oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + (os.getpid() * 7 + world * 131) % 1000
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    flat0 = res[0][4]
    for r in res[1:]:
        assert torch.equal(r[4], flat0)  # every rank holds the same summed gradient
    assert sorted(sum((r[1] for r in res), [])) == list(range(8))
    Ls = [r[2] for r in res]
    assert max(Ls) - min(Ls) <= 9
    # global-batch gradient with the same per-row noise (eps rows follow their segment)
    F = 17
    cfg = O.default_cfg(F=F, H=16, Hdec=16, Hm=16, D=16, K=16)
    P = O.init_params(cfg, 1111)
    seqs = _global_batch(F, [9, 8, 8, 7, 5, 5, 3, 2])
    # each rank's eps is per packed row; unpack per segment to rebuild the global packed eps
    per_seg = {}
    for _, mine, _, eps, _ in res:
        b, order = _pack([seqs[i] for i in mine])
        segs = torch.nn.utils.rnn.unpack_sequence(torch.nn.utils.rnn.PackedSequence(eps, b["batch_sizes"]))
        for k, i in enumerate(order):
            per_seg[mine[i]] = segs[k]
    gb, gorder = _pack(seqs)
    geps = torch.nn.utils.rnn.pack_sequence([per_seg[i] for i in gorder]).data
    # loss on the global batch with B = 8 = the sum of the rank losses (each / 8)
    _, grads, _, _, _ = O.train_step(P, gb, cfg, dict(feat=None, eps=geps), 40, pretrain=True)
    gflat = torch.cat([v.reshape(-1) for v in grads.values()])
    err = (gflat - flat0).abs().max().item() / gflat.abs().max().item()
    assert err < 1e-5, err


class _FakeLearner:
    def __init__(self, rank, world):
        self.rank, self.world = rank, world


def test_shard_host_side_empty_and_unequal():
    import learning
    seqs = _global_batch(5, [6, 4, 3])
    packed = torch.nn.utils.rnn.pack_sequence(seqs)
    off = torch.nn.utils.rnn.pack_sequence([torch.tensor([0.0] * (len(s) - 1) + [1.0]) for s in seqs])
    spk = torch.tensor([0, 1, 2])
    shards = [learning.Learner._shard(_FakeLearner(r, 4), packed, off, spk) for r in range(4)]
    assert shards[3] is None  # 3 segments over 4 ranks: rank 3 joins the all-reduce with zero gradients
    got = sorted(int(s[2][0]) for s in shards[:3])
    assert got == [0, 1, 2]
    for s in shards[:3]:
        assert int(s[0].batch_sizes[0]) == 1 and torch.equal(s[0].data, seqs[int(s[2][0])])


def test_philox_keys_per_rank():
    from modules import noise
    noise.manual_seed(1234)
    k0 = noise.get_state()["seed"]
    assert k0 == 1234  # rank 0 = the single-device stream
    keys = set()
    for r in range(8):
        noise.manual_seed(1234, rank=r)
        keys.add(noise.get_state()["seed"])
    assert len(keys) == 8 and k0 in keys
    # a checkpoint's state (rank 0's) re-keys per rank on restore
    noise.manual_seed(1234)
    st = dict(noise.get_state(), offset=96)
    noise.set_state(st, rank=3)
    s3 = noise.get_state()
    noise.manual_seed(1234, rank=3)
    assert s3["seed"] == noise.get_state()["seed"] and s3["offset"] == 96
    noise.manual_seed(1234)
