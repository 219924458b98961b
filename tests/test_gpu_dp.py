"""Data parallelism through the real fused step on one GPU (SURVEY.md §4
item 5): the production-shape global batch of
tests/golden/prod_lstm_k128.npz (B = 72, F = 129, H = 256, K = 128) is split
into length-balanced shards (parallel.shard_global_batch), each shard runs
FusedStep with the global loss normaliser, and a fake all-reduce hook (the
FusedStep.allreduce slot parallel.attach fills with RCCL) sums the shards'
flat gradients before clip + SGD.  The result must equal the REFERENCE's
global-batch step (learning.py:155-163: loss / batch_sizes[0], clip after the
reduce).  World sizes 2 and 3 (unequal shards: 24 + 24 + 24 and 36 + 36)."""
import pytest
import torch

from golden_io import load_prod, prod_inputs
from gpu_helpers import named_params, rel_err
from test_prod_fixtures import build_product

pytestmark = pytest.mark.gpu


def _shard_inputs(inp, mine):
    """Rows `mine` (indices into the length-sorted global batch) re-packed,
    with each segment's noise following it (Gumbel row, per-frame eps)."""
    bs = inp["batch_sizes"]
    segs = torch.nn.utils.rnn.unpack_sequence(torch.nn.utils.rnn.PackedSequence(inp["data"], bs))
    eps = torch.nn.utils.rnn.unpack_sequence(torch.nn.utils.rnn.PackedSequence(inp["eps"], bs))
    offs = torch.nn.utils.rnn.unpack_sequence(torch.nn.utils.rnn.PackedSequence(inp["is_offset"], bs))
    p = torch.nn.utils.rnn.pack_sequence([segs[i] for i in mine])
    return dict(data=p.data, batch_sizes=p.batch_sizes,
                eps=torch.nn.utils.rnn.pack_sequence([eps[i] for i in mine]).data,
                is_offset=torch.nn.utils.rnn.pack_sequence([offs[i] for i in mine]).data,
                speakers=inp["speakers"][mine],
                feat_noise=None if inp["feat_noise"] is None else inp["feat_noise"][mine])


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_fused_step_equals_reference_global_batch(world):
    from modules import engine, noise, parallel
    meta, arr = load_prod("lstm_k128")
    inp = prod_inputs(meta)
    B = meta["B"]
    enc, samp, dec = build_product(meta, "cuda")
    step = engine.FusedStep(enc, samp, dec)
    named = named_params(enc, samp, dec)
    init = {k: p.detach().clone() for k, p in named.items()}
    lengths = [int(x) for x in inp["lengths"]]
    shards = [parallel.shard_global_batch(lengths, r, world) for r in range(world)]
    assert sorted(sum(shards, [])) == list(range(B))
    grads, loss = [], 0.0
    for r in range(world - 1, -1, -1):  # rank 0 last: its step applies clip + SGD
        s = _shard_inputs(inp, shards[r])
        noise.replay(*([s["feat_noise"]] if s["feat_noise"] is not None else []), s["eps"])
        sc, _ = step.forward_backward(s["data"].cuda(), s["batch_sizes"], s["is_offset"].cuda(),
                                      s["speakers"].cuda(), meta["N"], loss_batch=B)
        loss += float(sc[engine.LOSS])
        if r:
            grads.append(step.flat.grad.clone())
    others = torch.stack(grads).sum(0)
    step.allreduce = lambda g: g.add_(others)  # the other ranks' contribution (SUM all-reduce)
    step.optimizer_step(lr=meta["lr"], momentum=0.0, clip=meta["clip"])
    torch.cuda.synchronize()
    assert abs(loss - float(arr["loss"])) <= 1e-4 * abs(float(arr["loss"])), (loss, float(arr["loss"]))
    assert abs(float(step.scalars[engine.NORM]) - float(arr["total_norm"])) <= 1e-4 * float(arr["total_norm"])
    for k, p in named.items():
        delta = p.detach().double().cpu() - init[k].double().cpu()
        ref_n = float(arr["dq_norm/" + k])
        assert abs(float(delta.norm()) - ref_n) <= 1e-3 * ref_n + 1e-9, (k, float(delta.norm()), ref_n)
        if "g/" + k in arr:  # clipped, scaled gradient = -delta / lr; compare directions via the full grad
            coef = min(1.0, meta["clip"] / (float(arr["total_norm"]) + 1e-6))
            assert rel_err(-delta / (meta["lr"] * coef), arr["g/" + k]) < 1e-3, k
