"""The bench line's parity anchor as a test: one HIP training step at the
bench configurations' shapes (b = 64 sub-batch of the c2 / c4 / c5 / c5gru
workloads: F = 129, H = 256, K = 128 / 1024, LSTM / GRU, plain; the
frame-parallel GEMMs on their production kernels) against the oracle step on
the same weights and replayed noise.  Logits within 1e-4 absolute, argmax categories identical,
reconstruction loss within 1e-5 relative."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("name", ["c2", "c4", "c5", "c5gru"])
def test_bench_parity_anchor(name):
    sys.path.insert(0, REPO)
    import bench
    cfg = bench.CONFIGS[name]
    _, parity = bench.cpu_baseline(cfg, name, "cuda", min_steps=0)
    assert parity["recon_loss_rel_delta"] <= 1e-5, parity
    if not cfg["plain"]:  # (c4: the plain Gaussian sampler has no categories)
        assert parity["argmax_equal"], parity
        assert parity["logits_max_abs_diff"] <= 1e-4, parity
