"""Standalone module surface the training step does not use but the reference
exposes: ``MLP.forward`` (model.py:316-334) and ``RNN_Cell.forward``
(model.py:287-300), both trainable through autograd on the HIP GEMMs
(``abcd::linear`` / ``abcd::linear_bwd``), against torch's own modules in
float64 on the CPU (the ops the reference's modules are)."""
import pytest
import torch

from gpu_helpers import modules_api, rel_err

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("In,Hid,Out,B", [(33, 40, 7, 50), (256, 256, 256, 512), (9, 16, 1, 3)])
def test_mlp_trains_like_torch(In, Hid, Out, B):
    M = modules_api()
    torch.manual_seed(3)
    mlp = M.MLP(In, Hid, Out)
    ref = torch.nn.Sequential(torch.nn.Linear(In, Hid), torch.nn.Tanh(), torch.nn.Linear(Hid, Out)).double()
    ref.load_state_dict({k: v.double() for k, v in mlp.whole_network.state_dict().items()})
    mlp.cuda()
    x = torch.randn(B, In)
    dy = torch.randn(B, Out)
    y = mlp(x.cuda())
    (y * dy.cuda()).sum().backward()
    yr = ref(x.double())
    (yr * dy.double()).sum().backward()
    assert rel_err(y, yr) < 1e-5
    for (k, p), (_, pr) in zip(mlp.whole_network.named_parameters(), ref.named_parameters()):
        assert rel_err(p.grad, pr.grad) < 1e-5, k
    # inference (no grad) takes the same path
    with torch.no_grad():
        assert torch.equal(mlp(x.cuda()), y.detach())


@pytest.mark.parametrize("mode", ["LSTM", "GRU"])
def test_rnn_cell_step_like_torch(mode):
    M = modules_api()
    torch.manual_seed(4)
    F, H, B = 33, 24, 10
    cell = M.RNN_Cell(F, H, model_type=mode)
    ref = getattr(torch.nn, mode + "Cell")(F, H).double()
    ref.load_state_dict({k: v.double() for k, v in cell.cell.state_dict().items()})
    cell.cuda()
    x = torch.randn(B, F)
    h0 = torch.randn(B, H)
    c0 = torch.randn(B, H)
    dh = torch.randn(B, H)
    if mode == "LSTM":
        h, c = cell(x.cuda(), (h0.cuda(), c0.cuda()))
        hr, cr = ref(x.double(), (h0.double(), c0.double()))
        (h * dh.cuda()).sum().add(c.sum()).backward()
        (hr * dh.double()).sum().add(cr.sum()).backward()
        assert rel_err(c, cr) < 1e-5
    else:
        h = cell(x.cuda(), h0.cuda())
        hr = ref(x.double(), h0.double())
        (h * dh.cuda()).sum().backward()
        (hr * dh.double()).sum().backward()
    assert rel_err(h, hr) < 1e-5
    for (k, p), (_, pr) in zip(cell.cell.named_parameters(), ref.named_parameters()):
        assert rel_err(p.grad, pr.grad) < 1e-5, k
