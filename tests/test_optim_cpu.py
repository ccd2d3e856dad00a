"""ddpx.optim.SGD (flat, fused) vs torch.optim.SGD on the reference hyper-parameters."""
import torch
import torch.nn.functional as F
from torch.optim.lr_scheduler import LambdaLR

import ddpx
from ddpx.models import DeepNN, VGG
from ddpx.optim.schedule import OneCycleLambda
from ddpx.optim.sgd import SGD


def _train(model, opt, sched, steps, seed=0):
    g = torch.Generator().manual_seed(seed)
    for _ in range(steps):
        x = torch.rand((8, 3, 32, 32), generator=g)
        t = torch.randint(0, 10, (8,), generator=g)
        opt.zero_grad()
        F.cross_entropy(model(x), t).backward()
        opt.step()
        sched.step()


def test_sgd_matches_torch_deepnn():
    torch.manual_seed(0)
    a = DeepNN()
    a.classifier[2].p = 0.0  # dropout off for determinism
    b = DeepNN()
    b.classifier[2].p = 0.0
    b.load_state_dict(a.state_dict())
    ddpx.prepare_model(a, "cpu")
    oa = SGD(a.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4)
    ob = torch.optim.SGD(b.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4)
    _train(a, oa, LambdaLR(oa, OneCycleLambda(4)), 6)
    _train(b, ob, LambdaLR(ob, OneCycleLambda(4)), 6)
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.allclose(p, q, atol=1e-5, rtol=1e-4), n


def test_sgd_state_dict_roundtrip():
    torch.manual_seed(0)
    a = VGG()
    ddpx.prepare_model(a, "cpu")
    oa = SGD(a.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
    _train(a, oa, LambdaLR(oa, lambda s: 1.0), 1)
    sd = oa.state_dict()
    assert len(sd["state"]) == 26
    b = VGG()
    b.load_state_dict(a.state_dict())
    ddpx.prepare_model(b, "cpu")
    ob = SGD(b.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
    ob.load_state_dict(sd)
    assert torch.equal(oa.momentum_buffer, ob.momentum_buffer)
