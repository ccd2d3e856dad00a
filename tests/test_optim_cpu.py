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


def test_flat_store_versions_and_fp8_alignment():
    """FlatParams bookkeeping behind the derived weight copies (VGG's prepared conv layouts, the fp8 MLP's MX
    copy): every update path moves the parameter's version; align=128 holds through a relayout."""
    from ddpx.models import MLP
    from ddpx.runtime.flat_params import FlatParams
    m = MLP(hidden=256)
    f = FlatParams(m, align=128)
    assert all(o % 128 == 0 for o in f.offsets) and f.total % 128 == 0
    w = m.fc1.weight
    v0 = f.version_of(w)
    f.mark_updated(w)
    assert f.version_of(w) == v0 + 1
    i = f.index[id(w)]
    o, n = f.offsets[i], f.numels[i]
    f.fp8_mark(o, o + n, False)  # a flat update of exactly this parameter's range
    assert f.version_of(w) == v0 + 2
    others = [f.version_of(p) for p in f.params if p is not w]
    f.refresh_shadow()  # e.g. a checkpoint load: everything moves past any version held before
    assert all(f.version_of(p) > max(others + [v0 + 2]) for p in f.params)
    held = {id(p): f.version_of(p) for p in f.params}
    f.relayout([[j] for j in reversed(range(len(f.params)))], pad_to=64)
    assert all(o % 128 == 0 for o in f.offsets) and f.total % 128 == 0
    assert all(f.version_of(p) > held[id(p)] for p in f.params)
    # the fp8 copy exists only once enabled; its views are 128-aligned per parameter
    assert f.mx8_views(w) is None
    f.enable_fp8_shadow()
    q, s = f.mx8_views(w)
    assert q.shape == w.shape and s.shape == (w.shape[0], w.shape[1] // 32)
    assert not f.fp8_fresh[f.index[id(w)]]
    f.mark_updated(w, fp8_written=True)
    assert f.fp8_fresh[f.index[id(w)]]
    f.fp8_mark(0, f.total, False)
    assert not any(f.fp8_fresh)
