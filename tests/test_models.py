"""Model zoo: exact reference state_dict format, parameter counts, model size."""
from collections import OrderedDict, defaultdict

import pytest
import torch
from torch import nn

from ddpx.models import MLP, VGG, DeepNN
from ddpx.utils.size import MiB, get_model_size


class VanillaVGG(nn.Module):
    """Independent plain-torch re-statement of the reference VGG used as the
    loader for checkpoint-compatibility checks."""

    def __init__(self):
        super().__init__()
        arch = [64, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"]
        layers, cnt, cin = [], defaultdict(int), 3
        for x in arch:
            if x == "M":
                layers.append((f"pool{cnt['pool']}", nn.MaxPool2d(2)))
                cnt["pool"] += 1
            else:
                layers.append((f"conv{cnt['conv']}", nn.Conv2d(cin, x, 3, padding=1, bias=False)))
                layers.append((f"bn{cnt['bn']}", nn.BatchNorm2d(x)))
                layers.append((f"relu{cnt['relu']}", nn.ReLU(True)))
                cnt["conv"] += 1
                cnt["bn"] += 1
                cnt["relu"] += 1
                cin = x
        self.backbone = nn.Sequential(OrderedDict(layers))
        self.classifier = nn.Linear(512, 10)

    def forward(self, x):
        return self.classifier(self.backbone(x).mean([2, 3]))


def test_vgg_state_dict_format():
    sd = VGG().state_dict()
    assert len(sd) == 50
    keys = list(sd.keys())
    chans = [(3, 64), (64, 128), (128, 256), (256, 256), (256, 512), (512, 512), (512, 512), (512, 512)]
    expect = []
    for i, (ci, co) in enumerate(chans):
        expect.append((f"backbone.conv{i}.weight", (co, ci, 3, 3), torch.float32))
        for n in ("weight", "bias", "running_mean", "running_var"):
            expect.append((f"backbone.bn{i}.{n}", (co,), torch.float32))
        expect.append((f"backbone.bn{i}.num_batches_tracked", (), torch.int64))
    expect += [("classifier.weight", (10, 512), torch.float32), ("classifier.bias", (10,), torch.float32)]
    assert keys == [e[0] for e in expect]
    for k, shape, dt in expect:
        assert tuple(sd[k].shape) == shape and sd[k].dtype == dt, k
    VanillaVGG().load_state_dict(sd, strict=True)


def test_param_counts_and_size():
    vgg = VGG()
    assert sum(p.numel() for p in vgg.parameters()) == 9228362
    assert len(list(vgg.parameters())) == 26
    assert f"{get_model_size(vgg) / MiB:.2f}" == "35.20"
    assert sum(p.numel() for p in DeepNN().parameters()) == 1186986
    toy = MLP(hidden=4096, layers=3)
    assert sum(p.numel() for p in toy.parameters()) == 3072 * 4096 + 4096 + 4096 * 4096 + 4096 + 4096 * 10 + 10
    assert list(toy.state_dict().keys()) == ["fc0.weight", "fc0.bias", "fc1.weight", "fc1.bias", "fc2.weight",
                                             "fc2.bias"]


def test_vgg_forward_matches_vanilla():
    torch.manual_seed(0)
    a, b = VGG(), VanillaVGG()
    b.load_state_dict(a.state_dict())
    x = torch.rand(4, 3, 32, 32)
    a.eval()
    b.eval()
    assert torch.allclose(a(x), b(x), atol=1e-5)


def test_flat_params_views_and_grad_routing():
    import ddpx
    from ddpx.runtime.flat_params import flat_of
    torch.manual_seed(0)
    m = DeepNN()
    ref = DeepNN()
    ref.load_state_dict(m.state_dict())
    f = ddpx.prepare_model(m, "cpu")
    assert flat_of(m) is f
    for p in m.parameters():
        assert p.data_ptr() >= f.master.data_ptr()
        assert (p.data_ptr() - f.master.data_ptr()) % 256 == 0  # 64-element aligned offsets
    # state dict unchanged by flattening
    for (k, v), (k2, v2) in zip(m.state_dict().items(), ref.state_dict().items()):
        assert k == k2 and torch.equal(v, v2)
    x = torch.rand(8, 3, 32, 32)
    m.eval()
    ref.eval()
    m(x).sum().backward()
    ref(x).sum().backward()
    for p, q in zip(m.parameters(), ref.parameters()):
        assert p.grad is None
        assert torch.allclose(p.main_grad, q.grad, atol=1e-6)


def test_mlp_cpu_forward_loss():
    import ddpx
    m = MLP(in_features=3072, hidden=64, layers=3)
    ddpx.prepare_model(m, "cpu")
    x = torch.rand(16, 3, 32, 32)
    t = torch.randint(0, 10, (16,))
    loss, logits = m.forward_loss(x, t)
    assert logits.shape == (16, 10)
    assert torch.allclose(loss, torch.nn.functional.cross_entropy(m(x), t))


def test_mlp_cpu_one_node_backward_matches_torch():
    """ops/mlp_cpu: the CPU training step writes the flat gradients directly (no per-parameter .grad), in
    grad-ready order, equal to torch autograd's, including accumulation over two backwards."""
    import copy

    import ddpx
    torch.manual_seed(0)
    m = MLP(in_features=3072, hidden=96, layers=4)
    ref = copy.deepcopy(m)
    ddpx.prepare_model(m, "cpu")
    flat = m.fc0.weight._ddpx_flat
    order = []
    orig = flat.grad_done
    pos = {id(p): i for i, p in enumerate(m.parameters())}  # fc0.w, fc0.b, ..., fc3.w, fc3.b
    flat.grad_done = lambda p, chunk=None: (order.append(pos[id(p)] // 2), orig(p, chunk))[1]
    x = torch.rand(24, 3, 32, 32)
    t = torch.randint(0, 10, (24,))
    for _ in range(2):
        loss, logits = m.forward_loss(x, t)
        loss.backward()
        l_ref = torch.nn.functional.cross_entropy(ref(x), t)
        l_ref.backward()
        assert torch.allclose(loss, l_ref, atol=1e-6)
    assert order[:8] == [3, 3, 2, 2, 1, 1, 0, 0]  # classifier first (gradient-ready order)
    for p, q in zip(m.parameters(), ref.parameters()):
        assert p.grad is None
        assert torch.allclose(p.main_grad, q.grad, atol=1e-6)
