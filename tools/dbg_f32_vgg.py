import copy, torch, torch.nn.functional as F, sys
sys.path.insert(0, "/root/repo")
import ddpx
from ddpx.models import build_model
from ddpx.ops import f32
gpu = torch.device("cuda", 0)
torch.manual_seed(7)
native = build_model("vgg", dtype="fp32", device=gpu)
r64 = copy.deepcopy(native).cpu().double(); r64.use_native = False
flat = ddpx.prepare_model(native, gpu)
x = torch.rand(64, 3, 32, 32, device=gpu); y = torch.randint(0, 10, (64,), device=gpu)
rec = {}
orig_bwd, orig_fwd = f32.bn_backward, f32.bn_forward
def bwd(g, yy, *a, **k):
    out = orig_bwd(g, yy, *a, **k); rec.setdefault("dy", []).append((g.clone(), out.clone())); return out
def fwd(yy, *a, **k):
    out = orig_fwd(yy, *a, **k); rec.setdefault("y", []).append((yy.clone(), out[0].clone())); return out
f32.bn_backward, f32.bn_forward = bwd, fwd
flat.zero_grad()
loss, _ = native.forward_loss(x, y); loss.backward(); torch.cuda.synchronize()
grads, outs = {}, {}
hs = []
for i in range(8):
    conv = getattr(r64.backbone, f"conv{i}"); bnm = getattr(r64.backbone, f"bn{i}")
    hs.append(conv.register_full_backward_hook(lambda m, gi, go, i=i: grads.__setitem__(i, go[0].detach())))
    hs.append(conv.register_forward_hook(lambda m, inp, o, i=i: outs.__setitem__(i, o.detach())))
hs.append(r64.backbone.pool3.register_full_backward_hook(lambda m, gi, go: grads.__setitem__("p3", go[0].detach())))
xr = x.cpu().double().requires_grad_(True)
F.cross_entropy(r64(xr), y.cpu()).backward()
rel = lambda a, b: ((a.double() - b).norm() / b.norm()).item()
for i in range(8):
    yv, _ = rec["y"][i]
    N, C, H, W = outs[i].shape
    print(i, "y err", rel(yv.cpu(), outs[i].permute(0, 2, 3, 1).reshape(-1, C)), end=" ")
    g, dy = rec["dy"][7 - i]
    print("dy err", rel(dy.cpu(), grads[i].permute(0, 2, 3, 1).reshape(-1, C)))
# layer-7 BN backward recomputed in fp64 from the native kernel's own inputs
g7, dy7 = rec["dy"][0]
y7, _ = rec["y"][7]
N, C, H, W = outs[7].shape
bn = copy.deepcopy(r64.backbone.bn7).train()
yy = y7.cpu().double().view(N, H, W, C).permute(0, 3, 1, 2).clone().requires_grad_(True)
z = F.max_pool2d(torch.relu(bn(yy)), 2)
z.backward(g7.cpu().double().permute(0, 3, 1, 2))
print("dy7 kernel vs fp64-from-same-inputs", rel(dy7.cpu(), yy.grad.permute(0, 2, 3, 1).reshape(-1, C)))
gp = grads["p3"].permute(0, 2, 3, 1)
print("g7 err vs fp64", rel(g7.cpu(), gp))
# routing: argmax of each 2x2 window from native y7 vs fp64 y7
def arg(yv):
    z = torch.relu(bn(yv)).detach()
    _, idx = F.max_pool2d(z, 2, return_indices=True)
    return idx, z
i_nat, z_nat = arg(y7.cpu().double().view(N, H, W, C).permute(0, 3, 1, 2))
i_ref, z_ref = arg(outs[7])
print("routing flips", (i_nat != i_ref).sum().item(), "of", i_nat.numel(), "zeros in z", (z_ref == 0).float().mean().item())
