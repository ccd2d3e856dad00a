"""Debug: per-layer dy of the native SyncBN VGG on 2 ranks (one GPU) vs the full-batch process."""
import os
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from _dist_util import free_port, init_gloo  # noqa: E402


def worker(rank, ws, port):
    import ddpx
    from ddpx.models import VGG
    from ddpx.ops import conv as K
    from ddpx.parallel.comm import HostStagedComm
    from ddpx.parallel.ddp import DistributedDataParallel
    init_gloo(rank, ws, port)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(11)
    ours, ref = VGG(), VGG()
    ref.load_state_dict(ours.state_dict())
    comm = HostStagedComm()
    for m in (ours, ref):
        m.use_native = True
    ours.sync_bn_comm = comm
    ddpx.prepare_model(ours, dev)
    ddpx.prepare_model(ref, dev)
    d = DistributedDataParallel(ours, comm=comm, bucket_cap_mb=4.0)
    rec = {"ours": [], "ref": []}
    orig_s, orig = K.bn_backward_sync, K.bn_backward

    orig_ar = comm.allreduce_

    def ar_(t, op="avg", stream=None, async_op=False):
        if op == "sum" and t.numel() <= 1024:
            before = t.detach().clone()
            r = orig_ar(t, op, stream, async_op)
            rec.setdefault("ar", []).append((before, t.detach().clone()))
            return r
        return orig_ar(t, op, stream, async_op)
    comm.allreduce_ = ar_

    def ws_(*a, **k):
        out = orig_s(*a, **k)
        rec["ours"].append((a[0].float().clone(), out.float().clone()))
        rec.setdefault("oin", []).append([t.float().clone() for t in a[1:6]])
        # the same inputs through the LOCAL backward, and the sync backward re-run
        loc = orig(*a[:11])
        again = orig_s(*a[:12])
        rec.setdefault("loc", []).append((loc.float().clone(), again.float().clone()))
        return out

    def w_(*a, **k):
        out = orig(*a, **k)
        rec["ref"].append((a[0].float().clone(), out.float().clone()))
        rec.setdefault("rin", []).append([t.float().clone() for t in a[1:6]])
        return out
    K.bn_backward_sync, K.bn_backward = ws_, w_
    B = 32
    g = torch.Generator(device="cpu").manual_seed(500)
    xg = torch.rand(ws * B, 32, 32, 8, generator=g)
    xg[..., 3:] = 0
    xg = xg.to(dev).to(torch.bfloat16)
    tg = torch.randint(0, 10, (ws * B,), generator=g).to(dev)
    loss, _ = d.forward_loss(xg[rank * B:(rank + 1) * B], tg[rank * B:(rank + 1) * B])
    lr_, _ = ref.forward_loss(xg, tg)
    loss.backward()
    lr_.backward()
    torch.cuda.synchronize()
    for i, (bf, af) in enumerate(rec.get("ar", [])[:2]):
        both = [torch.empty_like(bf.cpu()) for _ in range(ws)]
        torch.distributed.all_gather(both, bf.cpu())
        print(f"rank {rank} sums {i}: local {bf[:3].tolist()} after {af[:3].tolist()} expect "
              f"{(both[0] + both[1])[:3].tolist()} n={bf.numel()}", flush=True)
    for li, ((go, do), (gr, dr)) in enumerate(zip(rec["ours"], rec["ref"])):
        n = go.shape[0]
        grs = gr.view(ws, -1)[rank].view_as(go) * ws
        drs = dr.view(ws, -1)[rank].view_as(do) * ws
        eg = ((go - grs).norm() / grs.norm()).item()
        ed = ((do - drs).norm() / drs.norm()).item()
        yo, ao, bo, mo, ro = rec["oin"][li]
        yr, ar, br, mr, rr = rec["rin"][li]
        yrs = yr.view(ws, -1)[rank].view_as(yo)
        print(f"rank {rank} layer {7 - li}: y {((yo - yrs).norm() / yrs.norm()).item():.2e} a {((ao - ar).norm() / ar.norm()).item():.2e} "
              f"b {((bo - br).norm() / br.norm().clamp_min(1e-9)).item():.2e} mean {((mo - mr).norm() / mr.norm()).item():.2e} "
              f"rstd {((ro - rr).norm() / rr.norm()).item():.2e}", flush=True)
        lo, ag = rec["loc"][li]
        el = ((do - lo).norm() / lo.norm()).item()
        ea = ((do - ag).norm() / ag.norm()).item()
        print(f"rank {rank} layer {7 - li}: g rel {eg:.4f}  dy rel {ed:.4f}  vs local-BN {el:.4f}  vs rerun {ea:.4f}",
              flush=True)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    mp.spawn(worker, args=(2, free_port()), nprocs=2, join=True)
