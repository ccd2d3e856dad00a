"""Several ranks sharing ONE MI355X: the multi-rank DDP / ZeRO-1 paths with the native kernels.

RCCL refuses two ranks on one device, so the collectives go through ``HostStagedComm`` (gloo on
host copies).  Everything else is the production path: native MFMA kernels, flat store relayout
for shards, per-bucket optimizer overlap, shard-local SGD, in-place bf16 shadow all-gather,
``consolidate()``.  Each rank checks its result against a single-process ddpx model trained on the
global batch (the mean of the per-rank mean losses is the global mean loss).
"""
import os
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from tests._dist_util import free_port, init_gloo

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mlp_worker(rank, ws, port, overlap, shard, grad_dtype, steps, chunk_mb, defer, errq):
    import torch.distributed as dist
    try:
        import ddpx
        from ddpx.models import MLP
        from ddpx.optim.sgd import SGD
        from ddpx.parallel.comm import HostStagedComm
        from ddpx.parallel.ddp import DistributedDataParallel
        init_gloo(rank, ws, port)
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        torch.manual_seed(7 + rank)  # different init per rank: DDP must broadcast rank 0's weights
        ours = MLP(hidden=512)
        torch.manual_seed(7)
        ref = MLP(hidden=512)  # rank 0's init
        gd = torch.bfloat16 if grad_dtype == "bf16" else torch.float32
        ddpx.prepare_model(ours, dev, grad_dtype=gd)
        ddpx.prepare_model(ref, dev)
        d = DistributedDataParallel(ours, comm=HostStagedComm(), bucket_cap_mb=1.0, first_bucket_mb=0.25,
                                    overlap_optimizer=overlap, shard_optimizer=shard, chunk_mb=chunk_mb,
                                    defer_gather=defer)
        if shard:
            assert d.sharded and d.gather_what == "shadow"
        if chunk_mb:
            assert len(d.chunk_bucket) == 2 and all(len(v) >= 2 for v in d.chunk_bucket.values())
        assert d.defer_gather == bool(defer and shard)
        o = SGD(ours.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
        if overlap or shard:
            d.attach_optimizer(o)
        o_ref = SGD(ref.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
        for p, q in zip(ours.parameters(), ref.parameters()):
            assert torch.equal(p, q), "init broadcast mismatch"
        w0 = [p.detach().clone() for p in ref.parameters()]
        B = 128
        for s in range(steps):
            g = torch.Generator(device="cpu").manual_seed(1000 + s)
            xg = torch.rand(ws * B, 3072, generator=g).to(dev).to(torch.bfloat16)
            tg = torch.randint(0, 10, (ws * B,), generator=g).to(dev)
            o.zero_grad()
            loss, _ = d.forward_loss(xg[rank * B:(rank + 1) * B], tg[rank * B:(rank + 1) * B])
            loss.backward()
            o.step()
            o_ref.zero_grad()
            lr_, _ = ref.forward_loss(xg, tg)
            lr_.backward()
            o_ref.step()
        d.consolidate()
        torch.cuda.synchronize()
        for (n, p), q, p0 in zip(ours.named_parameters(), ref.parameters(), w0):
            du, dr = (p - p0).double(), (q - p0).double()
            rel = ((du - dr).norm() / dr.norm().clamp_min(1e-12)).item()
            # the reference runs the global batch in one process: its bf16 activations / dlogits round
            # differently from the per-rank halves, and the small head weight (10 x 512) amplifies that
            # in relative terms (one run in ~6 measured 1.19e-2 on fc2.weight with fp32 gradients)
            tol = 3e-2 if grad_dtype == "bf16" else 2e-2
            assert rel < tol, (rank, n, rel)
        # momentum (optimizer state) complete on every rank after consolidate()
        so, sr = o.state_dict()["state"], o_ref.state_dict()["state"]
        for i in sr:
            a, b = so[i]["momentum_buffer"].double(), sr[i]["momentum_buffer"].double()
            assert ((a - b).norm() / b.norm().clamp_min(1e-12)).item() < 5e-2, i
        flat = ours.fc0.weight._ddpx_flat.master.detach().cpu()
        lst = [torch.empty_like(flat) for _ in range(ws)]
        dist.all_gather(lst, flat)
        for other in lst:
            assert torch.equal(other, lst[0]), "replicas diverged"
        d.close()
        dist.destroy_process_group()
    except BaseException as e:  # report through the queue: spawn's own traceback loses assertion text
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")
        raise


def _run(fn, ws, *args):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    try:
        mp.spawn(fn, args=(ws, free_port()) + args + (q,), nprocs=ws, join=True)
    except Exception:
        msgs = []
        while not q.empty():
            msgs.append(q.get())
        raise AssertionError("\n".join(msgs) or "worker failed")


@pytest.mark.parametrize("overlap,shard,grad_dtype,chunk_mb,defer", [
    (False, False, "fp32", None, False),
    (True, False, "bf16", None, False),
    (True, True, "bf16", None, False),
    (False, True, "fp32", None, False),
    (True, False, "bf16", 0.125, False),   # row-chunk buckets, all-reduce
    (True, True, "bf16", 0.125, True),     # chunks + ZeRO-1 + deferred, per-chunk-waited all-gathers
    (False, True, "fp32", 0.25, True),
])
def test_mlp_two_ranks_one_gpu(gpu, overlap, shard, grad_dtype, chunk_mb, defer):
    _run(_mlp_worker, 2, overlap, shard, grad_dtype, 3, chunk_mb, defer)


def test_bench_two_ranks_one_gpu(gpu, tmp_path):
    """The bench.py multi-GPU code path (ZeRO-1, bf16 grads, overlap) at world size 2 on one device."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    out = tmp_path / "b.jsonl"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "4", "--warmup", "2", "--comm", "host", "--hidden", "1024",
           "--chunk_mb", "0.5", "--json_out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    import json
    rec = json.loads(out.read_text().strip().splitlines()[-1])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["sharded_optimizer"] is True and rec["config"]["replicas_consistent"] is True
    assert rec["config"]["defer_gather"] is True and rec["config"]["chunk_mb"] == 0.5
    assert rec["value"] > 0
