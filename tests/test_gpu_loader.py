"""GPU-resident loader: the device-cursor batch path equals the host-driven path, and is graph-capturable."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layout", ["flat_bf16", "nhwc8_bf16", "nchw_f32"])
def test_cursor_batch_matches_make_batch(gpu, layout):
    from ddpx.data.datasets import synthetic_cifar
    from ddpx.data.loader import DeviceLoader
    from ddpx.data.sampler import DistributedIndexSampler
    ds = synthetic_cifar(2048, seed=3)
    bs = 128
    loader = DeviceLoader(ds, bs, gpu, sampler=DistributedIndexSampler(len(ds), 1, 0, shuffle=True, seed=0),
                          train=True, layout=layout, seed=0)
    idx_all = loader._epoch_indices()
    nfull = idx_all.numel() // bs
    idx_dev = idx_all[:nfull * bs].contiguous()
    x0, y0 = loader.make_batch(idx_all[:bs], 0)
    sx, sy = torch.empty_like(x0), torch.empty_like(y0)
    for k in range(nfull + 2):  # wraps around the epoch
        loader.cursor_batch(idx_dev, nfull, sx, sy)
        b = k % nfull
        ex, ey = loader.make_batch(idx_all[b * bs:(b + 1) * bs], k)
        assert torch.equal(sx, ex), k
        assert torch.equal(sy, ey), k
    assert int(loader._cursor.item()) == nfull + 2
    # captured, with an external step counter advanced separately: every replay draws the next batch
    counter = torch.full((1,), nfull + 2, dtype=torch.int32, device=gpu)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            loader.cursor_batch(idx_dev, nfull, sx, sy, counter=counter)
            counter.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    for k in range(nfull + 2, nfull + 5):
        g.replay()
        b = k % nfull
        ex, ey = loader.make_batch(idx_all[b * bs:(b + 1) * bs], k)
        assert torch.equal(sx, ex) and torch.equal(sy, ey), k
