"""World size > 1 through the NATIVE reducer, on the CPU (reference ``multigpu.py:89,262-263``).

``csrc/runtime/rccl_comm.cpp`` — the C++ communicator + bucket reducer that ``DistributedDataParallel``
drives on MI355X — is compiled for the host together with ``csrc/tests/fake_world.cpp``: HIP streams become
FIFO worker threads, events become generation markers, and RCCL becomes an N-rank world of threads that
really reduces, scatters and gathers host buffers.  N ranks run as N Python threads (ctypes releases the
GIL), each with its own compute stream, communicator and reducer, exactly as N processes would.

What this pins, with the bucket layouts ``ddpx.parallel.ddp`` builds for the toy MLP (3072-4096-4096-10,
the headline model) and for a small MLP with row-chunked buckets, at N = 2 / 4 / 8:

* replicated all-reduce (the default DDP path): every rank's gradient buffer equals the numpy average,
  bit for bit (integer-valued data, N a power of two: every sum and quotient is exact in fp32 and bf16);
* ZeRO-1: the in-place reduce-scatter lands rank r's reduced shard at ``ptr + r*shard``, the shard update
  writes the bf16 shadow there, and the in-place all-gather from ``gptr + r*shard`` leaves every rank with
  the complete shadow — including the shard updates issued on the communicator stream itself
  (``comm_side_optimizer``);
* event ordering: each gradient "kernel" sleeps before writing; a collective that did not wait for its
  bucket's ready event would reduce stale bytes and fail the comparison.
"""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess
import threading
import types

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = [os.path.join(ROOT, "csrc", "runtime", "rccl_comm.cpp"), os.path.join(ROOT, "csrc", "tests", "fake_world.cpp")]

NCCL_F32, NCCL_BF16 = 7, 9


@pytest.fixture(scope="module")
def fake_lib(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None or not os.path.exists("/opt/rocm/include/rccl/rccl.h"):
        pytest.skip("host C++ toolchain / ROCm headers not available")
    out = str(tmp_path_factory.mktemp("fakeworld") / "libddpx_rt_fake.so")
    # -Bsymbolic: the runtime's HIP / RCCL calls bind to the fakes in this library even when the real
    # libamdhip64 / librccl are already loaded into the process by torch
    subprocess.run([cxx, "-std=c++17", "-O2", "-shared", "-fPIC", "-Wl,-Bsymbolic", "-Wno-unused-result",
                    "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", *SRC, "-o", out, "-lpthread"],
                   check=True, capture_output=True, text=True)
    lib = ctypes.CDLL(out, mode=os.RTLD_LOCAL)
    from ddpx.runtime import native
    native._declare_rt(lib)
    P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    native._sig(lib, "fake_stream_create", P)
    native._sig(lib, "fake_stream_destroy", None, P)
    native._sig(lib, "fake_stream_sync", None, P)
    native._sig(lib, "fake_launch_copy", None, P, P, P, S, I)
    native._sig(lib, "fake_launch_convert", None, P, P, I, P, I, S, I)
    native._sig(lib, "fake_violations", I)
    native._sig(lib, "fake_reset_violations", None)
    native._sig(lib, "fake_set_timeout_ms", None, I)
    native._sig(lib, "fake_last_violation", I, ctypes.c_char_p, I)
    lib.fake_set_timeout_ms(20000)
    return lib


class _LayoutComm:
    """Just enough of ddpx.parallel.comm.Comm for DistributedDataParallel to compute its bucket layout."""

    native = False
    supports_avg = True

    def __init__(self, rank, world):
        self.rank, self.world_size = rank, world

    def broadcast_(self, t, src=0, stream=None):
        pass

    def all_gather_object(self, obj):
        return [obj] * self.world_size

    def check(self):
        pass


def _layout(world, hidden, shard, chunk_mb=None, bucket_cap_mb=25.0, first_bucket_mb=1.0, grad_dtype=torch.float32):
    """The DDP object (CPU, layout only) for the native toy MLP at ``world`` ranks: flat store with a bf16
    shadow and shadow-only weights, exactly as ``prepare_model`` builds it on the GPU."""
    from ddpx.models import MLP
    from ddpx.parallel.ddp import DistributedDataParallel
    from ddpx.runtime.flat_params import FlatParams
    torch.manual_seed(0)
    model = MLP(hidden=hidden, layers=3)
    f = FlatParams(model, grad_dtype=grad_dtype, shadow_dtype=torch.bfloat16,
                   native_params=list(model.parameters()))
    f.shadow_only = {id(m.weight) for m in model.linears()}
    return DistributedDataParallel(model, comm=_LayoutComm(0, world), verify=False, shard_optimizer=shard,
                                   chunk_mb=chunk_mb, bucket_cap_mb=bucket_cap_mb, first_bucket_mb=first_bucket_mb)


def _bf16_bits(x32: np.ndarray) -> np.ndarray:
    return torch.from_numpy(np.ascontiguousarray(x32, dtype=np.float32)).to(torch.bfloat16).view(torch.int16).numpy()


def _run_world(lib, ddp, world, iters=2, comm_side=False, overlap=False, delay_us=8000):
    """Run ``iters`` backward passes + (ZeRO-1) shard updates on ``world`` rank threads through the native
    reducer; returns per-rank (grad, shadow) numpy copies of the last iteration and the expected average."""
    import ddpx.parallel.ddp as ddp_mod
    from ddpx.runtime import native

    f = ddp.flat
    total = f.total
    gdt = np.float32 if f.grad.dtype == torch.float32 else np.uint16
    esz = 4 if gdt is np.float32 else 2
    nccl_gdt = NCCL_F32 if gdt is np.float32 else NCCL_BF16
    ranges, modes, expected_marks = ddp.bucket_ranges, ddp.bucket_modes, ddp.bucket_expected
    # per-parameter production units in grad-ready order: (flat start, flat end, bucket)
    units = []
    for i in range(len(f.params)):
        o, n = f.offsets[i], f.numels[i]
        if i in ddp.chunk_bucket:
            cols = n // f.params[i].shape[0]
            for c, (r0, r1) in enumerate(f.chunk_rows[i]):
                units.append((o + r0 * cols, o + r1 * cols, ddp.chunk_bucket[i][c]))
        else:
            units.append((o, o + n, ddp.bucket_of[i]))
    for b, e in enumerate(expected_marks):
        assert sum(1 for u in units if u[2] == b) == e, "layout: marks per bucket"

    base = (np.arange(total, dtype=np.int64) % 61).astype(np.float32) - 30.0
    mask = np.zeros(total, dtype=bool)
    for s, e, _ in units:
        mask[s:e] = True

    def src_for(r, it):
        v = base + np.float32(((r * 13 + it * 5) % 17) - 8)
        return np.where(mask, v, np.float32(0)).astype(np.float32)

    srcs = {(r, it): src_for(r, it) for r in range(world) for it in range(iters)}
    if gdt is np.uint16:
        srcs = {k: _bf16_bits(v).view(np.uint16) for k, v in srcs.items()}
    expected = np.mean(np.stack([src_for(r, iters - 1) for r in range(world)]).astype(np.float64), axis=0)
    expected = expected.astype(np.float32)

    grads = [np.zeros(total, dtype=gdt) for _ in range(world)]
    shadows = [np.zeros(total, dtype=np.uint16) for _ in range(world)]
    errors = []
    tls = threading.local()
    shim = types.SimpleNamespace(ctypes=ctypes, check=native.check, runtime=lambda: lib,
                                 stream_handle=lambda s=None: s if s is not None else tls.stream)
    uid = (ctypes.c_char * 128)()
    assert lib.ddpx_comm_unique_id(uid, 128) == 0
    barrier = threading.Barrier(world)

    def rank_main(r):
        try:
            err = ctypes.c_int(0)
            h = lib.ddpx_comm_create(bytes(uid), world, r, 0, 1, 0.0, ctypes.byref(err))
            assert h, f"comm create failed {err.value}"
            comm_stream = lib.ddpx_comm_stream(h)
            tls.stream = lib.fake_stream_create()
            red = ddp_mod._NativeReducer.__new__(ddp_mod._NativeReducer)
            red.comm, red.ranges, red.modes, red.rt, red._gkeep = types.SimpleNamespace(handle=h), ranges, modes, lib, {}
            red.h = lib.ddpx_reducer_create(h, len(ranges), 4)  # ncclAvg
            gbuf = torch.from_numpy(grads[r])
            g_t = gbuf if gdt is np.float32 else gbuf.view(torch.bfloat16)
            red.setup(g_t, expected_marks)
            sh_t = torch.from_numpy(shadows[r]).view(torch.bfloat16)
            for b, (s, e) in enumerate(ranges):
                if modes[b] == 1:
                    red.set_gather(b, sh_t[s:e])
            gptr, sptr = grads[r].ctypes.data, shadows[r].ctypes.data
            poison = np.where(mask, np.float32(1e6), np.float32(0)).astype(np.float32)
            if gdt is np.uint16:
                poison = _bf16_bits(poison).view(np.uint16)
            for it in range(iters):
                # the previous iteration is complete on this rank (stream synced): poison what backward will
                # overwrite, so a collective that reads before its producer finished sees 1e6, not old data.
                # Host work that holds the GIL happens before the barrier: the issue loop below must not
                # stall behind another rank's numpy copies, or the producers could land before the marks.
                np.copyto(grads[r], poison)
                shadows[r].fill(0x4974)  # bf16 1e6: a gather that runs ahead of the shard update shows it
                barrier.wait()
                red.prepare()
                src = srcs[(r, it)]
                for s, e, b in units:  # backward: gradients in grad-ready order, each announced as produced
                    lib.fake_launch_copy(tls.stream, gptr + s * esz, src.ctypes.data + s * esz, (e - s) * esz,
                                         delay_us * (1 + (r + s) % 3))
                    red.mark_ready(b, 1)
                if overlap or any(modes):
                    red.finalize(join=False)  # overlap: the optimizer waits per bucket
                else:
                    assert red.finalize(join=True) == 0
                for b, (s, e) in enumerate(ranges):
                    upd_stream = comm_stream if (comm_side and modes[b] == 1) else tls.stream
                    red.wait_bucket(b, upd_stream)
                    if modes[b] == 1:  # ZeRO-1 shard update: reduced grad shard -> shadow shard, then all-gather
                        c = (e - s) // world
                        lo = s + r * c
                        lib.fake_launch_convert(upd_stream, sptr + lo * 2, NCCL_BF16, gptr + lo * esz, nccl_gdt, c,
                                                4 * delay_us)
                        rc = lib.ddpx_reducer_gather(red.h, b, upd_stream)
                        assert rc == 0, f"gather rc {rc}"
                for b in range(len(ranges)):
                    if modes[b] == 1:
                        red.wait_gather(b, tls.stream)
                lib.fake_stream_sync(tls.stream)
            red.close()
            assert lib.ddpx_comm_destroy(h, 0) == 0
            lib.fake_stream_destroy(tls.stream)
        except Exception as ex:  # noqa: BLE001 - reported by the main thread
            errors.append((r, repr(ex)))
            barrier.abort()

    old = ddp_mod.native
    ddp_mod.native = shim
    lib.fake_reset_violations()
    try:
        ts = [threading.Thread(target=rank_main, args=(r,), daemon=True) for r in range(world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=240)
        assert not any(t.is_alive() for t in ts), "a rank thread hung"
    finally:
        ddp_mod.native = old
    msg = ctypes.create_string_buffer(512)
    lib.fake_last_violation(msg, 512)
    assert lib.fake_violations() == 0, msg.value.decode()
    assert not errors, errors
    return grads, shadows, expected, ranges, modes


def _as_f32(g):
    if g.dtype == np.float32:
        return g
    return (g.astype(np.uint32) << 16).view(np.float32)


def _check(world, grads, shadows, expected, ranges, modes):
    exp_bf16 = _bf16_bits(expected).view(np.uint16)
    for r in range(world):
        g = _as_f32(grads[r])
        for b, (s, e) in enumerate(ranges):
            if modes[b] == 0:
                np.testing.assert_array_equal(g[s:e], expected[s:e], err_msg=f"rank {r} bucket {b} all-reduce")
            else:
                c = (e - s) // world
                lo, hi = s + r * c, s + (r + 1) * c
                np.testing.assert_array_equal(g[lo:hi], expected[lo:hi],
                                              err_msg=f"rank {r} bucket {b}: reduce-scatter shard at ptr+rank*shard")
                np.testing.assert_array_equal(shadows[r][s:e], exp_bf16[s:e],
                                              err_msg=f"rank {r} bucket {b}: all-gathered shadow")


@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_reducer_allreduce_toy_mlp(fake_lib, world):
    ddp = _layout(world, hidden=4096, shard=False)
    assert not any(ddp.bucket_modes)
    out = _run_world(fake_lib, ddp, world, iters=2)
    _check(world, *out)


@pytest.mark.parametrize("world", [2, 4, 8])
def test_native_reducer_zero1_toy_mlp(fake_lib, world):
    ddp = _layout(world, hidden=4096, shard=True)
    assert ddp.gather_what == "shadow" and 1 in ddp.bucket_modes and 0 in ddp.bucket_modes
    out = _run_world(fake_lib, ddp, world, iters=2)
    _check(world, *out)


@pytest.mark.parametrize("world", [2, 8])
def test_native_reducer_zero1_comm_side_chunked(fake_lib, world):
    """ZeRO-1 with row-chunk buckets and the shard updates issued on the RCCL stream itself."""
    ddp = _layout(world, hidden=512, shard=True, chunk_mb=0.25, bucket_cap_mb=0.5, first_bucket_mb=0.0625)
    assert any(c is not None for c in ddp.bucket_chunk), "expected row-chunk buckets"
    out = _run_world(fake_lib, ddp, world, iters=3, comm_side=True)
    _check(world, *out)


@pytest.mark.parametrize("world", [4])
def test_native_reducer_allreduce_chunked_overlap_bf16(fake_lib, world):
    """Replicated buckets, chunked, bf16 gradients, per-bucket waits (overlap optimizer mode)."""
    ddp = _layout(world, hidden=512, shard=False, chunk_mb=0.25, bucket_cap_mb=0.5, first_bucket_mb=0.0625,
                  grad_dtype=torch.bfloat16)
    out = _run_world(fake_lib, ddp, world, iters=3, overlap=True)
    _check(world, *out)


def test_fake_world_detects_missing_stream_dependency(fake_lib):
    """The harness itself: an all-reduce issued WITHOUT waiting for the producing stream reduces stale data
    (so the reducer tests above would catch a dropped hipStreamWaitEvent)."""
    world, n = 2, 4096
    uid = (ctypes.c_char * 128)()
    fake_lib.ddpx_comm_unique_id(uid, 128)
    bufs = [np.zeros(n, dtype=np.float32) for _ in range(world)]
    src = [np.full(n, 8.0 * (r + 1), dtype=np.float32) for r in range(world)]
    errors = []

    def rank_main(r):
        try:
            err = ctypes.c_int(0)
            h = fake_lib.ddpx_comm_create(bytes(uid), world, r, 0, 1, 0.0, ctypes.byref(err))
            s = fake_lib.fake_stream_create()
            fake_lib.fake_launch_copy(s, bufs[r].ctypes.data, src[r].ctypes.data, n * 4, 200000)
            # no event: the communicator stream runs ahead of the 200 ms producer
            assert fake_lib.ddpx_comm_allreduce(h, bufs[r].ctypes.data, bufs[r].ctypes.data, n, NCCL_F32, 0,
                                                fake_lib.ddpx_comm_stream(h)) == 0
            fake_lib.fake_stream_sync(fake_lib.ddpx_comm_stream(h))
            fake_lib.fake_stream_sync(s)
            fake_lib.ddpx_comm_destroy(h, 0)
            fake_lib.fake_stream_destroy(s)
        except Exception as ex:  # noqa: BLE001
            errors.append(repr(ex))

    ts = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not errors, errors
    # the all-reduce saw zeros (stale) and the late copies overwrote its result with each rank's own data
    assert not np.array_equal(bufs[0], bufs[1])
