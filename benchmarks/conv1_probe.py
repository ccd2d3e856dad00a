#!/usr/bin/env python3
"""Where VGG conv1 (64 -> 128 channels at 32x32, batch 512: M = 524288, N = 128, K = 576) loses time.

Times (median of 20 CUDA-event-bracketed launches, us) the native implicit-GEMM forward with and without the
BatchNorm-statistics epilogue for several tile configs, the same GEMM as a plain row-major product on the
ddpx pipe core and on hipBLASLt (torch.matmul), MIOpen's convolution, and the same set for conv1's data
gradient (M = 524288, N = 64, K = 1152).  One JSON line per measurement.

    python benchmarks/conv1_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


def ksweep():
    """Per-tile fixed cost vs per-K-step cost at the 32x32 geometry: the 256x128 forward tile over input channel
    counts C = 64..512 (K = 9 C, 9..72 K-steps per tile), Co = 128."""
    from ddpx.ops import conv as K
    dev = torch.device("cuda", 0)
    N, H, W, Co = 512, 32, 32, 128
    for C in (64, 128, 256, 512):
        x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
        w = torch.randn(Co, C, 3, 3, device=dev) * 0.05
        wf = torch.empty(Co * 9 * C, dtype=torch.bfloat16, device=dev)
        wd = torch.empty_like(wf)
        K.weight_prep(w, wf, wd)
        fl = 2.0 * N * H * W * Co * 9 * C
        for stats in (False, True):
            us = timed(lambda: K.conv_fwd(x, wf, Co, stats=stats, tile=8))
            print(json.dumps({"case": f"ksweep_C{C}_stats{int(stats)}", "ksteps": 9 * C // 64, "us": us,
                              "tflops": round(fl / us / 1e6, 1)}), flush=True)
        del x, w, wf, wd


def pmc_case(C):
    """Five launches of the 256x128 forward (statistics epilogue) at C input channels, 32x32, Co 128: the
    kernel a rocprofv3 --pmc pass reads."""
    from ddpx.ops import conv as K
    dev = torch.device("cuda", 0)
    N, H, W, Co = 512, 32, 32, 128
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(Co, C, 3, 3, device=dev) * 0.05
    wf = torch.empty(Co * 9 * C, dtype=torch.bfloat16, device=dev)
    wd = torch.empty_like(wf)
    K.weight_prep(w, wf, wd)
    for _ in range(5):
        K.conv_fwd(x, wf, Co, stats=True, tile=8)
    torch.cuda.synchronize()


def main():
    if "--ksweep" in sys.argv:
        return ksweep()
    if "--pmc" in sys.argv:
        return pmc_case(int(sys.argv[sys.argv.index("--pmc") + 1]))
    from ddpx.ops import conv as K
    from ddpx.ops import gemm as G
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    N, H, W, C, Co = 512, 32, 32, 64, 128
    P = N * H * W
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    w = torch.randn(Co, C, 3, 3, device=dev) * 0.05
    wf = torch.empty(Co * 9 * C, dtype=torch.bfloat16, device=dev)
    wd = torch.empty_like(wf)
    K.weight_prep(w, wf, wd)

    def out(name, us, flop):
        print(json.dumps({"case": name, "us": us, "tflops": round(flop / us / 1e6, 1)}), flush=True)

    fl = 2.0 * P * Co * 9 * C
    for tile in (-1, 0, 4, 5, 6, 8, 13, 14, 15):
        out(f"fwd_stats_t{tile}", timed(lambda: K.conv_fwd(x, wf, Co, stats=True, tile=tile)), fl)
        out(f"fwd_nostats_t{tile}", timed(lambda: K.conv_fwd(x, wf, Co, stats=False, tile=tile)), fl)
    a = torch.randn(P, 9 * C, device=dev).to(torch.bfloat16)
    b = torch.randn(Co, 9 * C, device=dev).to(torch.bfloat16)
    for tile in (-1, 0, 8, 13):
        out(f"plain_gemm_t{tile}", timed(lambda: G.matmul(a, b, out_dtype=torch.bfloat16, tile=tile)), fl)
    out("hipblaslt_gemm", timed(lambda: a @ b.t()), fl)
    xc = x.permute(0, 3, 1, 2)  # NCHW view of NHWC storage: channels_last
    wc = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    out("miopen_fwd", timed(lambda: torch.nn.functional.conv2d(xc, wc, padding=1)), fl)

    dy = torch.randn(P, Co, device=dev).to(torch.bfloat16)
    for tile in (-1, 0, 2, 6, 7, 8, 11):
        out(f"dgrad_t{tile}", timed(lambda: K.conv_dgrad(dy, wd, N, H, W, C, Co, tile=tile)), fl)
    a2 = torch.randn(P, 9 * Co, device=dev).to(torch.bfloat16)
    b2 = torch.randn(C, 9 * Co, device=dev).to(torch.bfloat16)
    for tile in (-1, 2, 6, 11):
        out(f"plain_dgrad_gemm_t{tile}", timed(lambda: G.matmul(a2, b2, out_dtype=torch.bfloat16, tile=tile)), fl)
    out("hipblaslt_dgrad_gemm", timed(lambda: a2 @ b2.t()), fl)


if __name__ == "__main__":
    main()
