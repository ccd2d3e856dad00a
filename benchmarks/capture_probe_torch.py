"""torch.cuda.graph on ROCm: what a failed capture leaves behind (current stream, capture status, the next
H2D copy), and the same through ddpx.runtime.graphs.capture_step.  One case per process
(``python benchmarks/capture_probe_torch.py CASE``; no argument runs every case in child processes).
Backs profiles/r5_capture/NOTES.md."""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = ["torch_raise_after_fork", "torch_unjoined", "torch_invalidated",
         "ddpx_raise_after_fork", "ddpx_unjoined", "ddpx_invalidated"]


def run(case):
    import torch
    dev = torch.device("cuda", 0)
    x = torch.zeros(1 << 16, device=dev)
    side = torch.cuda.Stream(dev)
    y = torch.zeros(4, device=dev)
    default = torch.cuda.current_stream()
    torch.cuda.synchronize()

    def body(mode):
        x.add_(1)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            x.mul_(2)
        if mode == "raise_after_fork":
            raise RuntimeError("injected failure after the fork")
        if mode == "invalidated":
            # an unsafe call on the capturing thread: a synchronous copy on a non-captured stream
            other = torch.cuda.Stream(dev)
            with torch.cuda.stream(other):
                y.copy_(torch.ones(4), non_blocking=False)
        if mode != "unjoined":
            torch.cuda.current_stream().wait_stream(side)

    engine, mode = case.split("_", 1)
    g = torch.cuda.CUDAGraph()
    err = None
    try:
        if engine == "torch":
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                body(mode)
        else:
            from ddpx.runtime.graphs import capture_step, register_side_stream
            register_side_stream(side, "probe side stream")
            capture_step(g, lambda: body(mode))
    except Exception as e:  # noqa: BLE001
        err = f"{type(e).__name__}: {str(e).splitlines()[0][:160]}"
    cur = torch.cuda.current_stream()
    print(f"case={case}")
    print(f"  capture error        : {err}")
    print(f"  current stream reset : {cur == default}")
    print(f"  current capturing    : {torch.cuda.is_current_stream_capturing()}")
    try:
        from ddpx.runtime.graphs import stream_capture_status
        print(f"  side stream status   : {stream_capture_status(side)}")
        print(f"  current stream status: {stream_capture_status(cur)}")
    except Exception as e:  # noqa: BLE001
        print(f"  status query failed  : {e}")
    try:
        t = torch.arange(8, dtype=torch.float32).to(dev)  # H2D through memcpy_and_sync
        torch.cuda.synchronize()
        print(f"  H2D after            : ok {float(t.sum())}")
    except Exception as e:  # noqa: BLE001
        print(f"  H2D after            : FAILED {type(e).__name__}: {str(e).splitlines()[0][:120]}")


def main():
    if len(sys.argv) > 1:
        run(sys.argv[1])
        return
    for c in CASES:
        r = subprocess.run([sys.executable, __file__, c], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                           text=True, timeout=180)
        print(r.stdout.strip() or f"case={c}: no output (rc {r.returncode})", flush=True)
        if r.returncode:
            print(f"  (rc {r.returncode})", flush=True)


if __name__ == "__main__":
    main()
