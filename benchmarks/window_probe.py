#!/usr/bin/env python3
"""What a short timed window pays besides its steps: the toy-MLP bench engine (bench.make_runner, graphs of
several sizes) timed over the same K-step window with different replay schedules, interleaved in one process.

    DDPX_GRAPH_SIZES=1,2,4,5,10,15,18,20 python benchmarks/window_probe.py [--steps 20] [--rounds 6]

Per schedule: host wall time of the window (sync, replays, sync) and, from events around each replay, the GPU
time of every replay — the gap between the window's start and the first replay's GPU start is the exposed
launch cost.  Every window runs real training steps (weights keep changing)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    os.environ.setdefault("DDPX_GRAPH_SIZES", "1,2,4,5,10,15,18,20")
    import torch
    import bench
    args = bench.parse(["--gpus", "1", "--steps", str(a.steps), "--warmup", "5", "--stock_ref", "0"])
    bench.resolve_defaults(args, 1)
    dev = torch.device("cuda", 0)
    loader = bench.make_data(args, dev, 0, 1)
    idx_all = loader._epoch_indices()
    full = [i for i in range(len(loader)) if (i + 1) * args.batch_size <= idx_all.numel()]
    eng = bench.make_runner(args, dev, 1, loader, idx_all, full, None)
    eng.run(0, 3)  # eager warm-up + capture of every size
    g = eng.runner.graphs
    for m in sorted(g):  # one replay of each graph (first-launch effects out of the way)
        g[m]()
    torch.cuda.synchronize()
    K = a.steps
    scheds = {"one_20": [20], "ramp_1_4_15": [1, 4, 15], "ones": [1] * K, "2_18": [2, 18], "5_15": [5, 15],
              "10_10": [10, 10], "1_2_4_5_...": [1, 2, 4, 5, 4, 4]}
    scheds = {k: v for k, v in scheds.items() if sum(v) == K and all(m in g for m in v)}
    res = {k: {"host_ms": [], "first_gap_us": [], "gpu_ms": []} for k in scheds}
    for _ in range(a.rounds):
        for name, sched in scheds.items():
            torch.cuda.synchronize()
            e0 = torch.cuda.Event(enable_timing=True)
            evs = []
            t0 = time.perf_counter()
            e0.record()
            for m in sched:
                s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s0.record()
                g[m]()
                s1.record()
                evs.append((s0, s1))
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            r = res[name]
            r["host_ms"].append((t1 - t0) * 1e3)
            r["first_gap_us"].append(e0.elapsed_time(evs[0][0]) * 1e3)
            r["gpu_ms"].append(e0.elapsed_time(evs[-1][1]))
    # first vs second replay of freshly captured graphs (GPU time between events around each replay)
    fresh = {}
    eng.runner.graphs = eng.runner.make_graphs()
    for m in sorted(eng.runner.graphs, reverse=True):
        gm = eng.runner.graphs[m]
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            s0.record()
            gm()
            s1.record()
            t_host = (time.perf_counter() - t0) * 1e3
            torch.cuda.synchronize()
            ts.append({"gpu_ms": round(s0.elapsed_time(s1), 4), "launch_host_ms": round(t_host, 4)})
        fresh[m] = ts
        print(f"fresh graph of {m} steps, replays 1..3: {ts}", flush=True)
    out = {"fresh_graph_replays": fresh}
    for name, r in res.items():
        med = {k: sorted(v)[len(v) // 2] for k, v in r.items()}
        out[name] = {k: round(v, 4) for k, v in med.items()}
        out[name]["ms_per_step_host"] = round(med["host_ms"] / K, 4)
        print(name, json.dumps(out[name]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
