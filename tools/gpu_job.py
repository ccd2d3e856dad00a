#!/usr/bin/env python3
"""Run a list of GPU steps on the gpurun box, each under its own time limit.

Usage: python tools/gpu_job.py STEPFILE   (one step per line: ``NAME|TIMEOUT_S|COMMAND``)

* stdout/stderr of each step go to gpurun_out/<NAME>.log;
* a step exiting 0 or 1 (test/bench failure) lets the job continue;
* a fault-like exit (signal, 124/137 timeout, 134 abort, 139 segv, anything
  >= 2 except listed soft codes) stops the job immediately: no further GPU step
  runs after a fault (gpurun rules);
* a summary is written to gpurun_out/job_summary.json.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

OUT = "gpurun_out"
SOFT = {0, 1, 5}


def main():
    steps = []
    with open(sys.argv[1]) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            name, tmo, cmd = line.split("|", 2)
            steps.append((name.strip(), int(tmo), cmd.strip()))
    os.makedirs(OUT, exist_ok=True)
    summary = []
    for name, tmo, cmd in steps:
        t0 = time.time()
        log = os.path.join(OUT, f"{name}.log")
        print(f"[gpu_job] {name}: {cmd}", flush=True)
        with open(log, "w") as lf:
            p = subprocess.run(["timeout", "-k", "10", str(tmo), "bash", "-c", cmd], stdout=lf,
                               stderr=subprocess.STDOUT)
        rc = p.returncode
        dt = time.time() - t0
        summary.append({"step": name, "rc": rc, "seconds": round(dt, 1)})
        print(f"[gpu_job] {name}: rc={rc} in {dt:.1f}s", flush=True)
        with open(os.path.join(OUT, "job_summary.json"), "w") as f:
            json.dump(summary, f, indent=1)
        if rc not in SOFT:
            print(f"[gpu_job] stopping after fault-like exit {rc} in {name}", flush=True)
            sys.exit(3)


if __name__ == "__main__":
    main()
