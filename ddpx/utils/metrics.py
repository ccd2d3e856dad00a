"""Opt-in JSON-lines metrics stream (the reference only prints)."""
from __future__ import annotations

import json
import time


class MetricsWriter:
    def __init__(self, path: str, rank: int = 0, all_ranks: bool = False):
        self.rank = rank
        self.f = open(path if not all_ranks else f"{path}.rank{rank}", "a") if (rank == 0 or all_ranks) else None

    def log(self, **kw):
        if self.f is None:
            return
        kw.setdefault("time", time.time())
        kw.setdefault("rank", self.rank)
        self.f.write(json.dumps(kw) + "\n")
        self.f.flush()

    def close(self):
        if self.f is not None:
            self.f.close()
            self.f = None
