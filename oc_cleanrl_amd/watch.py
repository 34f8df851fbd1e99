"""Fail fast when a rank of a multi-GPU run stops making progress.

SURVEY §5 asks the data-parallel path (ppo_atari_multigpu.py:174-175, 360-377) to fail fast on
RCCL errors. A collective whose peer never arrives blocks the waiting ranks inside a HIP call (or
a graph replay) that Python cannot interrupt, so a run would otherwise hang until an outer limit
kills it, leaving no record of where it stopped. RankWatch bounds that:

- every rank names its phase (`phase("warmup 2")`) and, optionally, beats within it;
- each phase change is written to `<dir>/rank<r>.json` (atomic replace), so any rank -- and a
  parent launcher -- can read where every rank of the node is;
- a daemon thread fires when the current phase has gone `stall_s` without progress or the whole
  run passes `deadline_s`: it builds one record naming this rank, its phase, every rank's last
  phase and the ranks that are behind (fewest phase changes), hands it to `on_fire` (bench.py
  prints it as its JSON line) and ends the process with `exit_code` (os._exit: the main thread
  may be blocked in a device call; no exec, nothing restarts);
- a rank that fires marks its status file failed and, unless it is rank 0, lingers `linger_s`
  before exiting: rank 0's thread sees the mark and fires first, so the run's one line (rank 0's)
  is written before the launcher tears the other ranks down.
"""
from __future__ import annotations

import json
import os
import threading
import time
from pathlib import Path


def run_token() -> str:
    """Names this run in the status records: OCPPO_RUN_ID when a launcher sets one, else the
    parent's pid -- the ranks of one node are the children of one launcher process (torchrun's
    agent, mp.spawn's parent), and a later run on the same status directory has another."""
    return os.getenv("OCPPO_RUN_ID") or f"ppid{os.getppid()}"


def read_status(dirname, since: float = 0.0, run: str | None = None) -> dict:
    """{rank: record} of every rank that wrote a status file in `dirname` at wall time >= since
    and, given `run`, carries that run token (other files are a previous run's: a directory keyed
    by the master port is shared by every run on that port)."""
    out = {}
    if not dirname:
        return out
    for p in sorted(Path(dirname).glob("rank*.json")):
        try:
            rec = json.loads(p.read_text())
            if rec.get("t", 0.0) >= since and (run is None or rec.get("run") == run):
                out[int(rec["rank"])] = rec
        except (OSError, ValueError, KeyError):
            continue
    return out


def behind(ranks: dict) -> list:
    """The ranks with the fewest phase changes: the ones the others are waiting for."""
    if not ranks:
        return []
    low = min(r["n"] for r in ranks.values())
    return sorted(k for k, r in ranks.items() if r["n"] == low)


class RankWatch:
    def __init__(self, rank: int, world: int, status_dir=None, stall_s: float = 120.0,
                 deadline_s: float | None = None, on_fire=None, exit_code: int = 3,
                 poll_s: float = 0.25, linger_s: float = 3.0):
        self.rank, self.world = rank, world
        self.dir = Path(status_dir) if status_dir else None
        if self.dir is not None:
            self.dir.mkdir(parents=True, exist_ok=True)
        self.stall_s, self.deadline_s = stall_s, deadline_s
        self.on_fire, self.exit_code, self.poll_s = on_fire, exit_code, poll_s
        self.linger_s = linger_s
        self.t0 = self.last = time.monotonic()
        self.since = time.time() - 600.0  # peers started within the launcher's rendezvous window
        self.run = run_token()
        self.name, self.n, self.bound = "start", 0, stall_s
        self.failed = None
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._write()
        self._thread = threading.Thread(target=self._loop, name=f"rankwatch{rank}", daemon=True)
        self._thread.start()

    def phase(self, name: str, stall_s: float | None = None):
        """Enter phase `name`; it may take up to stall_s (default: the watch's) without a beat."""
        with self._lock:
            self.name, self.n = name, self.n + 1
            self.bound = self.stall_s if stall_s is None else stall_s
            self.last = time.monotonic()
        self._write()

    def beat(self):
        with self._lock:
            self.last = time.monotonic()

    def stop(self):
        self._stop.set()
        self._thread.join(timeout=2 * self.poll_s + 1)
        with self._lock:
            self.name = "done"
        self._write()

    def _write(self):
        if self.dir is None:
            return
        rec = {"rank": self.rank, "phase": self.name, "n": self.n, "pid": os.getpid(),
               "t": round(time.time(), 3), "run": self.run}
        if self.failed:
            rec["failed"] = self.failed
        tmp = self.dir / f".rank{self.rank}.{os.getpid()}.tmp"
        try:
            tmp.write_text(json.dumps(rec))
            os.replace(tmp, self.dir / f"rank{self.rank}.json")
        except OSError:
            pass

    def record(self, reason: str) -> dict:
        now = time.monotonic()
        ranks = read_status(self.dir, self.since, self.run)
        return {"error": reason, "rank": self.rank, "world": self.world, "phase": self.name,
                "phase_s": round(now - self.last, 1), "elapsed_s": round(now - self.t0, 1),
                "ranks": {str(k): v["phase"] for k, v in sorted(ranks.items())},
                "failed": {str(k): v["failed"] for k, v in sorted(ranks.items())
                           if v.get("failed")},
                "behind": behind(ranks)}

    def _loop(self):
        while not self._stop.wait(self.poll_s):
            now = time.monotonic()
            with self._lock:
                stalled = now - self.last > self.bound
            late = self.deadline_s is not None and now - self.t0 > self.deadline_s
            if stalled or late:
                self.fire("stall" if stalled else "deadline")
            if self.rank == 0 and self.world > 1:
                peers = [k for k, v in read_status(self.dir, self.since, self.run).items()
                         if k != 0 and v.get("failed")]
                if peers:
                    self.fire(f"rank {peers[0]} failed")

    def fire(self, reason: str, exit_code: int | None = None):
        """End this rank: mark it failed, hand the record to on_fire, exit (never returns)."""
        if exit_code is not None:
            self.exit_code = exit_code
        self.failed = reason
        self._write()
        rec = self.record(reason)
        try:
            if self.on_fire is not None:
                self.on_fire(rec)
            if self.rank != 0 and self.world > 1:
                time.sleep(self.linger_s)  # rank 0 writes the run's line first
        finally:
            os._exit(self.exit_code)
