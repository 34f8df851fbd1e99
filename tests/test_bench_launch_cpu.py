"""bench.py --gpus N > 1 outside a torch.distributed launch starts its N ranks as a child
`torch.distributed.run` (ppo_atari_multigpu.py:162-175 is launched the same way: one process per
GPU, RANK / LOCAL_RANK / WORLD_SIZE from the env) and forwards every argument verbatim; the ranks'
parameter checksums are gathered and compared (the replica invariant of
ppo_atari_multigpu.py:360-377). CPU only: the child here is a probe script, not the trainer."""
import json
import os
import socket
import sys
import time
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oc_cleanrl_amd.trainer import PPOTrainer

PROBE = """
import json, os, sys
print("[Gloo] Rank", os.environ["RANK"], "chatter", flush=True)
if os.environ["RANK"] == "0":
    print(json.dumps({"argv": sys.argv[1:], "world": os.environ["WORLD_SIZE"],
                      "local_rank": os.environ["LOCAL_RANK"],
                      "ipc": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}), flush=True)
sys.exit(int(os.environ.get("PROBE_RC", "0")))
"""


def test_needs_launch():
    assert bench.needs_launch(2, {})
    assert bench.needs_launch(8, {"RANK": "0"})
    assert not bench.needs_launch(1, {})
    assert not bench.needs_launch(2, {"WORLD_SIZE": "2"})


def test_launcher_cmd_forwards_arguments():
    argv = ["--gpus", "2", "--steps", "7", "--backend", "gloo", "--device-index", "0",
            "--set", "x6_gemm=0"]
    cmd = bench.launcher_cmd(argv, 2, 29511)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29511"
    script = cmd.index(str(bench.ROOT / "bench.py"))
    assert cmd[script + 1:] == argv


def test_launch_runs_ranks_and_forwards_rank0_line(tmp_path, capfd):
    probe = tmp_path / "probe.py"
    probe.write_text(PROBE)
    argv = ["--gpus", "2", "--steps", "3", "--warmup", "1"]
    rc = bench.launch(argv, 2, script=probe)
    assert rc == 0
    cap = capfd.readouterr()
    lines = cap.out.splitlines()
    assert len(lines) == 1  # rank 0's line only; the ranks' other stdout went to stderr
    out = [json.loads(lines[0])]
    assert cap.err.count("chatter") == 2
    assert out[0]["argv"] == argv and out[0]["world"] == "2" and out[0]["local_rank"] == "0"
    assert out[0]["ipc"] == "0"


def test_launch_returns_child_exit_code(tmp_path, monkeypatch):
    probe = tmp_path / "probe.py"
    probe.write_text(PROBE)
    monkeypatch.setenv("PROBE_RC", "3")
    assert bench.launch(["--gpus", "2"], 2, script=probe) != 0


def _fake_trainer(seed):
    g = torch.Generator().manual_seed(seed)
    return types.SimpleNamespace(params=[torch.randn(5, 3, generator=g), torch.randn(7, generator=g)])


def test_param_checksum_is_exact_and_order_sensitive():
    a = _fake_trainer(0)
    s = PPOTrainer.param_checksum(a)
    assert s == PPOTrainer.param_checksum(_fake_trainer(0))
    b = _fake_trainer(0)
    b.params[1][3] = torch.nextafter(b.params[1][3], torch.tensor(10.0))  # one ulp
    assert PPOTrainer.param_checksum(b) != s
    c = _fake_trainer(0)
    c.params[0] = c.params[0].flip(0)
    assert PPOTrainer.param_checksum(c) != s


def _replica_worker(rank, world, port, diverge, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = _fake_trainer(0)
    tr.param_checksum = lambda: PPOTrainer.param_checksum(tr)
    if diverge and rank == 1:
        tr.params[0][0, 0] += 1.0
    try:
        out[rank] = bench.replica_check(tr, world, torch.device("cpu"))
    except SystemExit as e:
        out[rank] = str(e)
    dist.destroy_process_group()


@pytest.mark.parametrize("diverge", [False, True])
def test_replica_check_gloo_world2(diverge):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = mp.Manager().dict()
    mp.spawn(_replica_worker, args=(2, port, diverge, out), nprocs=2, join=True)
    if diverge:
        assert all("diverged" in out[r] for r in range(2))
    else:
        assert out[0] == out[1] and out[0]["equal"] and len(out[0]["param_checksums"]) == 2


def test_stalled_rank_fails_fast_with_a_line_naming_it(capfd):
    """The fail-fast path: 2 ranks over gloo, rank 1 stops
    before its second all-reduce while rank 0 waits inside it. Rank 0's watchdog fires after the
    stall bound, its line names both ranks' phases and rank 1 as the one behind, and the run
    exits non-zero well inside the bound -- the same RankWatch / launcher the GPU bench uses."""
    import time

    t0 = time.monotonic()
    rc = bench.launch(["--gpus", "2", "--backend", "gloo", "--rehearse-stall", "1", "--stall", "4",
                       "--deadline", "60", "--steps", "3"], 2, deadline_s=90)
    elapsed = time.monotonic() - t0
    assert rc != 0
    assert elapsed < 45, elapsed
    lines = capfd.readouterr().out.splitlines()
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["value"] is None and rec["error"] in ("stall", "rank 1 failed")
    assert rec["ranks"] == {"0": "timed 1 all-reduce", "1": "timed 1"}
    assert rec["behind"] == [1]


HANG = """
import time
while True:
    time.sleep(1)
"""


def test_launcher_deadline_kills_a_hung_tree(tmp_path, capfd):
    """Ranks that never finish (and whose own watchdog never fires) are killed as a process group
    at the launcher's deadline; exit code 3 and one error line."""
    import time

    probe = tmp_path / "hang.py"
    probe.write_text(HANG)
    t0 = time.monotonic()
    rc = bench.launch(["--gpus", "2"], 2, script=probe, deadline_s=3)
    assert rc == 3 and time.monotonic() - t0 < 30
    rec = json.loads(capfd.readouterr().out.splitlines()[-1])
    assert rec["error"] == "launcher deadline" and rec["value"] is None


def test_rehearsal_without_a_stall_completes(capfd):
    rc = bench.launch(["--gpus", "2", "--backend", "gloo", "--rehearse-stall", "7", "--stall", "20",
                       "--steps", "3"], 2, deadline_s=90)
    assert rc == 0
    rec = json.loads(capfd.readouterr().out.splitlines()[-1])
    assert rec == {"rehearsal": "no stall", "value": 8.0}


def test_status_of_a_previous_run_is_ignored(tmp_path, monkeypatch):
    """a port-keyed status directory is shared by every run on that port. A rank-1
    record marked failed by an earlier run (another run token) must not fire this run's rank 0."""
    import json as _json

    from oc_cleanrl_amd import watch

    (tmp_path / "rank1.json").write_text(_json.dumps(
        {"rank": 1, "phase": "timed", "n": 5, "t": time.time(), "failed": "stall",
         "run": "an-earlier-run"}))
    monkeypatch.setenv("OCPPO_RUN_ID", "this-run")
    assert watch.run_token() == "this-run"
    assert watch.read_status(tmp_path, run="this-run") == {}
    assert 1 in watch.read_status(tmp_path)  # unfiltered, the stale record is there
    w = watch.RankWatch(0, 2, tmp_path, stall_s=30.0, poll_s=0.05)
    try:
        time.sleep(0.3)  # several polls: a match on the stale record would have fired (os._exit)
        assert set(watch.read_status(tmp_path, run="this-run")) == {0}
    finally:
        w.stop()


def test_kernel_site_byte_counts():
    """The bench's algorithmic bytes per timer site (the line's HBM rooflines): the f32-mask and
    bitmask ReLU-backward passes, and the unmasked (no ReLU) form."""
    R, N = 401408, 64
    assert bench.relu_bias_grad_bytes(f"relu_bias_grad_{R}x{N}") == R * N * 12 + 4 * N
    assert bench.relu_bias_grad_bytes(f"relu_bias_grad_{R}x{N}_norelu") == R * N * 4 + 4 * N
    assert bench.relu_bias_grad_bytes(f"relu_bias_grad_bits_{R}x{N}") == \
        R * N * 8 + R * N // 8 + 4 * N
