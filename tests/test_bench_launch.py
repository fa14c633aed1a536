"""bench.py's --gpus contract on CPU: `bench.py --gpus N` (N > 1) without a launcher starts N
ranks itself through torch.distributed.run in a child process, and a WORLD_SIZE that does not
match --gpus is refused before anything touches torch or the GPU."""
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_module():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=60, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and not r.stdout.strip()


def test_gpus_n_spawns_torchrun_child(monkeypatch):
    bench = _bench_module()
    calls = []

    class Done:
        returncode = 0

    def fake_run(cmd, env=None, **kw):
        calls.append((cmd, env))
        return Done()

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--mode", "rlc", "--steps", "3"])
    rc = None
    try:
        bench.main()
    except SystemExit as e:
        rc = e.code
    assert rc == 0 and len(calls) == 1
    cmd, env = calls[0]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "4"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-6:] == ["--gpus", "4", "--mode", "rlc", "--steps", "3"]
    assert os.path.samefile(cmd[-7], os.path.join(ROOT, "bench.py"))
    assert env.get("HSA_ENABLE_IPC_MODE_LEGACY") == "0"
    # the parent never imported torch (the ranks are the only processes that touch the GPU)
    assert "torch" not in bench.__dict__


def test_child_failure_is_propagated(monkeypatch):
    bench = _bench_module()

    class Failed:
        returncode = -6

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", lambda cmd, env=None, **kw: Failed())
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    try:
        bench.main()
        rc = 0
    except SystemExit as e:
        rc = e.code
    assert rc == 134
