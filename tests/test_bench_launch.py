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


def test_fewer_gpus_than_ranks_is_refused():
    """A rank started where fewer GPUs are visible than WORLD_SIZE exits non-zero before any
    process group is set up (this container has none)."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "visible GPU" in r.stderr and not r.stdout.strip()


def test_c4_forged_indices_land_in_two_shards():
    """configs[3]'s forged variant: at 2, 4 and 8 ranks the forged global indices fall in exactly
    two ranks' shards, two in each; at one rank all four are rank 0's."""
    bench = _bench_module()
    sys.path.insert(0, os.path.join(ROOT, "chaum-pedersen-zkp_amd"))
    from chaum_pedersen.shard import shard_range
    for n_total in (1 << 21, 1 << 26, 1000003):
        f = bench.c4_forged_indices(n_total)
        assert len(set(f)) == 4 and all(0 <= i < n_total for i in f)
        for world in (1, 2, 4, 8):
            per = [sum(1 for i in f if shard_range(n_total, world, r)[0] <= i < shard_range(n_total, world, r)[1])
                   for r in range(world)]
            assert sum(per) == 4
            if world == 1:
                assert per == [4]
            else:
                assert sorted(per, reverse=True) == [2, 2] + [0] * (world - 2)


def test_cpu_threads_capped_at_cgroup_quota(monkeypatch):
    """The CPU baseline runs one thread per core the job can use: the affinity set capped at the
    whole CPUs of the cgroup quota (the GPU box: 256 affinity CPUs, quota 16)."""
    bench = _bench_module()
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    monkeypatch.setattr(bench, "_cgroup_cpu_quota", lambda: 16.0)
    th = bench.cpu_threads(0)
    assert th["threads"] == 16 and th["usable_cpus"] == 16 and th["affinity_cpus"] == 256
    monkeypatch.setattr(bench, "_cgroup_cpu_quota", lambda: None)
    assert bench.cpu_threads(0)["threads"] == 256
    monkeypatch.setattr(bench, "_cgroup_cpu_quota", lambda: 0.5)
    assert bench.cpu_threads(0)["threads"] == 1
    assert bench.cpu_threads(3)["threads"] == 3
