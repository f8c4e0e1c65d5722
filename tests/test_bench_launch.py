"""bench.py's N-rank launch (CPU, no GPU touched): `--gpus N` without a launcher starts N ranks as
a child torch.distributed.run on 127.0.0.1; under a launcher, WORLD_SIZE != N is an error."""
import os
import subprocess
import sys

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launcher_argv():
    argv = bench.launcher_argv(8, ["--gpus", "8", "--steps", "3"], 29512)
    assert argv[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in argv and "--nnodes=1" in argv
    assert argv[argv.index("--master-addr") + 1] == "127.0.0.1"
    assert argv[argv.index("--master-port") + 1] == "29512"
    assert argv[-5] == os.path.join(ROOT, "bench.py")
    assert argv[-4:] == ["--gpus", "8", "--steps", "3"]  # children see --gpus 8 = WORLD_SIZE


def test_free_port_is_bindable():
    import socket
    p = bench.free_port()
    with socket.socket() as s:
        s.bind(("127.0.0.1", p))


def test_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 4" in r.stderr
    assert not r.stdout.strip()  # no JSON line from a mis-launched bench


def test_self_launch_runs_n_ranks(tmp_path):
    """launch_ranks starts torch.distributed.run with WORLD_SIZE = N in every child: a stand-in
    script (the launcher argv with the bench swapped for a probe) reports what each rank saw."""
    probe = tmp_path / "probe.py"
    probe.write_text("import os\nprint('rank', os.environ['RANK'], 'of', os.environ['WORLD_SIZE'],"
                     " flush=True)\n")
    code = ("import sys; sys.path.insert(0, %r); import bench; real = bench.launcher_argv; "
            "bench.launcher_argv = lambda n, a, p: real(n, a, p)[:-1 - len(a)] + [%r]; "
            "sys.exit(bench.launch_ranks(2, []))" % (ROOT, str(probe)))
    # the launcher's rendezvous binds a port picked just before (bench.free_port): another
    # process on the host can take it in between, so a failed start is retried once, new port
    for _ in range(2):
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                           timeout=180)
        if r.returncode == 0:
            break
    assert r.returncode == 0, r.stderr[-2000:]
    lines = sorted(l for l in r.stdout.splitlines() if l.startswith("rank"))
    assert lines == ["rank 0 of 2", "rank 1 of 2"]
