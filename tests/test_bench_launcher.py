"""bench.py --gpus N launches its own N ranks (no GPU needed here): the
ranks' argv / env, the WORLD_SIZE check, and the launcher's wait / relay /
stop-on-failure behaviour with stand-in rank programs.  The reference's own
harness launches a run per process count the same way
(tests/scalability/run_tests.py:27-30, 185-198)."""
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_commands_argv_and_env():
    cmds = bench.rank_commands(4, ["--gpus", "4", "--steps", "7"], 29511, base_env={"KEEP": "1"})
    assert len(cmds) == 4
    for r, (argv, env) in enumerate(cmds):
        assert argv[0] == sys.executable and argv[-4:] == ["--gpus", "4", "--steps", "7"]
        assert os.path.basename(argv[argv.index("--gpus") - 1]) == "bench.py"
        assert env["RANK"] == str(r) and env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == "4" and env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29511"
        assert env["KEEP"] == "1"


def test_world_check():
    a = bench.parse(["--gpus", "8"])
    assert bench.world_check(a, {}) == "launch"
    assert bench.world_check(a, {"WORLD_SIZE": "8"}) is None
    assert "WORLD_SIZE=2" in bench.world_check(a, {"WORLD_SIZE": "2"})
    one = bench.parse([])
    assert bench.world_check(one, {}) is None
    assert bench.world_check(one, {"WORLD_SIZE": "1"}) is None
    assert bench.world_check(one, {"WORLD_SIZE": "4"}) is not None


def test_launch_relays_rank0_and_succeeds(capfd):
    code = ("import os, json, sys; r = int(os.environ['RANK']); "
            "print(json.dumps({'n_gpus': int(os.environ['WORLD_SIZE']), 'argv': sys.argv[1:]})) if r == 0 else None")
    rc = bench.launch(3, ["--gpus", "3"], child=[sys.executable, "-c", code], poll_s=0.05)
    out = capfd.readouterr().out.strip().splitlines()
    assert rc == 0
    assert out == ['{"n_gpus": 3, "argv": ["--gpus", "3"]}']


def test_launch_stops_the_others_when_a_rank_fails():
    # rank 1 fails at once, the others would block forever (as in a collective)
    code = "import os, sys, time; sys.exit(3) if os.environ['RANK'] == '1' else time.sleep(600)"
    t0 = time.time()
    rc = bench.launch(3, [], child=[sys.executable, "-c", code], poll_s=0.05)
    assert rc == 3
    assert time.time() - t0 < 60


def test_bench_refuses_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "WORLD_SIZE=2" in p.stderr and p.stdout == ""


@pytest.mark.parametrize("n", [2])
def test_launcher_parent_never_imports_torch(n):
    """The parent branch runs before `import torch`: a launched run whose
    ranks are stand-ins leaves torch unimported in the launcher process."""
    code = ("import sys, runpy; sys.argv = ['bench.py', '--gpus', '%d']; import bench; "
            "bench.launch = lambda n, argv, **k: 0; "
            "exec(\"try:\\n bench.main()\\nexcept SystemExit as e:\\n assert e.code == 0, e.code\"); "
            "assert 'torch' not in sys.modules, 'launcher imported torch'; print('ok')" % n)
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env={k: v for k, v in os.environ.items() if k != "WORLD_SIZE"})
    assert p.returncode == 0, p.stderr
    assert p.stdout.strip() == "ok"
