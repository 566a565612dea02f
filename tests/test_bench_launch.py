"""bench.py's own multi-rank launcher (no GPU): `bench.py --gpus N` without
a launcher starts torch.distributed.run as a CHILD process (never exec), the
ranks check that the process group they formed has exactly N ranks, and the
parent relays rank 0's single JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_launcher_command():
    cmd = bench.launcher_cmd(8, ["--gpus", "8", "--steps", "5"], 29555, python="py")
    assert cmd[:3] == ["py", "-m", "torch.distributed.run"]
    assert "--nproc-per-node" in cmd and cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert os.path.basename(cmd[-5]) == "bench.py"


def test_needs_launch_only_without_a_launcher():
    assert bench.needs_launch(2, {})
    assert not bench.needs_launch(2, {"WORLD_SIZE": "2"})
    assert not bench.needs_launch(1, {})


def test_world_size_must_match_gpus():
    bench.check_world(4, 4)
    with pytest.raises(SystemExit):
        bench.check_world(1, 8)


@pytest.mark.parametrize("n", [2, 3])
def test_self_launch_forms_n_ranks_and_prints_one_line(n):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["CF_DIST_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=240,
                       universal_newlines=True)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == n and rec["launched"] is True and rec["backend"] == "gloo"


def test_rank_count_mismatch_fails():
    """Under an external launcher with 2 ranks, --gpus 1 must fail."""
    env = dict(os.environ)
    env["CF_DIST_BACKEND"] = "gloo"
    port = bench.free_port()
    cmd = bench.launcher_cmd(2, ["--gpus", "1", "--dry-run"], port)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, env=env, timeout=240,
                       universal_newlines=True)
    assert r.returncode != 0


def test_epoch_order_charge():
    """bench.py charges only the epoch orders a timed region owes but did not
    compute on its clock (sorted batches)."""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert b.missing_orders(1.0, 2, 200, 95) == pytest.approx(200 / 95 - 2)   # 0.105 owed
    assert b.missing_orders(1.0, 0, 100, 762) == pytest.approx(100 / 762)     # region inside one epoch
    assert b.missing_orders(1.0, 3, 200, 95) == 0.0                           # an extra order: nothing owed
    assert b.missing_orders(0.0, 0, 200, 95) == 0.0                           # sorted batches off
