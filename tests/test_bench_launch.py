"""bench.py's launch contract on the CPU (no GPU): ``python bench.py --gpus N`` without a launcher starts
torch.distributed.run as a child before importing torch, a WORLD_SIZE that disagrees with --gpus is
refused, and the ranks' body (timed region, max over ranks, the base JSON line) runs at world 2 on gloo
with a stub step in place of the drop-in call."""
import contextlib
import io
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_launcher_dry_run_names_the_child_command():
    args = ["--gpus", "4", "--steps", "7", "--warmup", "3", "--config", "c2"]
    r = subprocess.run([sys.executable, "-X", "importtime", BENCH] + args + ["--launch-dry-run"], env=_env(),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout.strip().splitlines()[-1])
    cmd = out["launch"]
    assert out["nproc"] == 4
    assert cmd[0] == sys.executable and cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd
    assert any(c.startswith("--master-port=") for c in cmd)
    i = cmd.index(os.path.abspath(BENCH))
    assert cmd[i + 1:] == args + ["--launch-dry-run"], "the child gets the same arguments"
    # the parent never imported torch (nor anything that initialises the GPU) before launching
    imported = [ln.split("|")[-1].strip() for ln in r.stderr.splitlines() if ln.startswith("import time:")]
    assert imported and not any(m == "torch" or m.startswith("torch.") for m in imported)


@pytest.mark.parametrize("ws,gpus", [("1", "2"), ("4", "2"), ("2", "1"), ("x", "2")])
def test_world_size_disagreeing_with_gpus_exits_nonzero(ws, gpus):
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", gpus, "--steps", "2", "--warmup", "0"],
                       env=_env(WORLD_SIZE=ws, RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, (r.returncode, r.stdout, r.stderr)
    assert "WORLD_SIZE" in r.stderr and r.stdout == ""
    assert time.time() - t0 < 60


def test_world_mode_table():
    sys.path.insert(0, REPO)
    import bench

    def mode(gpus, env):
        return bench.world_mode(bench.parse(["--gpus", str(gpus)]), env)
    assert mode(1, {}) == ("run", 1)
    assert mode(8, {}) == ("launch", None)
    assert mode(8, {"WORLD_SIZE": "8"}) == ("run", 8)
    assert mode(2, {"WORLD_SIZE": "1"})[0] == "error"
    assert mode(0, {})[0] == "error"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_body(rank, world, port, out_dir):
    sys.path.insert(0, REPO)
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import bench

    def stub(i):  # rank r's step takes (r + 1) * 20 ms: the max over ranks is rank 1's time
        time.sleep(0.02 * (rank + 1))

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        rc = bench.main(["--gpus", str(world), "--steps", "5", "--warmup", "0"], backend="gloo", stub_step=stub)
    with open(os.path.join(out_dir, f"rank{rank}.txt"), "w") as f:
        f.write(f"{rc}\n{buf.getvalue()}")


def test_main_distributed_branch_world2_gloo(tmp_path):
    world = 2
    mp.spawn(_rank_body, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    lines = {r: open(tmp_path / f"rank{r}.txt").read().splitlines() for r in range(world)}
    assert lines[0][0] == "0" and lines[1][0] == "0"
    assert len(lines[1]) == 1, "only rank 0 prints"
    js = json.loads(lines[0][1])
    assert js["n_gpus"] == 2 and js["rccl_world"] == 2 and js["steps"] == 5 and js["backend"] == "gloo"
    # max over ranks: rank 1's 5 x 40 ms, not rank 0's 5 x 20 ms
    assert js["ms_per_step"] >= 40.0
    assert abs(js["value"] - 2 * 1e3 / js["ms_per_step"]) / js["value"] < 1e-3
    assert js["metric"].startswith("int8 GEMMs/sec") and js["scaling"] == "weak"


_DEADLINE_SCRIPT = r"""
import json, sys, time
sys.path.insert(0, {repo!r})
import bench
result = {{"metric": "m", "value": 1.0}}
def hang():
    time.sleep(60)  # a collective that never completes
def timed_out():
    result["c4_node"] = {{"error": "timed out"}}
    print(json.dumps(result), flush=True)
bench.run_with_deadline(hang, 1.0, timed_out)
print("not reached", flush=True)
"""


def test_node_watchdog_prints_the_line_and_exits():
    """bench.run_with_deadline (the c4_node guard): a step that never returns is cut off after the deadline; the
    timeout hook's JSON line is the process's output and the exit status is 0."""
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", _DEADLINE_SCRIPT.format(repo=REPO)], env=_env(), capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1 and json.loads(lines[0]) == {"metric": "m", "value": 1.0, "c4_node": {"error": "timed out"}}
    assert time.time() - t0 < 30


def test_node_watchdog_passes_results_through():
    import bench
    fired = []
    assert bench.run_with_deadline(lambda: {"ok": 1}, 5.0, lambda: fired.append(1)) == {"ok": 1}
    assert bench.run_with_deadline(lambda: 7, 0, lambda: fired.append(1)) == 7
    time.sleep(0.1)
    assert not fired
