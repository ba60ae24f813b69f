"""bench.py's N-rank launcher: `python bench.py --gpus N`
outside torchrun starts torch.distributed.run as a child with the same
arguments; inside torchrun each rank runs the sharded train."""
from __future__ import annotations

import importlib.util
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_launcher_starts_torchrun_child(monkeypatch):
    b = _bench()
    seen = {}

    def fake_call(cmd, env=None, cwd=None):
        seen["cmd"], seen["env"], seen["cwd"] = cmd, env, cwd
        return 7

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(b.subprocess, "call", fake_call)
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1", "--config", "C2", "--no-cpu"]
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    with pytest.raises(SystemExit) as e:
        b.main()
    assert e.value.code == 7                       # the child's status is ours
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd
    port = [c for c in cmd if c.startswith("--master-port=")]
    assert len(port) == 1 and int(port[0].split("=")[1]) > 0
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv                     # same arguments to every rank
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launcher_not_used_inside_torchrun_or_at_one_gpu(monkeypatch):
    b = _bench()
    calls = []
    monkeypatch.setattr(b.subprocess, "call", lambda *a, **k: calls.append(a) or 0)

    class Stop(Exception):
        pass

    def stop(*a, **k):
        raise Stop()

    # the rank path begins with the synthetic config: stop there
    import pypardis_amd.synth as synth
    monkeypatch.setattr(synth, "CONFIGS", {"C2": None}, raising=True)
    monkeypatch.setattr(b, "cpu_baseline", stop)
    for env, argv in (({"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, ["--gpus", "2"]),
                      ({}, ["--gpus", "1"])):
        monkeypatch.delenv("WORLD_SIZE", raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
        with pytest.raises((Stop, TypeError)):
            b.main()
    assert calls == []


def test_launcher_runs_children_for_real(tmp_path):
    """The real torch.distributed.run child with a stand-in script argument
    list: two ranks start, see WORLD_SIZE=2 and distinct RANKs (CPU only: the
    stand-in never imports the package)."""
    probe = tmp_path / "probe.py"
    probe.write_text("import os, json\n"
                     "print(json.dumps({k: os.environ.get(k) for k in "
                     "('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_ADDR')}), flush=True)\n")
    b = _bench()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={b._free_port()}", str(probe)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert sorted(r["RANK"] for r in rows) == ["0", "1"]
    assert {r["WORLD_SIZE"] for r in rows} == {"2"}
    assert {r["MASTER_ADDR"] for r in rows} == {"127.0.0.1"}


@pytest.mark.gpu
def test_bench_gpus2_rehearse_line():
    """`bench.py --gpus 2 --rehearse` on one GPU: two ranks (gloo, both on
    cuda:0) run the sharded train and rank 0 prints one line with n_gpus 2."""
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse",
           "--points", "2000000", "--no-cpu", "--no-host", "--steps", "2", "--warmup", "1"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
    assert out.returncode == 0, (out.stdout[-2000:], out.stderr[-3000:])
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2
    assert rec["config"]["parallelism"] == "kd-sharded2"
    assert rec["rccl_ranks"] == 0          # gloo rehearsal: no RCCL communicator
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    st = rec["shard_stats"]
    assert st["rank"] in (0, 1) and len(st["rank_seconds"]) == 2


def test_train_roofline_sums_kernels_times_launches():
    """bench.train_roofline: every kernel's per-launch PMC bytes x its
    launches per train, over the step time (the whole train's HBM fraction)."""
    b = _bench()
    pmc = {"_meta": {"trains": 2},
           "count4_kernel": {"hbm_bytes_per_launch": 3.0e9, "dispatches_per_train": 1.0},
           "trampoline_kernel": {"hbm_bytes_per_launch": 2.0e9, "dispatches_per_train": 5.0},
           "no_bytes_kernel": {"SQ_WAVES": 10.0}}
    r = b.train_roofline(pmc, "x.json", 10.0)
    assert r["bytes_per_train"] == 13.0e9
    assert abs(r["achieved_gbs"] - 1300.0) < 1e-6
    assert abs(r["frac"] - 1300.0 / 8000.0) < 1e-12
    assert list(r["top_kernels_bytes"]) == ["trampoline_kernel", "count4_kernel"]
    assert b.train_roofline({"count4_kernel": {"hbm_bytes_per_launch": 1.0}}, "old", 10.0) is None


def test_pmc_summary_counts_launches_per_train(tmp_path, monkeypatch):
    """tools/pmc_summary.py: mean counter value per dispatch (summed over the
    counter's instances) and dispatches per profiled train."""
    import csv
    d = tmp_path / "pmc_1"
    d.mkdir()
    with open(d / "p_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Counter_Name", "Counter_Value",
                                          "Dispatch_Id"])
        w.writeheader()
        for disp in (1, 2, 3, 4):   # two trains x two launches of one kernel
            for inst in range(2):
                w.writerow({"Kernel_Name": "void pd::gather_kernel<float, 3>(float const*)",
                            "Counter_Name": "FETCH_SIZE", "Counter_Value": 5.0,
                            "Dispatch_Id": disp})
    monkeypatch.setenv("PROF_REPS", "2")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(d)],
                         capture_output=True, text=True, env=dict(os.environ), check=True)
    s = json.loads(out.stdout)
    g = s["gather_kernel"]
    assert g["FETCH_SIZE"] == 10.0                 # two instances summed per dispatch
    assert g["dispatches_per_train"] == 2.0
    assert g["hbm_bytes_per_launch"] == 2 * 10.0 * 1024
    assert s["_meta"]["trains"] == 2
