"""CPU tests of the auxiliary subsystems: config resolution, metrics JSONL, model summary,
scaling report, launcher flags."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config_precedence(tmp_path):
    from pytorchdistributed_amd.config import Config

    f = tmp_path / "c.yaml"
    f.write_text("bucket_mb: 8\nschedule: gpipe\nmax_epochs: 3\nmy_extra: 1\n")
    env = {"PDA_BUCKET_MB": "16", "PDA_DEBUG_COLLECTIVES": "1", "PDA_SCHEDULE": "1f1b"}
    cfg = Config.load(["--max_epochs", "5", "--first-bucket-mb", "0.5"], file=str(f), env=env)
    assert cfg.max_epochs == 5            # CLI beats file
    assert cfg.bucket_mb == 16.0          # env beats file
    assert cfg.schedule == "1f1b"         # env beats file
    assert cfg.first_bucket_mb == 0.5 and cfg.debug_collectives is True
    assert cfg.extra == {"my_extra": 1}
    assert Config.load([], env={}).bucket_mb == 32.0
    assert cfg.to_env()["PDA_BUCKET_MB"] == "16.0"
    with pytest.raises(ValueError):
        Config.load([], env={"PDA_ALLREDUCE": "bogus"})
    # the reference's own flags parse unchanged
    assert Config.load(["--max_epochs", "2", "--batch_size", "64"], env={}).batch_size == 64


def test_metrics_jsonl_and_summary(tmp_path):
    from pytorchdistributed_amd.utils.metrics import MetricsLogger, bus_bandwidth_gbs, summarize

    for rank, ms in [(0, 10.0), (1, 12.0)]:
        with MetricsLogger(str(tmp_path), rank) as m:
            for step in range(3):
                m.log(step=step, step_ms=ms + step, items_per_s=100.0, loss=torch.tensor(1.5), exposed_comm_ms=0.5)
    s = summarize(str(tmp_path))
    assert s["ranks"] == [0, 1]
    assert s["steps"][2] == {"step": 2, "ranks": 2, "step_ms": 14.0, "items_per_s": 200.0, "exposed_comm_ms": 0.5}
    rec = json.loads((tmp_path / "rank1.jsonl").read_text().splitlines()[0])
    assert rec["loss"] == 1.5 and rec["rank"] == 1
    assert abs(bus_bandwidth_gbs("all_reduce", 10 ** 9, 1.0, 8) - 1.75) < 1e-9
    assert MetricsLogger("", 0).enabled is False


def test_model_summary_matches_reference_totals():
    from pytorchdistributed_amd.models import resnet50
    from pytorchdistributed_amd.utils.summary import summary

    s = summary(resnet50(), (3, 128, 128))
    text = str(s)
    # `03_model_parallel.ipynb` raw lines 301-308: 25,557,032 params, 97.49 MB of params
    assert "Total params: 25,557,032" in text and "Params size (MB): 97.49" in text
    layer2_out = [r for r in s.rows if r.name == "layer2.3.bn3"][0]
    assert layer2_out.out_shape == (1, 512, 16, 16)  # reference table: layer2 -> [-1, 512, 16, 16]
    assert s.rows[-1].out_shape == (1, 1000)


def test_scaling_report(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import scaling_report

    f = tmp_path / "b.jsonl"
    lines = [{"metric": "m", "value": 100.0 * n * (1 if n == 1 else 0.9), "n_gpus": n, "ms_per_step": 10.0,
              "unit": "img/s"} for n in (1, 2, 4, 8)]
    f.write_text("\n".join(json.dumps(x) for x in lines) + "\nnot json\n")
    text = scaling_report.report(scaling_report.load([str(f)]), markdown=True)
    assert "| 8 | 720.0 | 10.00 | 90.0% |" in text


def test_run_cli_flags_reach_workers(tmp_path):
    script = tmp_path / "w.py"
    script.write_text("import os, json, sys\n"
                      "json.dump({k: os.environ.get(k) for k in ('PDA_METRICS_DIR', 'PDA_DEBUG', "
                      "'PDA_COLLECTIVE_TIMEOUT_S', 'RANK', 'WORLD_SIZE')}, open(sys.argv[1] + os.environ['RANK'], 'w'))\n")
    out = str(tmp_path / "env")
    rc = subprocess.run([sys.executable, "-m", "pytorchdistributed_amd.run", "--standalone", "--nproc-per-node", "2",
                         "--metrics-dir", "/tmp/m", "--debug-collectives", "--collective-timeout", "30",
                         str(script), out], cwd=ROOT, timeout=120).returncode
    assert rc == 0
    for r in range(2):
        env = json.load(open(out + str(r)))
        assert env == {"PDA_METRICS_DIR": "/tmp/m", "PDA_DEBUG": "collectives", "PDA_COLLECTIVE_TIMEOUT_S": "30.0",
                       "RANK": str(r), "WORLD_SIZE": "2"}


def test_examples_run_on_cpu(tmp_path):
    """Chapter examples 01 / 02 (both launch flavours) and BASELINE config 1 run end to end on CPU."""
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, "examples/01_data_parallel.py"], cwd=ROOT, env=env, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0 and "Outside: input size [32, 10] output_size [32, 5]" in out.stdout
    out = subprocess.run([sys.executable, "examples/02_ddp_gpus.py", "--max_epochs", "1"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "Batchsize: 32 | Steps: 32" in out.stdout
    out = subprocess.run([sys.executable, "-m", "pytorchdistributed_amd.run", "--standalone", "--nproc-per-node", "2",
                          "examples/02_ddp_gpus_torchrun.py", "--max_epochs", "1"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.count("Steps: 32") == 2
    out = subprocess.run([sys.executable, "-m", "pytorchdistributed_amd.run", "--standalone", "--nproc-per-node", "2",
                          "-m", "pytorchdistributed_amd.bench.mnist_ddp", "--steps", "5", "--warmup", "1",
                          "--backend", "ring"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0
    rec = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["n_ranks"] == 2 and rec["value"] > 0
    out = subprocess.run([sys.executable, "-m", "pytorchdistributed_amd.run", "--standalone", "--nproc-per-node", "2",
                          "examples/04_parameter_server.py", "--epochs", "1"], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "server] epoch 0 | steps 32" in out.stdout and "worker] epoch 0 | steps 32" in out.stdout


def test_merge_rank_traces_and_overlap(tmp_path):
    """tools/merge_traces.py: per-rank rocprofv3 kernel traces -> one Perfetto trace + exposed RCCL time."""
    import importlib.util
    import json as _json

    hdr = "Kind,Queue_Id,Kernel_Name,Start_Timestamp,End_Timestamp\n"
    rows = {0: [("gemm", 0, 100), ("ncclDevKernel_AllReduce", 50, 150), ("bn", 100, 120)],
            1: [("gemm", 10, 110), ("ncclDevKernel_AllReduce", 200, 260)]}
    for r, ks in rows.items():
        d = tmp_path / "prof" / f"rank{r}" / "host"
        d.mkdir(parents=True)
        (d / "trace_kernel_trace.csv").write_text(hdr + "".join(f"KERNEL_DISPATCH,1,{n},{s * 10**6},{e * 10**6}\n" for n, s, e in ks))
    spec = importlib.util.spec_from_file_location("merge_traces", os.path.join(ROOT, "tools", "merge_traces.py"))
    mt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mt)
    out = tmp_path / "merged.json"
    rep = mt.merge(str(tmp_path / "prof"), str(out))
    assert rep[0]["comm_exposed_ms"] == 30 and rep[0]["overlap_ratio"] == 0.7
    assert rep[1]["overlap_ratio"] == 0.0
    ev = _json.loads(out.read_text())["traceEvents"]
    assert {e["pid"] for e in ev} == {0, 1} and min(e["ts"] for e in ev if e["ph"] == "X") == 0
