"""End-to-end CLI smoke tests of the three entry points on CPU (SURVEY.md §4 level 5; BASELINE.json
config #1 "t5-small summarization fine-tune on CPU, world_size=1" with a tiny random-init T5)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(tmp):
    e = dict(os.environ)
    e.update({"VH_ROOT": str(tmp), "DLLM_FORCE_CPU": "1", "OMP_NUM_THREADS": "2", "PYTHONPATH": ROOT})
    return e


def _json_lines(out):
    res = []
    for line in out.splitlines():
        line = line.strip()
        if line.startswith("{"):
            try:
                res.append(json.loads(line))
            except json.JSONDecodeError:
                pass
    return res


COMMON = ["--synthetic", "32", "--max-source-length", "40", "--max-target-length", "10", "--gen-max-length", "8"]


@pytest.mark.parametrize("model", ["t5-tiny", "mbart-tiny", "pegasus-tiny"])
def test_train_torchrun_single_process(tmp_path, model):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train-torchrun.py"), "--model-ckpt", model,
                        "--output-dir", "out", "--batch-size", "4", "--grad-accum", "2", "--evaluation-steps", "2",
                        "--warmup-steps", "1", *COMMON], env=_env(tmp_path), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    logs = _json_lines(r.stdout)
    assert any("eval_loss" in x for x in logs)
    final = [x for x in logs if "train_samples_per_second" in x]
    assert final and final[-1]["train_loss"] > 0
    out = tmp_path / "outputs" / "out"
    for f in ("config.json", "model.safetensors", "generation_config.json", "model.safetensors.metadata.json"):
        assert (out / f).exists(), f
    md = json.load(open(out / "model.safetensors.metadata.json"))
    assert md["valohai.dataset-versions"][0]["uri"].startswith("dataset://llm-models/")
    assert not any(p.name.endswith(".metadata.json.metadata.json") for p in out.iterdir())


@pytest.mark.slow
def test_train_accelerator_two_ranks(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "train-accelerator.py"), "--model-ckpt",
           "bart-tiny", "--output-dir", "acc", "--batch-size", "2", *COMMON]
    r = subprocess.run(cmd, env=_env(tmp_path), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    logs = _json_lines(r.stdout)
    assert any("rougeLsum" in x for x in logs)
    assert (tmp_path / "outputs" / "acc" / "model.safetensors").exists()


@pytest.mark.slow
def test_train_task_spawn_two_local_ranks(tmp_path):
    cmd = [sys.executable, os.path.join(ROOT, "train-task.py"), "--model-ckpt", "t5-tiny", "--output-dir", "task",
           "--batch-size", "2", "--local-procs", "2", "--master-port", str(_port()), *COMMON]
    r = subprocess.run(cmd, env=_env(tmp_path), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    logs = _json_lines(r.stdout)
    agg = [x for x in logs if "rouge1" in x]
    assert agg and agg[-1]["epoch"] == 0
    assert (tmp_path / "outputs" / "task" / "model.safetensors").exists()


def test_train_task_valohai_distributed_contract(tmp_path):
    """The Valohai distributed shim: master ip / world / rank from /valohai/config/distributed.json."""
    cfgdir = tmp_path / "config"
    cfgdir.mkdir()
    json.dump({"required_count": 4, "me": {"rank": 2, "primary_local_ip": "10.0.0.3"},
               "master": {"primary_local_ip": "10.0.0.1"}}, open(cfgdir / "distributed.json", "w"))
    os.environ["VH_ROOT"] = str(tmp_path)
    try:
        from distributed_llms_example_amd.platform import valohai
        assert valohai.distributed.required_count == 4
        assert valohai.distributed.me().rank == 2
        assert valohai.distributed.master().primary_local_ip == "10.0.0.1"
        (tmp_path / "inputs" / "dataset").mkdir(parents=True)
        (tmp_path / "inputs" / "dataset" / "train.json").write_text("[]")
        assert valohai.inputs("dataset").path().endswith("train.json")
        assert valohai.outputs().path("model-dir").startswith(str(tmp_path / "outputs"))
    finally:
        os.environ.pop("VH_ROOT", None)


def test_fault_injection_then_resume_matches_uninterrupted(tmp_path):
    """a worker killed mid-run (DLLM_FAULT_INJECT) restarts from its last checkpoint with
    --resume-from latest and ends bit-identical to a run that was never interrupted."""
    from safetensors.torch import load_file
    base = [sys.executable, os.path.join(ROOT, "train-torchrun.py"), "--model-ckpt", "t5-tiny", "--batch-size", "4",
            "--grad-accum", "1", "--evaluation-steps", "1000", "--warmup-steps", "1", "--max-steps", "6",
            "--save-steps", "2", *COMMON]
    env = _env(tmp_path)
    r = subprocess.run(base + ["--output-dir", "ref"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    env_f = dict(env, DLLM_FAULT_INJECT="step=5")
    r = subprocess.run(base + ["--output-dir", "ft"], env=env_f, capture_output=True, text=True, timeout=300)
    assert r.returncode == 43, (r.returncode, r.stderr[-3000:])
    assert "injected fault after step 5" in r.stderr
    r = subprocess.run(base + ["--output-dir", "ft", "--resume-from", "latest"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = tmp_path / "outputs"
    a = load_file(str(out / "ref" / "model.safetensors"))
    b = load_file(str(out / "ft" / "model.safetensors"))
    assert a.keys() == b.keys()
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=0, atol=0, msg=k)


@pytest.mark.slow
def test_train_torchrun_context_parallel_two_ranks(tmp_path):
    """train-torchrun with --context-parallel 2: both ranks share each batch, the encoder sequence is split in
    two and attention runs as a ring (parallel/context.py); evaluation and the save run as usual."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "train-torchrun.py"), "--model-ckpt",
           "t5-tiny", "--output-dir", "cp", "--batch-size", "4", "--grad-accum", "1", "--evaluation-steps", "2",
           "--warmup-steps", "1", "--context-parallel", "2", *COMMON]
    r = subprocess.run(cmd, env=_env(tmp_path), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    logs = _json_lines(r.stdout)
    assert any("eval_loss" in x for x in logs)
    final = [x for x in logs if "train_samples_per_second" in x]
    assert final and final[-1]["train_loss"] > 0
    assert (tmp_path / "outputs" / "cp" / "model.safetensors").exists()


def _comm_line(stdout):
    comm = [x["comm"] for x in _json_lines(stdout) if "comm" in x]
    assert comm, stdout[-2000:]
    return comm[0]


@pytest.mark.slow
@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_train_torchrun_four_ranks_match_one_rank(tmp_path, wire):
    """train-torchrun on 4 gloo ranks with the default probed bucket size (--bucket-mb auto) equals one rank running the
    same global batches as gradient-accumulation micro-batches (Trainer batches are dealt round-robin to ranks, the loss
    is normalised by the global token count): same parameters after 3 steps (dropout off).  The first JSON line reports
    the probed bucket choice and a bucket layout every rank agrees on."""
    from safetensors.torch import load_file
    base = [os.path.join(ROOT, "train-torchrun.py"), "--model-ckpt", "t5-tiny", "--max-steps", "3",
            "--evaluation-steps", "1000", "--warmup-steps", "1", "--model-overrides", "dropout_rate=0.0,attention_dropout=0.0",
            "--coalesce-grad-accum", "0", "--grad-reduce-dtype", wire, "--max-eval-samples", "4", *COMMON]
    env = _env(tmp_path)
    r1 = subprocess.run([sys.executable] + base + ["--output-dir", "one", "--batch-size", "2", "--grad-accum", "4"],
                        env=env, capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stderr[-3000:]
    assert _comm_line(r1.stdout)["world_size"] == 1
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(_port())] + base + ["--output-dir", "four", "--batch-size", "2",
                                                                 "--grad-accum", "1"]
    r4 = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r4.returncode == 0, r4.stderr[-3000:]
    comm = _comm_line(r4.stdout)
    assert comm["world_size"] == 4 and comm["bucket_layouts_agree"] is True, comm
    assert isinstance(comm["bucket_choice"], dict) and comm["bucket_choice"]["iters"] >= 10, comm
    assert comm["wire_dtype"] == ("bf16" if wire == "bf16" else "float32"), comm
    a = load_file(str(tmp_path / "outputs" / "one" / "model.safetensors"))
    b = load_file(str(tmp_path / "outputs" / "four" / "model.safetensors"))
    assert a.keys() == b.keys()
    tol = 1e-6 if wire == "fp32" else 2e-5
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=1e-4, atol=tol, msg=k)


@pytest.mark.slow
def test_train_task_four_local_ranks_probe_and_bf16_wire(tmp_path):
    """train-task --local-procs 4 (spawned ranks, gloo) with the default probed buckets and the bf16 wire: it trains,
    evaluates and saves, and its first JSON line reports the probe and an agreed bucket layout."""
    cmd = [sys.executable, os.path.join(ROOT, "train-task.py"), "--model-ckpt", "t5-tiny", "--output-dir", "task4",
           "--batch-size", "2", "--local-procs", "4", "--master-port", str(_port()), "--grad-reduce-dtype", "bf16",
           "--max-eval-samples", "8", *COMMON]
    r = subprocess.run(cmd, env=_env(tmp_path), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    comm = _comm_line(r.stdout)
    assert comm["world_size"] == 4 and comm["bucket_layouts_agree"] is True and comm["wire_dtype"] == "bf16", comm
    assert isinstance(comm["bucket_choice"], dict) and comm["bucket_choice"]["bucket_mb"] > 0, comm
    assert any("rouge1" in x for x in _json_lines(r.stdout))
    assert (tmp_path / "outputs" / "task4" / "model.safetensors").exists()
