"""Whole-step HIP graphs (train/graph.py): replayed steps == the same steps run eagerly, dropout masks advance, the
learning rate follows param_groups, and the data-parallel schedules ("split": eager bucket all-reduce between two
graphs; "capture": RCCL all-reduces recorded into the graph) on a 1-rank RCCL process group."""
import contextlib

import pytest
import torch
import torch.distributed as dist

from distributed_llms_example_amd.models import build_model, resolve_config

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _no_leaked_step_seeds():
    """Step-seed mode is process-wide (ops/rng.py StepSeed): whatever a test leaves on is switched off afterwards,
    even when its assertions fail, so later dropout tests in the same process run in the default mode."""
    from distributed_llms_example_amd.ops import rng as rng_mod
    yield
    st = rng_mod._active_step[0]
    if st is not None:
        st.disable()
    rng_mod.default_rng().site_mode = False


def _setup(seed_model=0, force_reducer=False, lr=1e-3):
    from distributed_llms_example_amd.ops.rng import manual_seed
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.engine import TrainEngine
    env = init_distributed()
    cfg = resolve_config("t5-base").replace(num_layers=2, num_decoder_layers=2, vocab_size=4096)
    torch.manual_seed(seed_model)
    m = build_model(cfg)
    manual_seed(11)
    eng = TrainEngine(m, env, lr=lr, dtype=torch.bfloat16, force_reducer=force_reducer, bucket_mb=8.0)
    eng.train()
    return cfg, eng


def _batches(cfg, n, B=4, S=256, T=64):
    g = torch.Generator().manual_seed(3)
    out = []
    for _ in range(n):
        out.append({"input_ids": torch.randint(3, cfg.vocab_size, (B, S), generator=g).cuda(),
                    "attention_mask": torch.ones(B, S, dtype=torch.long).cuda(),
                    "labels": torch.randint(3, cfg.vocab_size, (B, T), generator=g).cuda()})
    return out


@contextlib.contextmanager
def _one_rank_rccl():
    """A real RCCL process group of world size 1 (the collectives run; graph capture sees RCCL kernels)."""
    assert not dist.is_initialized()
    store = dist.HashStore()
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        yield
    finally:
        torch.cuda.synchronize()
        dist.destroy_process_group()


def _eager_reference(cfg, data, ga, steps, force_reducer=False):
    """The same steps without graphs (step seeds on, device hyper-parameters), params + per-step losses."""
    cfg, eng_e = _setup(force_reducer=force_reducer)
    eng_e.enable_step_seeds()
    t = torch.zeros((), dtype=torch.float32, device="cuda")
    losses_e = []
    for i in range(steps + 2):
        mbs = data[:ga] if i < 2 else data[ga * i:ga * (i + 1)]
        tot = 0.0
        for k, b in enumerate(mbs):
            tot += float(eng_e.forward_backward(b, grad_accum=ga, sync=k == ga - 1))
        t.add_(1.0)
        eng_e.step(hyper=eng_e.optimizer.device_hyper(t, eng_e.optimizer.param_groups[0]["lr"]))
        if i >= 2:
            losses_e.append(tot / ga)
    # canonical layout: a synchronised eager backward re-lays the flat buffers in gradient-ready order (reducer rebuild)
    pe = eng_e.flat.to_canonical(eng_e.flat.param_buf).float().clone()
    eng_e.disable_step_seeds()
    return losses_e, pe


@pytest.mark.parametrize("ga", [1, 2])
def test_graphed_steps_match_eager(ga):
    from distributed_llms_example_amd.train.graph import GraphedStep
    cfg, eng_g = _setup()
    steps = 4
    data = _batches(cfg, ga * (steps + 2))
    gs = GraphedStep(eng_g, data[:ga], warmup=2)  # 2 warmup steps on data[:ga]
    losses_g = [float(gs.replay(data[ga * (2 + i):ga * (3 + i)])) for i in range(steps)]
    pg = eng_g.flat.to_canonical(eng_g.flat.param_buf).float().clone()
    assert int(eng_g.step_seed.t.item()) == eng_g.step_seed.host == ga * (steps + 2)
    eng_g.disable_step_seeds()

    losses_e, pe = _eager_reference(cfg, data, ga, steps)
    assert losses_g == pytest.approx(losses_e, rel=1e-3), (losses_g, losses_e)
    assert ((pg - pe).norm() / pe.norm()).item() < 1e-3


def test_graph_replays_draw_new_dropout_masks():
    """Same batch, two replays: the device step counter advances inside the graph, so the masks (and the loss at the
    replay's forward) differ; with the counter frozen they would repeat."""
    from distributed_llms_example_amd.train.graph import GraphedStep
    cfg, eng = _setup()
    eng.optimizer.param_groups[0]["lr"] = 0.0  # no parameter change: only the masks can move the loss
    data = _batches(cfg, 1)
    gs = GraphedStep(eng, data, warmup=1)
    l1 = float(gs.replay(data))
    l2 = float(gs.replay(data))
    eng.disable_step_seeds()
    assert l1 != l2


def test_graph_follows_param_group_lr():
    """The captured AdamW reads the learning rate from a device scalar refreshed before every replay: setting
    param_groups[0]['lr'] to 0 after capture must freeze the parameters (it was 1e-3 at capture time)."""
    from distributed_llms_example_amd.train.graph import GraphedStep
    cfg, eng = _setup()
    data = _batches(cfg, 1)
    gs = GraphedStep(eng, data, warmup=1)
    gs.replay(data)
    p0 = eng.flat.param_buf.float().clone()
    eng.optimizer.param_groups[0]["lr"] = 0.0
    gs.replay(data)
    p1 = eng.flat.param_buf.float().clone()
    eng.optimizer.param_groups[0]["lr"] = 1e-3
    gs.replay(data)
    p2 = eng.flat.param_buf.float()
    assert torch.equal(p0, p1)
    assert not torch.equal(p1, p2)


@pytest.mark.parametrize("comm", ["overlap", "split", "capture"])
def test_graphed_data_parallel_step_on_one_rank_rccl(comm):
    """A reducer on a real 1-rank RCCL group: the overlap schedule (backward graph cut at the bucket boundaries, each
    bucket's all-reduce launched between the segment replays), the split schedule (eager bucket all-reduces between
    the forward/backward graph and the optimizer graph) and the captured schedule (RCCL all-reduces inside the graph)
    all give the eager data-parallel step's parameters."""
    from distributed_llms_example_amd.train.graph import GraphedStep
    ga, steps = 2, 3
    with _one_rank_rccl():
        cfg, eng_g = _setup(force_reducer=True)
        assert eng_g.reducer is not None and eng_g.reducer.dp and len(eng_g.reducer.buckets) >= 2
        data = _batches(cfg, ga * (steps + 2))
        gs = GraphedStep(eng_g, data[:ga], warmup=2, comm=comm)
        if comm == "overlap":
            sch = gs.schedule()
            nb = len(eng_g.reducer.buckets)
            assert sch["segments"] >= 2 and sch["buckets_launched_before_backward_end"] >= nb - 1, sch
        losses_g = [float(gs.replay(data[ga * (2 + i):ga * (3 + i)])) for i in range(steps)]
        pg = eng_g.flat.to_canonical(eng_g.flat.param_buf).float().clone()
        eng_g.disable_step_seeds()
        eng_g.reducer.remove()
        losses_e, pe = _eager_reference(cfg, data, ga, steps, force_reducer=True)
    assert losses_g == pytest.approx(losses_e, rel=1e-3), (losses_g, losses_e)
    assert ((pg - pe).norm() / pe.norm()).item() < 1e-3


@pytest.mark.parametrize("tol,keep", [(10.0, True), (-0.99, False)])
def test_step_runner_auto_policy(tol, keep, monkeypatch):
    """DLLM_GRAPH=auto (the entry points' default): eager warm-up steps and the first replays are timed; the graph is
    kept only if its replays are not slower than the eager steps.  Forced both ways through the tolerance, the runner
    must record the decision, keep replaying or fall back to eager steps, and give the same parameters as eager steps
    with the same dropout stream either way."""
    from distributed_llms_example_amd.train.graph import StepRunner
    monkeypatch.setenv("DLLM_GRAPH", "auto")
    monkeypatch.setattr(StepRunner, "GRAPH_TOL", tol)
    steps = 8
    cfg, eng = _setup()
    data = _batches(cfg, steps)
    runner = StepRunner(eng, enabled=True, warmup=2)
    assert runner.policy == "auto"
    for b in data:
        runner([b])
    torch.cuda.synchronize()
    assert runner.decision is not None and runner.decision["graph"] is keep, runner.decision
    assert runner.decision["eager_ms"] > 0 and runner.decision["replay_ms"] > 0
    # capture step + probe replays, then either replays to the end or eager steps
    assert runner.warmup == 1 + StepRunner.PROBE  # auto: PROBE timed eager steps after the untimed first one
    assert runner.replays == (steps - runner.warmup if keep else StepRunner.PROBE)
    p_auto = eng.flat.to_canonical(eng.flat.param_buf).float().clone()
    eng.disable_step_seeds()
    cfg, ref = _setup()
    ref.enable_step_seeds()
    t = torch.zeros((), device="cuda")
    for b in data:
        ref.forward_backward(b)
        t.add_(1.0)
        ref.step(hyper=ref.optimizer.device_hyper(t, ref.optimizer.param_groups[0]["lr"]))
    p_ref = ref.flat.to_canonical(ref.flat.param_buf).float()
    ref.disable_step_seeds()
    assert ((p_auto - p_ref).norm() / p_ref.norm()).item() < 1e-3
