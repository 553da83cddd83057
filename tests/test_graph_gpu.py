"""Whole-step HIP graph (train/graph.py): replayed steps == the same steps run eagerly, dropout masks advance."""
import pytest
import torch

from distributed_llms_example_amd.models import build_model, resolve_config

pytestmark = pytest.mark.gpu


def _setup(seed_model=0):
    from distributed_llms_example_amd.ops.rng import manual_seed
    from distributed_llms_example_amd.parallel.env import init_distributed
    from distributed_llms_example_amd.train.engine import TrainEngine
    env = init_distributed()
    cfg = resolve_config("t5-base").replace(num_layers=2, num_decoder_layers=2, vocab_size=4096)
    torch.manual_seed(seed_model)
    m = build_model(cfg)
    manual_seed(11)
    eng = TrainEngine(m, env, lr=1e-3, dtype=torch.bfloat16)
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


@pytest.mark.parametrize("ga", [1, 2])
def test_graphed_steps_match_eager(ga):
    from distributed_llms_example_amd.ops import rng as rng_mod
    from distributed_llms_example_amd.train.graph import GraphedStep
    cfg, eng_g = _setup()
    steps = 4
    data = _batches(cfg, ga * (steps + 2))
    gs = GraphedStep(eng_g, data[:ga], warmup=2)  # 2 warmup steps on data[:ga]
    losses_g = [float(gs.replay(data[ga * (2 + i):ga * (3 + i)])) for i in range(steps)]
    pg = eng_g.flat.param_buf.float().clone()
    assert int(eng_g.step_seed.t.item()) == eng_g.step_seed.host == ga * (steps + 2)
    eng_g.step_seed.disable()
    rng_mod.default_rng().site_mode = False

    cfg, eng_e = _setup()
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
    pe = eng_e.flat.param_buf.float()
    eng_e.step_seed.disable()
    rng_mod.default_rng().site_mode = False
    assert losses_g == pytest.approx(losses_e, rel=1e-3), (losses_g, losses_e)
    assert ((pg - pe).norm() / pe.norm()).item() < 1e-3


def test_graph_replays_draw_new_dropout_masks():
    """Same batch, two replays: the device step counter advances inside the graph, so the masks (and the loss at the
    replay's forward) differ; with the counter frozen they would repeat."""
    from distributed_llms_example_amd.ops import rng as rng_mod
    from distributed_llms_example_amd.train.graph import GraphedStep
    cfg, eng = _setup()
    eng.optimizer.param_groups[0]["lr"] = 0.0  # no parameter change: only the masks can move the loss
    data = _batches(cfg, 1)
    gs = GraphedStep(eng, data, warmup=1)
    l1 = float(gs.replay(data))
    l2 = float(gs.replay(data))
    eng.step_seed.disable()
    rng_mod.default_rng().site_mode = False
    assert l1 != l2
